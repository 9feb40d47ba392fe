"""World sharding across GPUs.

Worlds never interact, so a multi-GPU job is one process per GPU, each owning
a contiguous range of *global* world ids.  The manager is created with
`world_id_offset` = the first global id, which keys every per-world RNG
stream (sim.cpp:743-746 split_i(initKey, episodeIdx, worldID)), so the union
of the shards is bit-identical to one device running all worlds.  The step
itself needs no collective; `gather_to_learner` is the optional exchange that
brings observations/rewards to a learner rank (RCCL over xGMI when the
process group is "nccl").
"""
from typing import List, Sequence, Tuple


def shard_worlds(total_worlds: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous split of [0, total_worlds): returns (world_id_offset, count).
    The first `total_worlds % world_size` ranks get one extra world."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world_size {world_size}")
    base, extra = divmod(total_worlds, world_size)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_to_learner(tensors: Sequence, dst: int = 0, group=None) -> List:
    """Gather per-rank step outputs (leading dim = this rank's agents or
    worlds) to `dst`, concatenated in global world order.  Equal shard sizes
    are required (the bench uses total_worlds divisible by world_size).
    Returns the concatenated tensors on `dst` and [] elsewhere."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)
    rank = dist.get_rank(group)
    out = []
    for t in tensors:
        t = t.contiguous()
        bufs = [torch.empty_like(t) for _ in range(ws)] if rank == dst else None
        dist.gather(t, bufs, dst=dst, group=group)
        if rank == dst:
            out.append(torch.cat(bufs, 0))
    return out
