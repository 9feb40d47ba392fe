"""World sharding across GPUs.

Worlds never interact, so a multi-GPU job is one process per GPU, each owning
a contiguous range of *global* world ids.  The manager is created with
`world_id_offset` = the first global id, which keys every per-world RNG
stream (sim.cpp:743-746 split_i(initKey, episodeIdx, worldID)), so the union
of the shards is bit-identical to one device running all worlds.  The step
itself needs no collective.  The learner exchange (config C4: every rank's
trainInterface outputs to one learner rank, RCCL over xGMI when the process
group is "nccl") is `LearnerGather`: one flat, preallocated, double-buffered
gather per step that overlaps the next step; `gather_to_learner` is the
simple blocking per-tensor form kept for small runs and tests.

Bytes per step into the learner (C4, 6v6 x 16,384 worlds per rank, the 21
trainInterface outputs of mgr.cpp:2383-2431): 3,924 B per agent of
observations + 8 B reward/done + 120 B per world of episode_results =
773.5 MB per rank, 7 x 773.5 MB = 5.4 GB arriving at the learner over its
7 xGMI links (~153 GB/s each, ~1.07 TB/s ingress): >= 5.1 ms per step, about
2.7x a 1.9 ms simulator step, so a single learner rank caps C4 at ~37% of
the simulators' throughput however well the transfer overlaps; the
learner-replica form (`all_gather`, each rank a learner over the whole
batch) has the same per-rank ingress.  Keeping observations where they are
produced (learner data parallelism: each rank trains on its own shard and
all-reduces gradients) moves only the gradients.
"""
from typing import Dict, List, Sequence, Tuple


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


class LearnerGather:
    """Per-step learner exchange of trainInterface outputs, double-buffered.

    Each step, `submit()` copies this rank's outputs (on the current
    stream, after the step that produced them) into one flat byte buffer of
    a 2-slot ring and starts ONE asynchronous gather of that buffer to rank
    `dst`; the collective runs on the process group's own stream, so it
    overlaps the next step, and the engine's output buffers are free for
    that step as soon as the copy is done.  A slot is reused only after its
    previous gather completed (work.wait() orders the current stream after
    it).  Nothing is allocated or concatenated per step.

    On `dst`, `outputs(slot)` returns each output as a zero-copy view of the
    receive buffer with a leading rank axis: [world_size, rows, ...] -- rank
    r holds global worlds [r W, (r + 1) W) (shard_worlds), so flattening the
    first two axes is global world order.

    sources: {name: tensor} (contiguous; same shapes on every rank), e.g.
    SimManager.train_interface()["outputs"] as torch tensors, or
    `from_sim(sim)`.
    """

    # agent_map / unmasked_agent_map (4 KB per agent each) are never written
    # by the simulator: constant zeros the learner already
    # has, so they are not shipped.
    NOT_SHIPPED = ("agent_map", "unmasked_agent_map")

    def __init__(self, sources, dst: int = 0, group=None, slots: int = 2, exclude=NOT_SHIPPED):
        import torch
        import torch.distributed as dist

        if hasattr(sources, "train_interface"):
            sources = self.from_sim(sources)
        sources = {n: t for n, t in sources.items() if n not in exclude}
        self.dist = dist
        self.group = group
        self.dst = dst
        self.rank = dist.get_rank(group)
        self.ws = dist.get_world_size(group)
        self.names = list(sources.keys())
        self.src = [sources[n].contiguous() for n in self.names]
        dev = self.src[0].device
        self.layout = []  # (name, byte offset, nbytes, dtype, shape)
        off = 0
        for n, t in zip(self.names, self.src):
            nb = t.numel() * t.element_size()
            self.layout.append((n, off, nb, t.dtype, tuple(t.shape)))
            off += (nb + 255) // 256 * 256  # 256-B aligned segments
        self.nbytes = off
        self.flat = [torch.empty(off, dtype=torch.uint8, device=dev) for _ in range(slots)]
        self.recv = None
        if self.rank == dst:
            self.recv = [torch.empty((self.ws, off), dtype=torch.uint8, device=dev) for _ in range(slots)]
        self.pending = [None] * slots
        self.k = 0
        self.last_slot = None

    @staticmethod
    def from_sim(sim) -> Dict[str, object]:
        """Every trainInterface output of a madrona_mp_env.SimManager
        (mgr.cpp:2383-2431) as torch tensors (zero-copy views)."""
        outs = sim.train_interface()["outputs"]
        return {n: t.to_torch() for n, t in outs.items()}

    def submit(self, stream_ptr=None):
        import torch

        slot = self.k % len(self.flat)
        self.k += 1
        if self.pending[slot] is not None:
            self.pending[slot].wait()
            self.pending[slot] = None
        buf = self.flat[slot]
        for (n, off, nb, dt, shape), t in zip(self.layout, self.src):
            buf[off:off + nb].copy_(t.view(-1).view(torch.uint8))
        gl = list(self.recv[slot].unbind(0)) if self.recv is not None else None
        self.pending[slot] = self.dist.gather(buf, gl, dst=self.dst, group=self.group, async_op=True)
        self.last_slot = slot
        return slot

    def drain(self):
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None

    def outputs(self, slot=None):
        """{name: [world_size, rows, ...] view} of a completed gather (dst only)."""
        if self.recv is None:
            return {}
        slot = self.last_slot if slot is None else slot
        if self.pending[slot] is not None:
            self.pending[slot].wait()
            self.pending[slot] = None
        r = self.recv[slot]
        out = {}
        for n, off, nb, dt, shape in self.layout:
            out[n] = r[:, off:off + nb].view(dt).view((self.ws,) + shape)
        return out

    def close(self):
        self.drain()

