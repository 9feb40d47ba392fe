"""Multi-rank world sharding on CPU with gloo, world_size 2.

Each rank steps its shard of worlds (global ids via world_id_offset, action
tape indexed by global agent id) and the step outputs are gathered to rank 0
with mpenv_dist.gather_to_learner; the union must be bit-identical to a
single run over all worlds.  The oracle stands in for the per-rank engine
here (no GPU on CPU runners); the GPU tests check the engine with the same
world_id_offset mechanism.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mpenv_testlib as T
from mpenv_dist import shard_worlds, gather_to_learner

TOTAL_WORLDS, TEAM, STEPS = 6, 2, 60
OUTS = ["SELF_OBSERVATION", "FWD_LIDAR", "REWARD", "DONE", "HP", "MATCH_RESULT"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(sim, first_agent, n_agents):
    sim.put_ctrl([0, 1, 1])
    sim.init()
    for s in range(STEPS):
        sim.set_actions(T.mpenv_tape.tape_actions(1234, s, first_agent, n_agents))
        sim.step()
    return [torch.from_numpy(sim.get(n).copy()) for n in OUTS]


def _worker(rank, world_size, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        off, cnt = shard_worlds(TOTAL_WORLDS, rank, world_size)
        N = 2 * TEAM
        o = T.Oracle(cnt, TEAM, world_id_offset=off)
        outs = _run(o, off * N, cnt * N)
        gathered = gather_to_learner(outs, dst=0)
        if rank == 0:
            np.savez(result_path, *[g.numpy() for g in gathered])
    finally:
        dist.destroy_process_group()


def test_shard_worlds_partition():
    for total in (1, 7, 16384, 131072):
        for ws in (1, 2, 3, 8):
            spans = [shard_worlds(total, r, ws) for r in range(ws)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for off, c in spans:
                assert off == pos
                pos += c
    with pytest.raises(ValueError):
        shard_worlds(8, 2, 2)


def test_two_rank_shards_equal_single_run(tmp_path):
    path = str(tmp_path / "gathered.npz")
    mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    got = np.load(path)
    full = _run(T.Oracle(TOTAL_WORLDS, TEAM), 0, TOTAL_WORLDS * 2 * TEAM)
    for k, name in enumerate(OUTS):
        np.testing.assert_array_equal(got[f"arr_{k}"], full[k].numpy(), err_msg=name)
