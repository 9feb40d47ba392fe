"""The learner exchanges (mpenv_dist) on the GPU over RCCL.

The one-GPU box cannot run a multi-GPU collective, so this runs a one-rank
"nccl" (RCCL) process group: every collective is a real RCCL launch on the
engine's device buffers, ordered against the steps on the same stream --
which is what the exchanges add on top of the gloo-tested layout logic.

* LearnerGather: each step's outputs are packed into a ring slot and
  gathered asynchronously while the next step runs; a slot read after the
  following step still holds its own step's outputs (the ring, not the live
  engine buffers, is what ships), equal to snapshots taken at that step.
* LearnerLocal: the gradient-sized all-reduce runs every update_every steps
  and leaves the (one-rank) sum.
"""
import os
import socket

import pytest

import mpenv_testlib as T

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_learner_exchanges_on_rccl_one_rank():
    import torch
    import torch.distributed as dist

    import madrona_mp_env as m
    from mpenv_dist import LearnerGather, make_exchange

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        W, ts = 512, 6
        A = W * 2 * ts
        sim = m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                           auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                           team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE)
        ctrl = sim.sim_control_tensor().to_torch()
        ctrl.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device="cuda").view_as(ctrl))
        torch.cuda.synchronize()
        sim.init()
        ring = torch.from_numpy(T.mpenv_tape.tape_ring(1234, 0, A, 16)).cuda()
        stream = torch.cuda.current_stream()
        lg = LearnerGather(sim, dst=0)
        live = LearnerGather.from_sim(sim)
        snaps, slots = {}, {}
        for s in range(12):
            sim.copy_actions(ring[s % 16].data_ptr(), stream.cuda_stream)
            sim.step_async(stream.cuda_stream)
            slots[s] = lg.submit()
            if s >= 10:
                snaps[s] = {n: t.clone() for n, t in live.items() if n not in lg.NOT_SHIPPED}
        # step 10's slot, read after step 11 was stepped and submitted
        for s in (10, 11):
            outs = lg.outputs(slots[s])
            torch.cuda.synchronize()
            assert set(outs) == set(snaps[s])
            for n, t in outs.items():
                assert t.shape[0] == 1
                assert torch.equal(t[0], snaps[s][n]), (s, n)
        # consecutive steps differ somewhere, so the check above is not vacuous
        assert not torch.equal(snaps[10]["self"], snaps[11]["self"])
        lg.close()

        ex = make_exchange("local", sim, grad_bytes=1 << 20, update_every=5)
        ex.grad.fill_(2.0)
        for s in range(12, 22):
            sim.copy_actions(ring[s % 16].data_ptr(), stream.cuda_stream)
            sim.step_async(stream.cuda_stream)
            ex.submit()
        ex.drain()
        torch.cuda.synchronize()
        assert ex.updates == 2
        assert bool((ex.grad == 2.0).all())  # one rank: the sum is the buffer itself
        outs = ex.outputs()
        assert torch.equal(outs["self"][0], live["self"])  # the engine's own buffers, zero-copy
        ex.close()
    finally:
        dist.destroy_process_group()
