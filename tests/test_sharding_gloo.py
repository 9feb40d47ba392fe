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
from mpenv_dist import LearnerGather, shard_worlds, gather_to_learner

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


TRAIN_OUTPUTS = T.TRAIN_OUTPUTS
LG_STEPS = 40


def _lg_worker(rank, world_size, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        off, cnt = shard_worlds(TOTAL_WORLDS, rank, world_size)
        N = 2 * TEAM
        o = T.Oracle(cnt, TEAM, world_id_offset=off)
        o.put_ctrl([0, 1, 1])
        o.init()
        # zero-copy views of the rank's live outputs, as train_interface() hands out
        src = {n: torch.from_numpy(o.view(e)) for n, e in TRAIN_OUTPUTS.items()}
        lg = LearnerGather(src, dst=0)
        slots = {}
        for s in range(LG_STEPS):
            o.set_actions(T.mpenv_tape.tape_actions(1234, s, off * N, cnt * N))
            o.step()
            slots[s] = lg.submit()
        lg.drain()
        if rank == 0:
            out = {}
            for s in (LG_STEPS - 2, LG_STEPS - 1):  # both ring slots hold a completed step
                for n, t in lg.outputs(slots[s]).items():
                    out[f"{s}:{n}"] = t.reshape((-1,) + tuple(t.shape[2:])).numpy().copy()
            np.savez(result_path, **out)
        lg.close()
    finally:
        dist.destroy_process_group()


def test_learner_gather_ships_every_train_output_in_global_order(tmp_path):
    """LearnerGather (C4's learner exchange): every trainInterface output of
    both ranks lands on rank 0 in one flat double-buffered gather per step;
    the two ring slots hold the last two steps, and flattening the rank axis
    gives the single-run tensors in global world order."""
    path = str(tmp_path / "lg.npz")
    mp.spawn(_lg_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    got = np.load(path)
    o = T.Oracle(TOTAL_WORLDS, TEAM)
    o.put_ctrl([0, 1, 1])
    o.init()
    A = TOTAL_WORLDS * 2 * TEAM
    for s in range(LG_STEPS):
        o.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, A))
        o.step()
        if s >= LG_STEPS - 2:
            for n, e in TRAIN_OUTPUTS.items():
                np.testing.assert_array_equal(got[f"{s}:{n}"], o.get(e), err_msg=f"{n} @ {s}")
    assert len(TRAIN_OUTPUTS) == 19  # 21 outputs minus the two never-written agent maps


def _local_worker(rank, world_size, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from mpenv_dist import make_exchange

        off, cnt = shard_worlds(TOTAL_WORLDS, rank, world_size)
        N = 2 * TEAM
        o = T.Oracle(cnt, TEAM, world_id_offset=off)
        o.put_ctrl([0, 1, 1])
        o.init()
        src = {n: torch.from_numpy(o.view(e)) for n, e in TRAIN_OUTPUTS.items()}
        ex = make_exchange("local", src, grad_bytes=4096, update_every=10)
        ex.grad.fill_(float(rank + 1))
        for s in range(LG_STEPS):
            o.set_actions(T.mpenv_tape.tape_actions(1234, s, off * N, cnt * N))
            o.step()
            ex.submit()
        ex.drain()
        outs = ex.outputs()
        np.savez(result_path + f".{rank}.npz", grad=ex.grad.numpy(), updates=ex.updates,
                 bytes=ex.bytes_per_step()["sent_per_rank"],
                 **{n: t[0].numpy().copy() for n, t in outs.items()})
        ex.close()
    finally:
        dist.destroy_process_group()


def test_learner_local_exchange_keeps_shards_and_allreduces_gradients(tmp_path):
    """LearnerLocal (the data-parallel learner layout, bench.py --exchange
    local): each rank's outputs stay its own shard's (equal to the single
    run's rows of those worlds), and every `update_every` steps one
    all-reduce of the gradient-sized buffer runs (sum over ranks)."""
    path = str(tmp_path / "loc")
    mp.spawn(_local_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    o = T.Oracle(TOTAL_WORLDS, TEAM)
    o.put_ctrl([0, 1, 1])
    o.init()
    A = TOTAL_WORLDS * 2 * TEAM
    for s in range(LG_STEPS):
        o.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, A))
        o.step()
    for rank in range(2):
        got = np.load(path + f".{rank}.npz")
        off, cnt = shard_worlds(TOTAL_WORLDS, rank, 2)
        assert int(got["updates"]) == LG_STEPS // 10
        # ranks start at 1 and 2: the first all-reduce gives 3, each later one doubles it
        np.testing.assert_array_equal(got["grad"], np.full(1024, 3.0 * 2 ** (LG_STEPS // 10 - 1), np.float32))
        assert float(got["bytes"]) == 2 * 1 * 4096 / 2 / 10
        for n, e in TRAIN_OUTPUTS.items():
            full = o.get(e)
            rpw = full.shape[0] // TOTAL_WORLDS
            np.testing.assert_array_equal(got[n], full[off * rpw:(off + cnt) * rpw], err_msg=n)


def _uneven_worker(rank, world_size, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        off, cnt = shard_worlds(5, rank, world_size)  # 3 + 2 worlds
        o = T.Oracle(cnt, TEAM, world_id_offset=off)
        src = {n: torch.from_numpy(o.view(e)) for n, e in TRAIN_OUTPUTS.items()}
        try:
            LearnerGather(src, dst=0)
            msg = "no error"
        except ValueError as ex:
            msg = str(ex)
        open(result_path + f".{rank}", "w").write(msg)
    finally:
        dist.destroy_process_group()


def test_learner_gather_rejects_unequal_shards(tmp_path):
    """An uneven split (5 worlds on 2 ranks) would make RCCL's gather truncate
    or overrun silently: LearnerGather checks every rank's layout up front."""
    path = str(tmp_path / "uneven")
    mp.spawn(_uneven_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    for rank in range(2):
        assert "different layout" in open(path + f".{rank}").read()


def test_learner_gather_rejects_non_contiguous_sources():
    """A strided source would be snapshotted by .contiguous(); LearnerGather
    refuses it instead (the live engine buffer is what must ship)."""
    t = torch.zeros(8, 4)[:, :2]
    with pytest.raises(ValueError, match="contiguous"):
        LearnerGather.__init__(object.__new__(LearnerGather), {"x": t})


# ---- LearnerWire transport (the compact wire format's exchange): byte-level
# stand-ins for pack / unpack, three ranks on gloo.  Every message of every
# sender must reach the learner's unpack in order, the first and then every
# WIRE_KF-th as a keyframe (periodic keyframes, so a shadow that
# refused a message recovers), each sized as its kind, with its bytes intact.
WIRE_NB, WIRE_NK, WIRE_STEPS, WIRE_KF = 1000, 1600, 7, 3


def _wire_bytes(rank, step, keyframe):
    n = WIRE_NK if keyframe else WIRE_NB
    return (np.arange(n, dtype=np.int64) * 7 + rank * 131 + step * 17 + (5 if keyframe else 0)).astype(np.uint8)


def _wire_worker(rank, world_size, port, result_path, dedicated=False):
    import ctypes as C

    from mpenv_dist import LearnerWire

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        step = [0]
        seen = []

        def pack(ptr, keyframe, stream):
            b = _wire_bytes(rank, step[0], keyframe)
            C.memmove(ptr, b.ctypes.data, len(b))

        def unpack(r, ptr, keyframe, stream):
            n = WIRE_NK if keyframe else WIRE_NB
            seen.append((r, bool(keyframe), bytes((C.c_uint8 * n).from_address(ptr))))

        if dedicated and rank == 0:
            def pack(ptr, keyframe, stream):  # the dedicated learner never packs
                raise AssertionError("dedicated learner packed a message")
        lw = LearnerWire(None, dst=0, pack=pack, unpack=unpack, dedicated=dedicated,
                         nbytes=lambda kf: WIRE_NK if kf else WIRE_NB, device=torch.device("cpu"),
                         keyframe_every=WIRE_KF)
        assert lw.bytes_per_step() == {"sent_per_rank": WIRE_NB, "learner_ingress": WIRE_NB * (world_size - 1),
                                       "keyframe": WIRE_NK}
        for s in range(WIRE_STEPS):
            step[0] = s
            lw.submit()
        lw.drain()
        if rank == 0:
            import pickle  # our own file, written and read by this test only

            with open(result_path, "wb") as f:
                pickle.dump(seen, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dedicated", [False, True], ids=["learner_simulates", "dedicated_learner"])
def test_learner_wire_transport_three_ranks(tmp_path, dedicated):
    """Three gloo ranks; rank 0 the learner.  dedicated: the learner
    simulates nothing (sim None, never packs) and only receives and unpacks
    ranks 1 and 2 -- C4's 7 simulators + 1 learner layout;
    every message still arrives in order, keyframes first and every
    WIRE_KF-th, bytes intact."""
    import pickle  # reads the file _wire_worker wrote above

    path = str(tmp_path / "wire.pkl")
    mp.spawn(_wire_worker, args=(3, _free_port(), path, dedicated), nprocs=3, join=True)
    with open(path, "rb") as f:
        seen = pickle.load(f)
    for r in (1, 2):
        msgs = [(kf, b) for rr, kf, b in seen if rr == r]
        assert len(msgs) == WIRE_STEPS
        for s, (kf, b) in enumerate(msgs):
            assert kf == (s % WIRE_KF == 0)
            assert b == _wire_bytes(r, s, kf).tobytes(), (r, s)


def test_learner_wire_check_raises_when_a_shadow_refused_a_message():
    """a shadow that refused a message (overflow, wrong kind,
    another configuration or shard) is out of sync until a keyframe;
    LearnerWire raises on its next check (every `check_every` submits, and in
    outputs() / close()) instead of serving stale rows.  Byte-level stand-ins,
    one gloo rank (loopback)."""
    from mpenv_dist import LearnerWire

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        err = {0: 0}
        lw = LearnerWire(None, make_shadow=lambda r: object(), pack=lambda p, k, s: None,
                         unpack=lambda r, p, k, s: None, nbytes=lambda kf: 64, device=torch.device("cpu"),
                         check_every=3, wire_error=lambda r: err[r])
        for _ in range(3):
            lw.submit(1)  # the third submit checks: clean
        lw.check()
        err[0] = 3  # refused | out of sync
        lw.submit(1)
        lw.submit(1)
        with pytest.raises(RuntimeError, match="refused"):
            lw.submit(1)  # sixth submit: checked
        with pytest.raises(RuntimeError, match="refused"):
            lw.close()
    finally:
        dist.destroy_process_group()
