"""The learner exchange's compact wire format (csrc/wire.hip).

unpack(pack(x)) on a shadow manager of the sender's configuration must give
every trainInterface output (mgr.cpp:2383-2431) bit for bit: the lidar from
depth + class bit-planes, the observation rows from the shipped state through
the shadow's own k_obs, the last-known rows from the shadow's history
(cleared when a world's episode counter moves, carried once by a keyframe).
Driven at the full C3 batch with the device aim-bot (kills, respawns and
last-known updates) and triggered resets (episode counters move), from the
first step and from a keyframe mid-episode; plus the rejections."""
import ctypes as C
import time

import numpy as np
import pytest

import mpenv_testlib as T

pytestmark = pytest.mark.gpu

RING = 64
SEED = 1234


def _lib():
    lib = T.lib_mpenv()
    lib.mpenv_wire_bytes.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]
    lib.mpenv_wire_pack.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.mpenv_wire_unpack.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.mpenv_wire_error.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    return lib


def _bytes(e, keyframe):
    n = C.c_int64()
    assert e.lib.mpenv_wire_bytes(e.h, int(keyframe), C.byref(n)) == 0
    return n.value


def _error(e):
    v = C.c_uint32(99)
    assert e.lib.mpenv_wire_error(e.h, C.byref(v)) == 0
    return v.value


def _ship(e, sh, buf, keyframe):
    # pack on the sender's stream, unpack on the shadow's: the device sync
    # in between stands in for the transfer's completion
    assert e.lib.mpenv_wire_pack(e.h, buf, int(keyframe), None) == 0
    e.mem.hip.hipDeviceSynchronize()
    assert sh.lib.mpenv_wire_unpack(sh.h, buf, int(keyframe), None) == 0
    e.mem.hip.hipDeviceSynchronize()  # read before anything packs into buf again


def _compare(e, sh, where):
    e.mem.hip.hipDeviceSynchronize()
    for n, ex in T.TRAIN_OUTPUTS.items():
        T.compare(sh.get(ex), e.get(ex), f"{n} (shadow vs sender) @ {where}")


def test_wire_roundtrip_full_batch_combat_and_resets():
    ts, W, steps = 6, 16384, 300
    N = 2 * ts
    A = W * N
    t0 = time.time()
    _lib()
    e = T.Engine(W, ts)
    sh = T.Engine(W, ts)        # the learner's shadow of e, shipped from step 0
    late = T.Engine(W, ts)      # a shadow joining at step 50 with a keyframe
    e.put_ctrl([0, 1, 1])
    e.init()
    nb, nk = _bytes(e, False), _bytes(e, True)
    assert nb < 500 * A and nk > nb
    buf = e.mem.upload(np.zeros(nk, np.uint8))
    ring = e.mem.upload(T.mpenv_tape.tape_ring(SEED, 0, A, RING))
    _ship(e, sh, buf, True)
    assert _error(sh) == 0
    _compare(e, sh, "init")
    e.enable_stats(True)
    rng = np.random.default_rng(3)
    for s in range(steps):
        if s in (30, 200):  # episode counters move: the shadow must clear last-known rows
            for w in rng.choice(W, 64, replace=False):
                e.trigger_reset(int(w))
        e.combat_actions(ring + (s % RING) * A * 24, None, 1)
        e.step()
        _ship(e, sh, buf, False)
        if s == 150:
            _ship(e, late, buf, True)  # keyframe: last-known rows included
        elif s > 150:
            assert late.lib.mpenv_wire_unpack(late.h, buf, 0, None) == 0
        e.mem.hip.hipDeviceSynchronize()  # unpacks done before the next pack overwrites buf
        if s % 25 == 24 or s == steps - 1:
            _compare(e, sh, f"step {s}")
            if s > 150:
                _compare(e, late, f"step {s} (keyframe at 150)")
            print(f"  step {s}: shadows equal, test {time.time() - t0:.0f} s", flush=True)
    assert _error(sh) == 0 and _error(late) == 0
    st = e.read_stats()
    assert st["kills"] > 0
    lk = e.get("OPPONENT_LAST_KNOWN_OBSERVATIONS")
    assert (lk != 0).any()
    print(f"\nwire: {nb / A:.1f} B per agent ({nb / 1e6:.1f} MB per C3 message, keyframe {nk / 1e6:.1f} MB) "
          f"against {sum(e.get(x).nbytes for x in T.TRAIN_OUTPUTS.values()) / A:.1f} B exported; "
          f"{steps} combat steps, {st['kills']} kills, {st['lk_rows']} last-known rows written, resets at 30 "
          f"and 200, keyframe shadow from 150; test {time.time() - t0:.1f} s")
    e.mem.free(buf)
    e.mem.free(ring)


def test_wire_rejects_foreign_or_mismatched_messages():
    """Refused messages (another configuration, another shard's world offset,
    the other kind) raise REFUSED | DESYNC; the shadow then refuses plain
    messages (its history is behind) and skips its observation rows until a
    keyframe resynchronises it (a silently drifting shadow)."""
    REF, DES = 1, 2
    _lib()
    a = T.Engine(64, 3)
    b = T.Engine(32, 3)
    c = T.Engine(64, 3, world_id_offset=64)  # the same configuration, another shard
    for x in (a, b, c):
        x.put_ctrl([0, 1, 1])
        x.init()
    buf = a.mem.upload(np.zeros(_bytes(a, True), np.uint8))
    kbuf = a.mem.upload(np.zeros(_bytes(a, True), np.uint8))
    assert a.lib.mpenv_wire_pack(a.h, buf, 0, None) == 0
    assert a.lib.mpenv_wire_pack(a.h, kbuf, 1, None) == 0
    a.mem.hip.hipDeviceSynchronize()
    # another configuration
    assert b.lib.mpenv_wire_unpack(b.h, buf, 0, None) == 0
    assert _error(b) == REF | DES
    # another shard (header world offset 0, shadow offset 64)
    assert c.lib.mpenv_wire_unpack(c.h, buf, 0, None) == 0
    assert _error(c) == REF | DES
    # a plain message unpacked as a keyframe
    assert a.lib.mpenv_wire_unpack(a.h, buf, 1, None) == 0
    assert _error(a) == REF | DES
    # out of sync: the right kind is still refused
    a.step()  # the engine's own step writes its rows (no gate on the step path)
    stepped = a.get("OPPONENT_OBSERVATIONS").copy()
    assert a.lib.mpenv_wire_pack(a.h, buf, 0, None) == 0
    a.mem.hip.hipDeviceSynchronize()
    assert a.lib.mpenv_wire_unpack(a.h, buf, 0, None) == 0
    assert _error(a) == REF | DES
    assert _error(a) == DES  # the read cleared REFUSED only
    # a keyframe resynchronises; plain messages are accepted again
    assert a.lib.mpenv_wire_unpack(a.h, kbuf, 1, None) == 0
    assert _error(a) == 0
    assert a.lib.mpenv_wire_unpack(a.h, buf, 0, None) == 0
    assert _error(a) == 0
    T.compare(a.get("OPPONENT_OBSERVATIONS"), stepped, "rows rebuilt after the resync")
    a.mem.free(buf)
    a.mem.free(kbuf)


def test_learner_wire_raises_on_a_refused_message_then_recovers_at_a_keyframe():
    """LearnerWire (loopback through the Python module) must not serve a
    shadow that refused a message: a message whose header carries the pack
    kernel's overflow flag is refused, and outputs() raises (the periodic
    asynchronous check too).  The periodic keyframe (keyframe_every) then
    resynchronises the shadow: after it the outputs equal the engine's again
    (a refused message must not freeze a shadow for good)."""
    import socket

    import torch
    import torch.distributed as dist
    import madrona_mp_env as m
    from mpenv_dist import LearnerWire

    ts, W = 3, 64
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        def mk():
            return m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                                auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                                team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE)

        sim = mk()
        sim.init()
        corrupt = [False]
        lw = None

        def pack(ptr, kf, st):
            sim.wire_pack(ptr, kf, st)
            if corrupt[0]:  # the header's flags word (offset 8): kWireOverflow
                t = [b for slot in lw.bufs for b in slot if b.data_ptr() == ptr][0]
                t[8] = t[8] | 2

        from mpenv_dist import LearnerGather

        st = torch.cuda.Stream()
        torch.cuda.set_stream(st)
        lw = LearnerWire(sim, make_shadow=lambda r: mk(), pack=pack, device=torch.device("cuda", 0),
                         keyframe_every=8, check_every=2)
        assert lw._err_async
        for s in range(4):
            sim.step_async(st.cuda_stream)
            lw.submit(st.cuda_stream)
        lw.outputs()  # in sync
        corrupt[0] = True
        sim.step_async(st.cuda_stream)
        lw.submit(st.cuda_stream)  # message 4: refused
        corrupt[0] = False
        with pytest.raises(RuntimeError, match="refused"):
            lw.outputs()
        def step():
            sim.step_async(st.cuda_stream)
            lw.submit(st.cuda_stream)

        step()  # message 5: refused (out of sync); the periodic check (k = 6) queues its read
        step()  # message 6: refused
        with pytest.raises(RuntimeError, match="refused"):
            step()  # message 7: the check (k = 8) raises on what the k = 6 read fetched
        step()  # message 8: a keyframe resynchronises
        step()  # message 9: accepted; the check (k = 10) queues a read (messages 6-7's refusals)
        step()  # message 10
        with pytest.raises(RuntimeError, match="refused"):
            lw.check()  # those refusals, reported once
        got = lw.outputs()  # clean again
        own = LearnerGather.from_sim(sim)
        torch.cuda.synchronize()
        for n, t in got.items():
            a, b = t[0].contiguous(), own[n].contiguous()
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)), n
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_learner_wire_loopback_matches_the_engine(overlap):
    """LearnerWire at one rank (bench.py --exchange wire): the rank's own
    message packed on the step stream and unpacked into its shadow every
    step through the Python module, on the learner's own unpack stream
    ordered by GPU events (overlap) or on the step stream -- the shadow's
    trainInterface outputs (outputs()) equal the engine's bit for bit, with
    combat actions driving kills and last-known rows."""
    import socket

    import torch
    import torch.distributed as dist
    import madrona_mp_env as m
    from mpenv_dist import LearnerGather, LearnerWire

    ts, W, steps = 6, 512, 60
    A = W * 2 * ts
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        def mk():
            return m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                                auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                                team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE)

        sim = mk()
        ctrl = sim.sim_control_tensor().to_torch()
        ctrl.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device=ctrl.device).view_as(ctrl))
        torch.cuda.synchronize()
        sim.init()
        lw = LearnerWire(sim, make_shadow=lambda r: mk(), device=torch.device("cuda", 0), overlap=overlap)
        assert (lw.ustream is not None) == overlap
        ring = torch.from_numpy(T.mpenv_tape.tape_ring(SEED, 0, A, RING)).to("cuda")
        torch.cuda.synchronize()
        st = torch.cuda.Stream()
        torch.cuda.set_stream(st)
        sptr = st.cuda_stream
        assert sptr != 0
        with pytest.raises(ValueError):
            lw.submit(0)  # loopback needs the step's stream
        for s in range(steps):
            sim.combat_actions(ring[s % RING].data_ptr(), 0, 1, sptr)
            sim.step_async(sptr)
            lw.submit(sptr)
            if s % 20 == 19:
                got = lw.outputs()
                own = LearnerGather.from_sim(sim)
                torch.cuda.synchronize()
                for n, t in got.items():
                    a, b = t[0].contiguous(), own[n].contiguous()
                    assert a.shape == b.shape and torch.equal(a.view(torch.uint8), b.view(torch.uint8)), (n, s)
        lw.close()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())
        dist.destroy_process_group()
