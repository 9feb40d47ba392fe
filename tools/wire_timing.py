"""Times the learner exchange's wire kernels on the C3 batch (run on the GPU
box): the sender's pack, the learner's unpack into a shadow manager (which
includes the shadow's k_obs over the batch), each alone over 50 messages of
a combat-regime step, wall clock around a device sync; then C4's dedicated
learner on one GPU: 7 peers' unpacks per step over 4 streams, against a
sender's step + pack (the learner keeps up when its step is the shorter;
c4_scaling_bound = 7 x min(1, sender / learner))."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import mpenv_testlib as T  # noqa: E402


def main():
    ts, W = 6, 16384
    A = W * 2 * ts
    import ctypes as C
    lib = T.lib_mpenv()
    lib.mpenv_wire_bytes.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]
    lib.mpenv_wire_pack.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.mpenv_wire_unpack.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    e, sh = T.Engine(W, ts), T.Engine(W, ts)
    e.put_ctrl([0, 1, 1])
    e.init()
    n = C.c_int64()
    lib.mpenv_wire_bytes(e.h, 1, C.byref(n))
    buf = e.mem.upload(np.zeros(n.value, np.uint8))
    ring = e.mem.upload(T.mpenv_tape.tape_ring(1234, 0, A, 64))
    for s in range(150):
        e.combat_actions(ring + (s % 64) * A * 24, None, 1)
        e.step()
    hip = e.mem.hip
    assert lib.mpenv_wire_pack(e.h, buf, 1, None) == 0
    hip.hipDeviceSynchronize()
    assert lib.mpenv_wire_unpack(sh.h, buf, 1, None) == 0
    hip.hipDeviceSynchronize()
    res = {}
    for name, fn in (("pack_ms", lambda: lib.mpenv_wire_pack(e.h, buf, 0, None)),
                     ("unpack_ms", lambda: lib.mpenv_wire_unpack(sh.h, buf, 0, None))):
        for _ in range(5):
            fn()
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            fn()
        hip.hipDeviceSynchronize()
        res[name] = round((time.perf_counter() - t0) / 50 * 1e3, 4)
    # the dedicated learner of C4 (bench.py --learner-dedicated): per step it
    # unpacks 7 peers' messages into 7 shadows, dealt over 4 unpack streams
    # (LearnerWire(unpack_streams=4)); here the same message 7 times, timed
    # against the simulator's own step (+ its pack), which is what a sender
    # spends per message
    peers = int(os.environ.get("WIRE_PEERS", 7))
    shadows = [sh] + [T.Engine(W, ts) for _ in range(peers - 1)]
    kbuf = e.mem.upload(np.zeros(n.value, np.uint8))
    assert lib.mpenv_wire_pack(e.h, kbuf, 1, None) == 0  # a keyframe of the current step first
    hip.hipDeviceSynchronize()
    for x in shadows[1:]:
        assert lib.mpenv_wire_unpack(x.h, kbuf, 1, None) == 0
    hip.hipDeviceSynchronize()
    lib.mpenv_wire_error.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    nstreams = int(os.environ.get("WIRE_STREAMS", 4))
    streams = [C.c_void_p() for _ in range(nstreams)]
    hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    for st in streams:
        assert hip.hipStreamCreate(C.byref(st)) == 0

    def learner_step():
        for j, x in enumerate(shadows):
            lib.mpenv_wire_unpack(x.h, buf, 0, streams[j % nstreams])

    def sim_step(s):
        e.combat_actions(ring + (s % 64) * A * 24, None, 1)
        e.step()
        lib.mpenv_wire_pack(e.h, buf, 0, None)

    for name, fn in (("learner_step_ms", lambda s: learner_step()), ("sender_step_ms", sim_step)):
        for s in range(5):
            fn(150 + s)
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        for s in range(40):
            fn(155 + s)
        hip.hipDeviceSynchronize()
        res[name] = round((time.perf_counter() - t0) / 40 * 1e3, 4)
    for x in shadows:  # every unpack above was accepted (a refused one is a no-op and times nothing)
        err = C.c_uint32(9)
        assert lib.mpenv_wire_error(x.h, C.byref(err)) == 0 and err.value == 0, err.value
    res["peers"] = peers
    res["learner_keeps_up"] = res["learner_step_ms"] <= res["sender_step_ms"]
    res["c4_scaling_bound"] = round(peers * min(1.0, res["sender_step_ms"] / res["learner_step_ms"]), 2)
    lib.mpenv_wire_bytes(e.h, 0, C.byref(n))
    res["message_bytes"] = n.value
    res["bytes_per_agent"] = round(n.value / A, 1)
    res["workload"] = "C3 6v6 x 16384, after 150 combat steps; unpack includes the shadow's k_obs"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
