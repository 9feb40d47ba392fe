"""Times the learner exchange's wire kernels on the C3 batch (run on the GPU
box), for the tape and the combat workloads: the sender's pack, the
learner's unpack into a shadow manager (which includes the shadow's k_obs
over the batch), each alone over 50 messages, wall clock around a device
sync; then C4's dedicated learner on one GPU: 7 peers' unpacks per step over
WIRE_STREAMS streams, against a sender's step + pack (the learner keeps up
when its step is the shorter; c4_scaling_bound = 7 x min(1, sender /
learner))."""
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
    lib.mpenv_wire_error.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    peers = int(os.environ.get("WIRE_PEERS", 7))
    nstreams = int(os.environ.get("WIRE_STREAMS", 4))
    workloads = os.environ.get("WIRE_WORKLOADS", "tape,combat").split(",")
    e = T.Engine(W, ts)
    shadows = [T.Engine(W, ts) for _ in range(peers)]
    hip = e.mem.hip
    n = C.c_int64()
    lib.mpenv_wire_bytes(e.h, 1, C.byref(n))
    buf = e.mem.upload(np.zeros(n.value, np.uint8))
    kbuf = e.mem.upload(np.zeros(n.value, np.uint8))
    ring = e.mem.upload(T.mpenv_tape.tape_ring(1234, 0, A, 64))
    streams = [C.c_void_p() for _ in range(nstreams)]
    hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    for st in streams:
        assert hip.hipStreamCreate(C.byref(st)) == 0
    out = {"peers": peers, "unpack_streams": nstreams}
    for wl in workloads:
        def act(s):
            if wl == "combat":
                e.combat_actions(ring + (s % 64) * A * 24, None, 1)
            else:
                e.copy_actions(ring + (s % 64) * A * 24)

        e.put_ctrl([0, 1, 1])
        e.init()
        for s in range(150):
            act(s)
            e.step()
        # every shadow joins with a keyframe of the current step
        assert lib.mpenv_wire_pack(e.h, kbuf, 1, None) == 0
        hip.hipDeviceSynchronize()
        for x in shadows:
            assert lib.mpenv_wire_unpack(x.h, kbuf, 1, None) == 0
        hip.hipDeviceSynchronize()
        res = {}
        sh = shadows[0]
        assert lib.mpenv_wire_pack(e.h, buf, 0, None) == 0
        hip.hipDeviceSynchronize()
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

        # the dedicated learner of C4 (bench.py --learner-dedicated): per step
        # it unpacks its peers' messages into their shadows, dealt over the
        # unpack streams (LearnerWire(unpack_streams=...)); here the same
        # message for every peer, timed against a simulator's own step + pack,
        # which is what a sender spends per message
        def learner_step(s):
            for j, x in enumerate(shadows):
                lib.mpenv_wire_unpack(x.h, buf, 0, streams[j % nstreams])

        def sim_step(s):
            act(s)
            e.step()
            lib.mpenv_wire_pack(e.h, buf, 0, None)

        for name, fn in (("learner_step_ms", learner_step), ("sender_step_ms", sim_step)):
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
        res["learner_keeps_up"] = res["learner_step_ms"] <= res["sender_step_ms"]
        res["c4_scaling_bound"] = round(peers * min(1.0, res["sender_step_ms"] / res["learner_step_ms"]), 2)
        out[wl] = res
    lib.mpenv_wire_bytes(e.h, 0, C.byref(n))
    out["message_bytes"] = n.value
    out["bytes_per_agent"] = round(n.value / A, 1)
    out["workload"] = ("C3 6v6 x 16384, after 150 steps of each action workload (tape: the bench's action "
                       "tape; combat: the device aim-bot); unpack includes the shadow's k_obs")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
