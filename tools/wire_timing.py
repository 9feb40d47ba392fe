"""Times the learner exchange's wire kernels on the C3 batch (run on the GPU
box): the sender's pack, the learner's unpack into a shadow manager (which
includes the shadow's k_obs over the batch), each alone over 50 messages of
a combat-regime step, wall clock around a device sync."""
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
    lib.mpenv_wire_bytes(e.h, 0, C.byref(n))
    res["message_bytes"] = n.value
    res["bytes_per_agent"] = round(n.value / A, 1)
    res["workload"] = "C3 6v6 x 16384, after 150 combat steps; unpack includes the shadow's k_obs"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
