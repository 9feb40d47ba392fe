"""Sphere-cast stuck rate under the two sphereCastLeaf read rules (oracle,
analysis only): the reference's two consecutive triangles per
leaf (mesh_bvh.inl:867-880) vs round 1's triSize triangles.  Prints the
fraction of casts that end at t = 0 and whether the rollouts diverge.

    python tools/cast_stats.py [worlds] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mpenv_testlib as T  # noqa: E402


def run(read_two, W, steps, ts=6):
    lib = T.lib_oracle()
    lib.oracle_cast_stats.argtypes = [C.c_int32, C.POINTER(C.c_uint64)]
    lib.oracle_cast_stats(read_two, None)
    o = T.Oracle(W, ts)
    o.put_ctrl([0, 1, 1])
    o.init()
    digest = []
    for s in range(steps):
        o.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, W * 2 * ts))
        o.step()
        if s % 50 == 49:
            digest.append(o.get("SELF_OBSERVATION").tobytes())
    out = (C.c_uint64 * 2)()
    lib.oracle_cast_stats(-1, out)
    o.close()
    return out[0], out[1], digest


if __name__ == "__main__":
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    res = {}
    for mode, name in ((0, "triSize"), (1, "two consecutive (reference)")):
        casts, zero, dig = run(mode, W, steps)
        res[mode] = dig
        print(f"{name:28s}: {casts} casts, {zero} at t=0 ({100.0 * zero / max(1, casts):.3f}%)")
    same = [a == b for a, b in zip(res[0], res[1])]
    first = same.index(False) * 50 + 49 if False in same else None
    print(f"self obs identical at every 50th step: {all(same)}" + ("" if first is None else f" (first diff by step {first})"))
