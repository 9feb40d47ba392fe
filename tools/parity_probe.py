"""Parity probe: runs engine and oracle side by side and reports the first
divergence per export (diagnostic tool, not a test)."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mpenv_testlib as T  # noqa: E402


def first_diff(a, b):
    if a.dtype.kind == "f":
        bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    else:
        bad = a != b
    if not bad.any():
        return None
    idx = tuple(np.argwhere(bad)[0])
    return idx, a[idx], b[idx], int(bad.sum())


def run(team_size, worlds, steps, seed=1234, stop_after=3):
    e = T.Engine(worlds, team_size)
    o = T.Oracle(worlds, team_size)
    ctrl = np.array([0, 1, 1], dtype=np.int32)
    e.put("SIM_CONTROL", ctrl)
    o.view("SIM_CONTROL")[:] = ctrl
    A = worlds * 2 * team_size
    reported = 0
    names = T.STEP_OUTPUTS + T.DEBUG_OUTPUTS
    t0 = time.time()
    for s in range(-1, steps):
        if s < 0:
            e.init()
            o.init()
        else:
            acts = T.mpenv_tape.tape_actions(seed, s, 0, A)
            e.set_actions(acts)
            o.set_actions(acts)
            e.step()
            o.step()
        diffs = []
        for n in names:
            d = first_diff(e.get(n), o.get(n))
            if d is not None:
                diffs.append((n, d))
        if diffs:
            print(f"[{team_size}v{team_size} x{worlds}] step {s}: {len(diffs)} exports differ")
            for n, (idx, av, bv, cnt) in diffs:
                print(f"   {n:40s} n={cnt:7d} first {idx} engine={av!r} oracle={bv!r}")
            reported += 1
            if reported >= stop_after:
                return False
    print(f"[{team_size}v{team_size} x{worlds}] {steps} steps bit-identical ({time.time() - t0:.1f}s)")
    return True


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1:64:300,3:16:300,6:16:300")
    args = ap.parse_args()
    ok = True
    for c in args.configs.split(","):
        t, w, s = (int(x) for x in c.split(":"))
        ok &= run(t, w, s)
    sys.exit(0 if ok else 1)
