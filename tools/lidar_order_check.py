"""Closest-hit lidar under two rules (oracle, CPU): slot order as
mesh_bvh.inl:160-204 is written, and the octant child order the product's
k_lidar follows (DESIGN.md §2 definition 12; or the order-independent
smallest-t rule with LIDAR_B=lex).  Reports
how many rays differ, by how many ulps, and whether any discrete channel
(wall / teammate / opponent one-hot) or any other output differs.

    python tools/lidar_order_check.py [worlds] [steps] [team_size]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mpenv_testlib as T  # noqa: E402


def main(W=64, steps=300, ts=6):
    A = W * 2 * ts
    sims = [T.Oracle(W, ts, lidar_order=o) for o in ("slot", os.environ.get("LIDAR_B", "octant"))]
    for o in sims:
        o.put_ctrl([0, 1, 1])
        o.init()
    rays = diff_rays = disc = other = 0
    max_ulp = 0
    for s in range(steps):
        acts = T.mpenv_tape.tape_actions(1234, s, 0, A)
        for o in sims:
            o.set_actions(acts)
            o.step()
        for name in ("FWD_LIDAR", "REAR_LIDAR"):
            a, b = (o.view(name).reshape(-1, 4) for o in sims)
            rays += len(a)
            d = a[:, 0] != b[:, 0]
            diff_rays += int(d.sum())
            if d.any():
                ua = a[d, 0].view(np.int32).astype(np.int64)
                ub = b[d, 0].view(np.int32).astype(np.int64)
                max_ulp = max(max_ulp, int(np.abs(ua - ub).max()))
            disc += int((a[:, 1:] != b[:, 1:]).any(1).sum())
        for name in ("SELF_OBSERVATION", "OPPONENT_OBSERVATIONS", "REWARD", "HP", "OPPONENT_MASKS"):
            other += int((sims[0].view(name) != sims[1].view(name)).sum())
    print(f"{W} worlds {ts}v{ts}, {steps} steps: {rays} lidar rays, {diff_rays} with a different depth "
          f"({diff_rays / rays:.2e}), max {max_ulp} ulp; discrete channels differing: {disc}; "
          f"other outputs differing: {other}")
    return rays, diff_rays, max_ulp, disc, other


if __name__ == "__main__":
    args = [int(a) for a in sys.argv[1:]]
    main(*args)
