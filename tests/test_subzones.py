"""SubZones sim flag in the oracle: sub-zone membership
and control (subzoneSystem, sim.cpp:1978-2041), spawn-time membership
(utils.cpp:906-926) and the sub-zone reward (sim.cpp:3734-3847).  The GPU
engine is compared with the oracle on the same case in
tests/test_parity_gpu.py and the 3v3_subzones golden fixture.
"""
import numpy as np

import mpenv_testlib as T
from golden.make_golden import CASES, rollout

STAND_HALF = np.float32(65.0 / 2.0)
# level_gen.cpp:297-326 (the axis-aligned sub-zones 2..7)
BOXES = {2: ((-950, -500, 0), (-50, 500, 1000)), 3: ((50, -500, 0), (950, 500, 1000)),
         4: ((-1000, -1650, 0), (-50, -600, 1000)), 5: ((50, -1650, 0), (1000, -600, 1000)),
         6: ((-1000, 600, 0), (-50, 1650, 1000)), 7: ((1000, 600, 0), (50, 1650, 1000))}


def test_subzone_membership_and_control():
    case = CASES["3v3_subzones"]
    W, ts = case["worlds"], case["team_size"]
    N = 2 * ts
    o = T.Oracle(W, ts, sim_flags=case["sim_flags"])
    seen_in = seen_ctrl = 0
    for s in rollout(o, case):
        if s < 0:
            continue
        pol = np.clip(o.get("AGENT_POLICY").ravel(), 0, 7).reshape(W, N)
        ai = o.get("DEBUG_AGENT_I32").reshape(W, N, -1)
        af = o.get("DEBUG_AGENT_F32").reshape(W, N, -1)
        wi = o.get("DEBUG_WORLD_I32").reshape(W, -1)
        for w in range(W):
            if wi[w, 1] == 0:  # reset this step: positions moved after the system ran
                continue
            inside = (ai[w, :, 9] >> 5) & 1
            st = int(wi[w, 21]) & 0xFFFFFFFF
            for k in range(8):
                members = np.where(pol[w] == k)[0]
                na = sum(1 for i in members if inside[i] and i // ts == 0)
                nb = sum(1 for i in members if inside[i] and i // ts == 1)
                ctrl = ((st >> (4 * k)) & 3) - 1
                contested = (st >> (4 * k + 2)) & 1
                assert contested == int(na > 0 and nb > 0)
                if contested or (na == 0 and nb == 0):
                    assert ctrl == -1
                else:
                    assert ctrl == (0 if na else 1)
                    seen_ctrl += 1
                if k in BOXES:
                    lo, hi = np.array(BOXES[k], np.float32)
                    for i in members:
                        p = af[w, i, 0:3].copy()
                        p[2] = np.float32(p[2] + STAND_HALF)
                        geo = bool(np.all(lo <= p) and np.all(p <= hi))
                        assert geo == bool(inside[i]), (s, w, i, k, p)
                        if inside[i]:
                            assert af[w, i, 23] == 0.0
                            seen_in += 1
            assert not any((inside[i] for i in np.where(pol[w] == 7)[0])), "sub-zone 7 is empty (inverted box)"
    assert seen_in > 0 and seen_ctrl > 0
    o.close()
