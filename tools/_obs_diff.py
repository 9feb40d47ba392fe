# development probe: where the float-mask k_obs variant differs from the oracle at init
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import mpenv_testlib as T
from golden.make_golden import make_sim, CASES
case = CASES["2v2_navmesh_curriculum"]
from golden.make_golden import rollout
e = make_sim(T.Engine, case)
o = make_sim(T.Oracle, case)
next(rollout(e, case)); next(rollout(o, case))
for n in ("OPPONENT_OBSERVATIONS", "OPPONENT_LAST_KNOWN_OBSERVATIONS", "OPPONENT_MASKS", "SELF_OBSERVATION"):
    a, b = e.get(n), o.get(n)
    d = np.argwhere(a != b)
    print(n, a.shape, "diffs", len(d), d[:8].tolist())
    for idx in d[:4]:
        print("   ", tuple(idx), a[tuple(idx)], b[tuple(idx)])
m = o.get("OPPONENT_MASKS"); print("oracle masks", m.reshape(-1, 6)[:8].tolist())
print("engine masks", e.get("OPPONENT_MASKS").reshape(-1, 6)[:8].tolist())
