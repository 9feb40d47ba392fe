"""RewardMode::Flank (train_flank=True, Task.Zone) in the oracle:
flankRewardSystem (sim.cpp:4202-4278).  Each reward is 0.001 per teammate
out of sight or >= 100 away plus 0.001 per opponent that cannot see the
agent, +0.2 / +1 for a hit / kill from behind, plus exploration.  The engine
is compared with the oracle in tests/test_parity_gpu.py.
"""
import numpy as np

import mpenv_testlib as T


def test_flank_reward_decomposes():
    W, ts = 8, 3
    o = T.Oracle(W, ts, sim_flags=1, flank=True)
    o.put_ctrl([0, 1, 1])
    o.init()
    explore = np.float32(0.005)  # RewardHyperParams default exploreScale
    behind = 0
    for s in range(150):
        o.set_actions(T.combat_actions(o, s))
        o.step()
        for r in o.get("REWARD").ravel():
            ok = False
            for m in range(2 * ts):
                for bonus in (0.0, 0.2, 1.0):
                    for n in range(3):
                        if abs(r - (0.001 * m + bonus + float(explore) * n)) < 1e-5:
                            ok = True
                            behind += bonus > 0
            assert ok, r
    o.close()
