"""Task.ZoneCaptureDefend in the oracle: every episode
starts at zone 3 (sim.cpp:822-825); the match ends on the attacker's first
point, the defender's eighth, or when every attacker has died once, and
names the winner accordingly (sim.cpp:4534-4575, 4640-4651); the reward is
zoneCaptureDefendRewardSystem (sim.cpp:4089-4200).  simple_map has three
zones, so the tests use it with a fourth zone appended
(mpenv_testlib.four_zone_scene).  The engine is compared with the oracle on
the same case in tests/test_parity_gpu.py and the 6v6_capture_defend
golden fixture.
"""
import numpy as np
import pytest

import mpenv_testlib as T

ZCD = T.TASK_ZONE_CAPTURE_DEFEND


def test_capture_defend_rules(tmp_path):
    scene = T.four_zone_scene(tmp_path)
    W, ts = 8, 6
    o = T.Oracle(W, ts, sim_flags=1 | (1 << 6) | (1 << 4), task=ZCD, scene=scene)
    o.put_ctrl([0, 1, 1])
    o.init()
    wi = o.get("DEBUG_WORLD_I32").reshape(W, -1)
    assert np.all(wi[:, 3] == 3)
    results = {0: 0, 1: 0, 2: 0}
    for s in range(1500):
        prev_wi = o.get("DEBUG_WORLD_I32").reshape(W, -1).copy()
        o.set_actions(T.combat_actions(o, s))
        o.step()
        done = o.get("DONE").reshape(W, 2 * ts)[:, 0]
        mr = o.get("MATCH_RESULT").reshape(W, 30)
        rew = o.get("REWARD").reshape(W, 2 * ts)
        wi = o.get("DEBUG_WORLD_I32").reshape(W, -1)
        for w in range(W):
            if not done[w]:
                continue
            attacker = 1 if prev_wi[w, 0] == 1 else 0
            defender = attacker ^ 1
            win = mr[w, 0]
            results[int(win)] += 1
            if mr[w, 3 + attacker] == 1:
                assert win == attacker
            elif mr[w, 3 + defender] == 8:
                assert win == defender
            elif win != defender:  # attackers all died, or the episode ran out
                assert win == 2
            # the new episode starts at zone 3 again
            assert wi[w, 3] == 3
            assert np.all(np.abs(rew[w]) >= 4.0), rew[w]  # +-20 / -5 dominate (before team spirit mixing)
    assert sum(results.values()) > 5 and results[0] + results[1] > 0
    o.close()


def test_scene_with_three_zones_is_rejected():
    with pytest.raises(AssertionError):
        T.Oracle(2, 2, task=ZCD)
