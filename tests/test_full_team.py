"""FullTeamInterface outputs in the oracle:
fullTeamObservationsSystem (sim.cpp:3054-3301) and fullTeamDoneRewardSystem
(sim.cpp:4720-4747), checked through relations to the per-agent exports.
The engine is compared with the oracle on every FULL_TEAM_* export in every
GPU parity case (mpenv_testlib.STEP_OUTPUTS).
"""
import numpy as np
import pytest

import mpenv_testlib as T

COMMON, PLAYER, ENEMY, GLOBAL = 24, 28, 33, 16


def snapshot(o):
    return {n: o.get(n).copy() for n in T.STEP_OUTPUTS}


@pytest.mark.parametrize("ts,flags", [(2, 1 | 8), (3, 1 | 2), (6, 1)])  # 8 = NoRespawn
def test_full_team_relations(ts, flags):
    W = 4
    N = 2 * ts
    o = T.Oracle(W, ts, sim_flags=flags)
    o.put_ctrl([0, 1, 1])
    o.init()
    prev = snapshot(o)
    # after init: the lidar copy is the (zero) lidar before the first trace
    assert not o.get("FULL_TEAM_FWD_LIDAR").any()
    saw_knows = saw_dead = 0
    for s in range(120):
        o.set_actions(T.combat_actions(o, s))
        o.step()
        cur = snapshot(o)
        fwd = cur["FULL_TEAM_FWD_LIDAR"].reshape(W, 2, 6, -1)
        rear = cur["FULL_TEAM_REAR_LIDAR"].reshape(W, 2, 6, -1)
        pfwd = prev["FWD_LIDAR"].reshape(W, 2, ts, -1)
        prear = prev["REAR_LIDAR"].reshape(W, 2, ts, -1)
        np.testing.assert_array_equal(fwd[:, :, :ts], pfwd)
        np.testing.assert_array_equal(rear[:, :, :ts], prear)
        assert not fwd[:, :, ts:].any() and not rear[:, :, ts:].any()

        rew = cur["REWARD"].reshape(W, 2, ts)
        done = cur["DONE"].reshape(W, 2, ts)
        ft_r = cur["FULL_TEAM_REWARD"].reshape(W, 2)
        for w in range(W):
            for t in range(2):
                acc = np.float32(0)
                for k in range(ts):
                    acc = np.float32(acc + rew[w, t, k])
                assert ft_r[w, t] == acc
        np.testing.assert_array_equal(cur["FULL_TEAM_DONE"].reshape(W, 2), done.all(-1).astype(np.int32))

        g = cur["FULL_TEAM_GLOBAL"].reshape(W, 2, GLOBAL)
        np.testing.assert_array_equal(g[:, 0, :2], [[0, 1]] * W)
        np.testing.assert_array_equal(g[:, 1, :2], [[1, 0]] * W)
        assert np.all(g[:, :, 12:16].sum(-1) == 1)

        pl = cur["FULL_TEAM_PLAYERS"].reshape(W, 2, 6, PLAYER)
        en = cur["FULL_TEAM_ENEMIES"].reshape(W, 2, 6, ENEMY)
        lk = cur["FULL_TEAM_LAST_KNOWN_ENEMIES"].reshape(W, 2, 6, COMMON)
        hp = cur["HP"].reshape(W, 2, ts)
        alive = cur["ALIVE"].reshape(W, 2, ts)
        opp = cur["OPPONENT_OBSERVATIONS"].reshape(W, 2, ts, 6, 32)
        assert not pl[:, :, ts:].any() and not en[:, :, ts:].any() and not lk[:, :, ts:].any()
        for w in range(W):
            for t in range(2):
                for k in range(ts):
                    p = pl[w, t, k]
                    assert p[0] == 1 and p[1 + k] == 1 and p[1:7].sum() == 1
                    e = en[w, t ^ 1, k]
                    np.testing.assert_array_equal(e[:COMMON], p[:COMMON])
                    if alive[w, t, k] == 0:
                        saw_dead += 1
                        assert not p[7:].any() and not e[COMMON:].any() and not lk[w, t ^ 1, k].any()
                        continue
                    assert p[7] == 1 and p[24] == np.float32(hp[w, t, k] / np.float32(100))
                    # hasLOS[m]: own agent m's OpponentsVisibility of this enemy,
                    # as the per-agent opponent observation exports it
                    for m in range(ts):
                        if alive[w, t ^ 1, m]:
                            assert e[26 + m] == opp[w, t ^ 1, m, k, 30]
                    if e[32] == 1:
                        saw_knows += 1
                        np.testing.assert_array_equal(lk[w, t ^ 1, k], e[:COMMON])
                    else:
                        assert not lk[w, t ^ 1, k].any()
        prev = cur
    assert saw_knows > 0 and (saw_dead > 0 or not flags & 8)
    o.close()
