"""Spawn-mode sim flags in the oracle: HardcodedSpawns,
NavmeshSpawn and EnableCurriculum (LearnShooting).  The GPU engine is checked
against the oracle for the same flags in tests/test_parity_gpu.py (LIVE cases
and test_curriculum_resets_match_oracle) and the golden fixtures.

utils.cpp:734-948 spawnAgents picks, per dead agent: the hardcoded table on
episode start, else a navmesh sample, else (curriculum world in
LearnShooting) a random point in the spawn's half of the arena, else the
standard spawn search.
"""
import numpy as np
import pytest

import mpenv_testlib as T

HARDCODED = 1 << 6
NAVMESH = 1 << 2
CURRICULUM = 1 << 5

# utils.cpp:503-541 (pos.xyz, yaw)
TABLE = np.array([[510.0, 179.1, -64], [525.8, 17.1, -64], [434.3, 184.7, -64],
                  [1037.2, 449.0, -56], [1094.3, 200.1, -56], [1045.8, 416.8, -56]], np.float32)


def positions(o):
    o.lib.oracle_refresh_debug(o.h)
    return o.get("DEBUG_AGENT_F32")[:, :3].copy()


@pytest.mark.parametrize("ts", [1, 2, 3])
def test_hardcoded_spawns_use_the_table(ts):
    W = 6
    o = T.Oracle(W, ts, sim_flags=HARDCODED)
    o.put_ctrl([0, 0, 1])  # RandomFlipTeams: team A varies per world
    o.init()
    p = positions(o).reshape(W, 2 * ts, 3)
    team_a = o.get("DEBUG_WORLD_I32").reshape(W, -1)[:, 0]
    assert set(team_a.tolist()) <= {0, 1}
    for w in range(W):
        for i in range(2 * ts):
            team, off = divmod(i, ts)
            idx = (0 if team == team_a[w] else 3) + off
            np.testing.assert_array_equal(p[w, i], TABLE[idx])
    o.close()


def _in_triangle(pt, tri, eps=1e-2):
    a, b, c = tri.astype(np.float64)
    v0, v1, v2 = b - a, c - a, pt.astype(np.float64) - a
    m = np.array([[v0 @ v0, v0 @ v1], [v0 @ v1, v1 @ v1]])
    if abs(np.linalg.det(m)) < 1e-9:
        return False
    u, v = np.linalg.solve(m, [v2 @ v0, v2 @ v1])
    off = v2 - u * v0 - v * v1
    return u >= -eps and v >= -eps and u + v <= 1 + eps and np.linalg.norm(off) < 1e-2


def test_navmesh_spawns_lie_on_the_navmesh():
    W, ts = 16, 3
    o = T.Oracle(W, ts, sim_flags=NAVMESH)
    o.put_ctrl([0, 0, 0])
    o.init()
    p = positions(o)
    tris = o.navmesh()[0]
    hit = []
    for pt in p:
        on = [t for t in range(len(tris)) if _in_triangle(pt, tris[t])]
        assert on, pt
        hit.append(on[0])
    assert len(set(hit)) > len(p) // 4, "samples should spread over many triangles"
    o.close()


def test_navmesh_sampler_is_area_uniform():
    """The DEFINED Navmesh::samplePoint (mpenv_core.h): the share of samples
    per triangle tracks its share of the area."""
    tris = T.scene_navmesh()[0].reshape(-1, 3, 3).astype(np.float64)
    area = 0.5 * np.linalg.norm(np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]), axis=1)
    # Run many respawns: NavmeshSpawn also applies to respawns, NoRespawn off.
    W, ts = 64, 6
    o = T.Oracle(W, ts, sim_flags=NAVMESH)
    o.put_ctrl([0, 0, 0])
    o.init()
    p = positions(o)
    big = np.argsort(-area)[:5]
    counts = np.zeros(len(tris))
    for pt in p:
        for t in big:
            if _in_triangle(pt, tris[t].astype(np.float32)):
                counts[t] += 1
                break
    share = counts[big].sum() / len(p)
    expect = area[big].sum() / area.sum()
    assert abs(share - expect) < 0.12, (share, expect)
    o.close()


def test_curriculum_learn_shooting_spawns_and_reward():
    W, ts = 32, 2
    o = T.Oracle(W, ts, sim_flags=CURRICULUM)
    o.put_ctrl([0, 0, 0])
    o.init()
    cur = o.get("WORLD_CURRICULUM").ravel().copy()
    # first episode: FullMatch with probability 1/50 (sim.cpp:852-867)
    assert (cur == 0).sum() >= W - 4
    p = positions(o).reshape(W, 2 * ts, 3)
    for w in np.where(cur == 0)[0]:
        assert np.all(np.abs(p[w, :, 0]) <= 700) and np.all(np.abs(p[w, :, 1]) <= 350)
        assert np.all(p[w, :, 2] == 0)
    for s in range(40):
        acts = T.combat_actions(o, s)
        o.set_actions(acts)
        o.step()
        r = o.get("REWARD").reshape(W, 2 * ts)
        # learnShootingRewardSystem (sim.cpp:3707-3732) takes values in
        # {0.5, -0.05, 0, -0.5, 0, -0.55}
        vals = np.array([0.5, -0.05, 0.0, -0.5, -0.55], np.float32)
        ok = np.isclose(r[cur == 0][..., None], vals, atol=1e-6).any(-1)
        assert ok.all(), r[cur == 0]
    o.close()


def test_curriculum_tends_to_full_match_over_episodes():
    W, ts = 16, 1
    o = T.Oracle(W, ts, sim_flags=CURRICULUM, auto_reset=False)
    o.put_ctrl([0, 0, 0])
    o.init()
    frac = []
    for ep in range(60):
        o.view("RESET")[:] = 1
        o.set_actions(np.zeros((W * 2 * ts, 6), np.int32))
        o.step()
        frac.append(o.get("WORLD_CURRICULUM").mean())
    assert np.mean(frac[:10]) < 0.4 and all(f == 1.0 for f in frac[50:])
    o.close()


@pytest.mark.parametrize("ts", [4, 6])
def test_hardcoded_spawns_large_teams(ts):
    """team_size > 3: in-table indices as the reference; the other team's
    offsets 3..5 (past the table in the reference) reuse its entries."""
    W = 4
    o = T.Oracle(W, ts, sim_flags=HARDCODED)
    o.put_ctrl([0, 0, 1])
    o.init()
    p = positions(o).reshape(W, 2 * ts, 3)
    team_a = o.get("DEBUG_WORLD_I32").reshape(W, -1)[:, 0]
    for w in range(W):
        for i in range(2 * ts):
            team, off = divmod(i, ts)
            idx = (0 if team == team_a[w] else 3) + off
            np.testing.assert_array_equal(p[w, i], TABLE[idx if idx < 6 else idx - 3])
    o.close()
