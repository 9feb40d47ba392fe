"""Trajectory curriculum (curriculum_data_path) in the
oracle: at an episode start, half the time (not in eval mode) a recorded
match state replaces the spawned one (level_gen.cpp:498-580).  The engine is
compared with the oracle on the same file in tests/test_parity_gpu.py.
"""
import numpy as np

import mpenv_testlib as T


def test_snapshots_applied_at_episode_start(tmp_path):
    path = T.make_curriculum_file(str(tmp_path / "curriculum.bin"), n=32)
    snaps = np.fromfile(path, T.CURRICULUM_SNAPSHOT)
    W, ts = 16, 6
    o = T.Oracle(W, ts, sim_flags=1, curriculum=path)
    o.put_ctrl([0, 0, 1])
    o.init()
    o.lib.oracle_refresh_debug(o.h)
    af = o.get("DEBUG_AGENT_F32").reshape(W, 12, -1)
    wi = o.get("DEBUG_WORLD_I32").reshape(W, -1)
    hp = o.get("HP").reshape(W, 12)
    mag = o.get("MAGAZINE").reshape(W, 12, 2)
    matched = 0
    for w in range(W):
        cands = [k for k in range(len(snaps)) if snaps[k]["step"] == wi[w, 1]]
        if not cands:
            continue
        sn = snaps[cands[0]]
        order = np.arange(12) if wi[w, 0] == 0 else np.r_[6:12, 0:6]
        for i in range(12):
            j = order[i]
            p = sn["players"][i]
            np.testing.assert_array_equal(af[w, j, 0:3], p["pos"].astype(np.float32))
            assert hp[w, j] == np.float32(p["hp"])
            assert mag[w, j, 0] == p["mag"] and mag[w, j, 1] == p["reloading"]
        assert wi[w, 3] == sn["cur_zone"]
        assert wi[w, 4] == sn["controller"]
        matched += 1
    # half the episodes start from a snapshot
    assert 2 <= matched <= W - 2
    o.close()


def test_eval_mode_skips_the_curriculum(tmp_path):
    path = T.make_curriculum_file(str(tmp_path / "curriculum.bin"), n=8)
    W = 8
    o = T.Oracle(W, 2, sim_flags=1 | (1 << 10), curriculum=path)  # SimEvalMode
    o.put_ctrl([1, 0, 0])
    o.init()
    assert np.all(o.get("DEBUG_WORLD_I32").reshape(W, -1)[:, 1] == 0)
    o.close()
