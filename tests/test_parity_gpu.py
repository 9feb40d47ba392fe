"""Engine (gfx950 HIP, through the C ABI) vs the CPU oracle.

Bar: bit-exact for every export — discrete state, and also
the floats, because both sides compile the same IEEE-exact definitions
(mpenv_core.h, -ffp-contract=off).  `FLOAT_RTOL` below is the stated ceiling
the north star allows (1e-5 relative); the tests run with 0 (bit-exact) and
only fall back to the tolerance where a test says so.
"""
import ctypes as C
import json
import os
import glob

import numpy as np
import pytest

import mpenv_testlib as T
from golden.make_golden import make_sim, rollout, set_bots, step_hashes

pytestmark = pytest.mark.gpu

FLOAT_RTOL = 1e-5  # north_star tolerance; asserted bit-exact (0) below
ALL = T.STEP_OUTPUTS + T.DEBUG_OUTPUTS
GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json")))


def _compare_all(e, o, where):
    for n in ALL:
        T.compare(e.get(n), o.get(n), f"{n} @ {where}")
    T.compare(T.explore_visited(e), T.explore_visited(o), f"explore cells @ {where}")


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
def test_engine_matches_golden_fixture(path):
    g = json.load(open(path))
    case = g["case"]
    e = make_sim(T.Engine, case)
    for k, s in enumerate(rollout(e, case)):
        got = step_hashes(e)
        bad = [n for n in got if got[n] != g["hashes"][k][n]]
        assert not bad, f"step {s}: {bad}"
    for n, v in g["final"].items():
        np.testing.assert_array_equal(e.get(n).ravel(), np.asarray(v, np.float32), err_msg=n)
    e.close()


LIVE = [
    # team_size, worlds, steps, sim_flags, ctrl, policy
    (1, 64, 300, 0, [0, 1, 1], "tape"),
    # agent counts that are not a multiple of 4 / 64: k_lidar's 4-agent wave
    # units and k_obs's per-wave row transpose end in a partial unit
    (3, 7, 120, 0, [0, 1, 1], "tape"),
    (1, 3, 120, 1, [0, 1, 1], "combat"),
    (5, 13, 120, 1, [0, 1, 1], "combat"),
    (2, 32, 300, 0, [0, 1, 1], "tape"),
    (3, 16, 300, 0, [0, 1, 1], "tape"),
    (6, 16, 300, 0, [0, 1, 1], "tape"),
    (3, 32, 400, 1 | 2, [0, 1, 1], "combat"),           # middle spawns, random hp/mag
    (6, 8, 400, 1, [0, 1, 1], "combat"),
    (2, 16, 300, 1 | 8 | 16, [0, 0, 0], "combat"),      # NoRespawn | StaggerStarts
    (4, 8, 300, 1 | (1 << 7) | (1 << 10), [1, 0, 1], "combat"),  # RandomFlip | SimEvalMode
    (5, 8, 300, 1 | (1 << 8), [0, 1, 0], "combat"),     # StaticFlipTeams
    (3, 16, 300, 1, [0, 1, 1], "bots_team1"),           # A* bots vs tape
    (6, 8, 300, 0, [0, 1, 1], "bots_all"),              # everyone an A* bot
    (3, 16, 300, 1 | (1 << 6), [0, 1, 1], "combat"),    # HardcodedSpawns
    (6, 8, 200, 1 | (1 << 6), [0, 1, 1], "combat"),     # HardcodedSpawns past the table
    (6, 16, 300, 2 | (1 << 2), [0, 1, 1], "combat"),    # NavmeshSpawn
    (2, 32, 300, 1 | (1 << 5), [0, 1, 1], "combat"),    # EnableCurriculum
    (4, 8, 200, 1 | 8 | (1 << 9), [0, 1, 1], "combat"),  # FullTeamPolicy | NoRespawn
    (3, 16, 300, 1 | (1 << 11), [0, 1, 1], "bots_cycle"),     # SubZones, policies -1..8
    (6, 8, 300, 1 | 2 | (1 << 11), [0, 1, 1], "bots_cycle"),
]


@pytest.mark.parametrize("ts,worlds,steps,flags,ctrl,policy", LIVE,
                         ids=[f"{c[0]}v{c[0]}x{c[1]}_f{c[3]}_{c[5]}" for c in LIVE])
def test_engine_matches_oracle_live(ts, worlds, steps, flags, ctrl, policy):
    e = T.Engine(worlds, ts, sim_flags=flags)
    o = T.Oracle(worlds, ts, sim_flags=flags)
    for sim in (e, o):
        sim.put_ctrl(ctrl)
        sim.init()
        if policy.startswith("bots"):
            set_bots(sim, dict(worlds=worlds, team_size=ts, bots=policy[5:]))
    _compare_all(e, o, "init")
    A = worlds * 2 * ts
    for s in range(steps):
        acts = T.combat_actions(o, s) if policy == "combat" else T.mpenv_tape.tape_actions(1234, s, 0, A)
        e.set_actions(acts)
        o.set_actions(acts)
        e.step()
        o.step()
        if s % 10 == 0 or s == steps - 1:
            _compare_all(e, o, f"step {s}")
        else:
            for n in ("SELF_OBSERVATION", "REWARD", "DONE", "HP", "DEBUG_AGENT_I32"):
                T.compare(e.get(n), o.get(n), f"{n} @ step {s}")
    e.close()
    o.close()


def test_device_combat_actions_match_numpy_and_drive_combat():
    """mpenv_combat_actions (the bench's combat action source) equals the
    tests' numpy aim-bots on the engine's own observations -- mode 0
    (combat_actions) and mode 1 (seek_combat_actions) -- and the fused form
    (written straight into the step inputs) keeps the engine bit-exact with
    the oracle stepped with the numpy actions; kills and respawns happen."""
    ts, W, steps = 6, 64, 600
    N = 2 * ts
    A = W * N
    e = T.Engine(W, ts)
    o = T.Oracle(W, ts)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    ring = T.mpenv_tape.tape_ring(1234, 0, A, 8)
    dev_ring = e.mem.upload(ring)
    out = e.mem.upload(np.zeros((A, 6), np.int32))
    got = np.empty((A, 6), np.int32)
    e.enable_stats(True)  # kill counter (a killed agent respawns within its step)
    for s in range(steps):
        mode = 0 if s < 40 else 1
        fn = T.combat_actions if mode == 0 else T.seek_combat_actions
        slot = dev_ring + (s % 8) * A * 24
        e.combat_actions(slot, out, mode)
        e.mem.d2h(out, got.nbytes, got)
        np.testing.assert_array_equal(got, fn(e, s, base=ring[s % 8]), err_msg=f"mode {mode} step {s}")
        acts = fn(o, s, base=ring[s % 8])
        e.combat_actions(slot, None, mode)
        o.set_actions(acts)
        e.step()
        o.step()
        if s % 10 == 0 or s == steps - 1:
            _compare_all(e, o, f"step {s}")
        else:
            for n in ("SELF_OBSERVATION", "PVP_DISCRETE_ACTION", "PVP_DISCRETE_AIM_ACTION", "HP", "REWARD"):
                T.compare(e.get(n), o.get(n), f"{n} @ step {s}")
    e.mem.free(dev_ring)
    e.mem.free(out)
    st = e.read_stats()
    print(f"\n{W} worlds {ts}v{ts}, {steps} steps of device combat actions: {st['kills']} kills, "
          f"{st['hit_agents']} agent-steps hit")
    assert st["kills"] > 0 and st["hit_agents"] > st["kills"]
    e.close()
    o.close()


def test_auto_reset_off_and_triggered_resets():
    """auto_reset=False: episodes end only through the reset tensor
    (mgr.cpp:2484-2500 triggerReset; sim.cpp resetSystem)."""
    ts, W = 2, 8
    e = T.Engine(W, ts, auto_reset=False)
    o = T.Oracle(W, ts, auto_reset=False)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    A = W * 2 * ts
    for s in range(200):
        if s in (5, 77, 150):
            w = s % W
            e.trigger_reset(w)
            o.view("RESET")[w] = 1
        if s == 40:
            e.set_hp(1, 0, 7)
            o.view("HP")[1 * 2 * ts + 0] = 7
        acts = T.mpenv_tape.tape_actions(1234, s, 0, A)
        e.set_actions(acts)
        o.set_actions(acts)
        e.step()
        o.step()
        _compare_all(e, o, f"step {s}")


def test_zone_capture_defend_matches_oracle(tmp_path):
    """Task.ZoneCaptureDefend, 6v6 as scripts/jax_train.py sets it up
    (HardcodedSpawns | StaggerStarts, random team sides), on simple_map
    with a fourth zone; long enough for several matches to end."""
    scene = T.four_zone_scene(tmp_path)
    ts, W = 6, 16
    flags = 1 | (1 << 6) | (1 << 4)
    e = T.Engine(W, ts, sim_flags=flags, task=T.TASK_ZONE_CAPTURE_DEFEND, scene=scene)
    o = T.Oracle(W, ts, sim_flags=flags, task=T.TASK_ZONE_CAPTURE_DEFEND, scene=scene)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    _compare_all(e, o, "init")
    ends = 0
    for s in range(700):
        acts = T.combat_actions(o, s)
        e.set_actions(acts)
        o.set_actions(acts)
        e.step()
        o.step()
        ends += int(o.get("DONE").reshape(W, -1)[:, 0].sum())
        if s % 10 == 0:
            _compare_all(e, o, f"step {s}")
        else:
            for n in ("SELF_OBSERVATION", "REWARD", "DONE", "MATCH_RESULT", "DEBUG_WORLD_I32"):
                T.compare(e.get(n), o.get(n), f"{n} @ step {s}")
    assert ends > 0
    e.close()
    o.close()


def test_curriculum_data_matches_oracle(tmp_path):
    """curriculum_data_path: recorded match states applied at episode
    starts (level_gen.cpp:498-580), over many triggered resets."""
    path = T.make_curriculum_file(str(tmp_path / "curriculum.bin"), n=48)
    for ts in (6, 3):
        W = 16
        e = T.Engine(W, ts, sim_flags=1, curriculum=path)
        o = T.Oracle(W, ts, sim_flags=1, curriculum=path)
        for sim in (e, o):
            sim.put_ctrl([0, 1, 1])
            sim.init()
        _compare_all(e, o, f"ts {ts} init")
        for s in range(200):
            if s % 10 == 0:
                for w in range(W):
                    if (s // 10 + w) % 4 == 0:
                        e.trigger_reset(w)
                        o.view("RESET")[w] = 1
            acts = T.combat_actions(o, s)
            e.set_actions(acts)
            o.set_actions(acts)
            e.step()
            o.step()
            if s % 5 == 0:
                _compare_all(e, o, f"ts {ts} step {s}")
            else:
                for n in ("SELF_OBSERVATION", "REWARD", "HP", "DEBUG_WORLD_I32"):
                    T.compare(e.get(n), o.get(n), f"{n} @ ts {ts} step {s}")
        e.close()
        o.close()


def test_flank_reward_matches_oracle():
    """train_flank: flankRewardSystem's visibility checks run per agent in
    k_sim (sim.cpp:4202-4278)."""
    for ts in (2, 6):
        W = 16
        e = T.Engine(W, ts, sim_flags=1, flank=True)
        o = T.Oracle(W, ts, sim_flags=1, flank=True)
        for sim in (e, o):
            sim.put_ctrl([0, 1, 1])
            sim.init()
        for s in range(200):
            acts = T.combat_actions(o, s)
            e.set_actions(acts)
            o.set_actions(acts)
            e.step()
            o.step()
            if s % 10 == 0:
                _compare_all(e, o, f"ts {ts} step {s}")
            else:
                for n in ("REWARD", "DEBUG_AGENT_I32"):
                    T.compare(e.get(n), o.get(n), f"{n} @ ts {ts} step {s}")
        e.close()
        o.close()


def test_curriculum_resets_match_oracle():
    """EnableCurriculum across many episodes: the LearnShooting/FullMatch
    draw per reset (sim.cpp:852-867), LearnShooting spawns and rewards
    (utils.cpp:819-837, sim.cpp:3707-3732), with NavmeshSpawn on half the
    runs taking precedence for spawns (utils.cpp:805-809)."""
    for flags in (1 << 5, (1 << 5) | (1 << 2)):
        ts, W = 2, 16
        e = T.Engine(W, ts, sim_flags=flags, auto_reset=False)
        o = T.Oracle(W, ts, sim_flags=flags, auto_reset=False)
        for sim in (e, o):
            sim.put_ctrl([0, 1, 1])
            sim.init()
        for s in range(400):
            if s % 8 == 0:
                for w in range(W):
                    if (s // 8 + w) % 3 == 0:
                        e.trigger_reset(w)
                        o.view("RESET")[w] = 1
            acts = T.combat_actions(o, s)
            e.set_actions(acts)
            o.set_actions(acts)
            e.step()
            o.step()
            if s % 5 == 0:
                _compare_all(e, o, f"flags {flags} step {s}")
            else:
                for n in ("SELF_OBSERVATION", "REWARD", "WORLD_CURRICULUM"):
                    T.compare(e.get(n), o.get(n), f"{n} @ flags {flags} step {s}")
        cur = o.get("WORLD_CURRICULUM").ravel()
        assert 0 < cur.sum() < W or s > 0
        e.close()
        o.close()


LONG = [
    # team_size, worlds (the configuration's full batch), steps, probe world offsets
    (6, 16384, 3100, [0, 4097, 12345, 16384 - 3]),   # C3, the headline batch
    (3, 4096, 3100, [0, 1001, 2050, 4096 - 3]),      # C2
]


@pytest.mark.parametrize("ts,W,steps,probes", LONG, ids=["C3_6v6x16384", "C2_3v3x4096"])
def test_full_batch_long_horizon_matches_oracle(ts, W, steps, probes):
    """A full configuration batch (C3 / C2 size) stepped past one whole
    episode (3,000 steps, consts.hpp episodeLen) against oracle runs of
    3-world slices of the same global worlds (world_id_offset), bit-exact on
    every STEP_OUTPUT and the internal state every 50 steps.

    Actions: the bench's hash tape (ring of 64 steps resident in HBM) with
    team slot 1 of every even world an A* bot (AgentPolicy -1,
    planAStarAISystem), which walks to the zone and holds it; every other
    agent of the whole batch follows the zone-seeking aim-bot computed on the
    device from the engine's own observations (mpenv_combat_actions mode 1,
    written straight into the step inputs), the oracle slices the same
    function in numpy (mpenv_testlib.seek_combat_actions) from theirs, so
    both teams converge on the zone and kills, respawns and combat rewards
    happen throughout the horizon.  That drives the zone systems through their natural events
    (sim.cpp:1892-1976 rotation after 600 controlled steps, 4470-4673 a point
    every 20 controlled steps and the 3,000-step end).  A 125-point win needs
    2,500 controlled steps, which the bots reach too rarely, so at steps
    1000 and 2000 the learner-visible episode_results buffer
    (pbt.episode_results = MATCH_RESULT, mgr.cpp:2252-2260, read and
    accumulated in place by zoneMatchInfoSystem) is raised to 124 points per
    team in the probed worlds, identically on both sides: the next point
    earned ends the match by the 125-point rule (sim.cpp:4529-4532)."""
    from concurrent.futures import ThreadPoolExecutor

    N = 2 * ts
    RING = 64
    PW = 3  # worlds per probe slice
    e = T.Engine(W, ts)
    e.put_ctrl([0, 1, 1])
    e.init()
    pol = np.zeros((W, 2, ts), np.int32)
    pol[0::2, 1, :] = -1
    e.put("AGENT_POLICY", pol.reshape(-1, 1))
    ring = np.stack([T.mpenv_tape.tape_actions(1234, k, 0, W * N) for k in range(RING)])
    dev_ring = e.mem.upload(ring)
    oracles = []
    for w0 in probes:
        o = T.Oracle(PW, ts, world_id_offset=w0)
        o.put_ctrl([0, 1, 1])
        o.init()
        o.view("AGENT_POLICY")[:] = pol[w0:w0 + PW].reshape(-1, 1)
        oracles.append(o)
    names = T.STEP_OUTPUTS + ["DEBUG_AGENT_I32", "DEBUG_WORLD_I32", "DEBUG_AGENT_F32"]

    def compare(s):
        for w0, o in zip(probes, oracles):
            for n in names:
                _, _, shape = e.desc(n)
                rpw = shape[0] // W  # rows per world: 1 (world), 2 (team interface) or N (agent)
                T.compare(e.get_rows(n, w0 * rpw, (w0 + PW) * rpw), o.get(n), f"{n} worlds {w0}.. @ {s}")

    ev = dict(rotations=0, points=0, wins=0, episode_ends=0, kills=0)
    prev = [o.get("DEBUG_WORLD_I32").copy() for o in oracles]
    prev_kills = [np.zeros(PW, np.int32) for _ in oracles]

    acts = [None] * len(oracles)

    def ostep(k, s):
        oracles[k].set_actions(acts[k])
        oracles[k].step()

    compare("init")
    e.enable_stats(True)  # whole-batch hit / kill counters
    with ThreadPoolExecutor(len(oracles)) as pool:
        for s in range(steps):
            if s in (1000, 2000):
                for w0, o in zip(probes, oracles):
                    mr = o.view("MATCH_RESULT")
                    mr[:, 3] = np.maximum(mr[:, 3], 124)
                    mr[:, 4] = np.maximum(mr[:, 4], 124)
                    e.put_rows("MATCH_RESULT", w0, mr)
            slot = dev_ring + (s % RING) * W * N * 6 * 4
            for k, (w0, o) in enumerate(zip(probes, oracles)):
                acts[k] = T.seek_combat_actions(o, s, base=ring[s % RING, w0 * N:(w0 + PW) * N])
            e.combat_actions(slot, None, 1)
            e.step()
            list(pool.map(lambda k: ostep(k, s), range(len(oracles))))
            for k, o in enumerate(oracles):
                o.lib.oracle_refresh_debug(o.h)
                wi = o.view("DEBUG_WORLD_I32")
                done = o.view("DONE").reshape(PW, N)[:, 0] == 1
                mr = o.view("MATCH_RESULT")
                ev["rotations"] += int(((wi[:, 3] != prev[k][:, 3]) & (wi[:, 1] == prev[k][:, 1] + 1)).sum())
                ev["points"] += int(wi[:, 7].sum())
                ev["wins"] += int((done & (np.maximum(mr[:, 3], mr[:, 4]) >= 125)).sum())
                ev["episode_ends"] += int(done.sum())
                kills = mr[:, 1] + mr[:, 2]
                ev["kills"] += int(np.where(wi[:, 1] == prev[k][:, 1] + 1, np.maximum(kills - prev_kills[k], 0), 0).sum())
                prev_kills[k] = kills.copy()
                prev[k] = wi.copy()
            if s % 50 == 49 or s == steps - 1:
                compare(f"step {s}")
    e.mem.free(dev_ring)
    batch = e.read_stats()
    e.enable_stats(False)
    print(f"\n{ts}v{ts} x {W}, {steps} steps, {len(probes)} x {PW} probed worlds: {ev}; whole batch: "
          f"{batch['kills']} kills, {batch['hit_agents']} agent-steps hit, {batch['los_seen']} LOS rays seen")
    # every zone/match event fired in the probed worlds, and combat throughout
    assert ev["rotations"] > 0 and ev["points"] > 0 and ev["wins"] > 0, ev
    assert ev["kills"] >= 20, ev
    assert batch["kills"] >= W, batch  # more kills than worlds over the horizon
    assert ev["episode_ends"] >= len(probes) * PW, ev  # every world passed a 3,000-step end or a win
    # size-independent properties over the whole batch
    hp = e.get("HP")
    assert np.isfinite(e.get("SELF_OBSERVATION")).all()
    assert ((hp >= 0) & (hp <= 100)).all()
    assert np.isfinite(e.get("FWD_LIDAR")).all()
    e.close()


def test_python_module_zero_copy_and_stream_step():
    """madrona_mp_env.SimManager (bindings.cpp surface): torch views of the
    engine's buffers, step_async on a torch stream, copy_actions, and the
    train_interface table — results equal the oracle's."""
    import torch
    import madrona_mp_env as m

    ts, W = 3, 8
    sim = m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                       auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                       team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE)
    o = T.Oracle(W, ts)
    ctrl = sim.sim_control_tensor().to_torch()
    ctrl.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device=ctrl.device).view_as(ctrl))
    o.put_ctrl([0, 1, 1])
    sim.init()
    o.init()
    obs = sim.self_observation_tensor().to_torch()
    rew = sim.reward_tensor().to_torch()
    assert obs.device.type == "cuda" and obs.shape == (W * 2 * ts, 43)
    A = W * 2 * ts
    stream = torch.cuda.Stream()
    ring = torch.from_numpy(np.stack([T.mpenv_tape.tape_actions(1234, s, 0, A) for s in range(50)]))
    ring = ring.to("cuda")
    for s in range(50):
        with torch.cuda.stream(stream):
            sim.copy_actions(ring[s].data_ptr(), stream.cuda_stream)
            sim.step_async(stream.cuda_stream)
        o.set_actions(ring[s].cpu().numpy())
        o.step()
        stream.synchronize()
        np.testing.assert_array_equal(obs.cpu().numpy(), o.get("SELF_OBSERVATION"))
        np.testing.assert_array_equal(rew.cpu().numpy(), o.get("REWARD"))
    ti = sim.train_interface()
    assert set(ti) == {"inputs", "outputs"}
    assert "rewards" in ti["outputs"] and "discrete" in ti["inputs"]
    reg = sim.jax(True)  # the XLA targets (test_jax_custom_call_targets_match_gpu_stream_step)
    assert set(reg["output_names"]) == set(ti["outputs"])
    with pytest.raises(Exception):
        sim.jax(False)  # no CPU (ExecMode.CPU) targets


def test_kernel_timing_hooks():
    e = T.Engine(256, 6)
    assert e.lib.mpenv_enable_kernel_timing(e.h, 1) == 0
    e.init()
    for s in range(5):
        e.step()
    import ctypes as C

    names = (C.c_char_p * 16)()
    ms = (C.c_float * 16)()
    launches = (C.c_int32 * 16)()
    n = e.lib.mpenv_kernel_timings(e.h, 16, names, ms, launches)
    got = {names[i].decode(): (ms[i], launches[i]) for i in range(n)}
    assert set(got) >= {"k_move", "k_sim", "k_vis", "k_obs", "k_lidar"}
    assert all(v[1] == 5 and v[0] > 0 for v in got.values())


def test_cpp_manager_headless_runs():
    """The C++ Manager wrapper (include/mpenv_manager.hpp) drives the engine."""
    import subprocess

    r = subprocess.run([T.build_native.HEADLESS, "CUDA", "256", "50", T.SCENE, "--rand-actions"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "FPS" in r.stdout and float(r.stdout.split("FPS")[1].split()[0]) > 0


@pytest.mark.parametrize("groups", [1, 2])
def test_gpu_stream_step_buffers_abi(groups):
    """Manager::gpuStreamInit/gpuStreamStep (mgr.cpp:507-645): a flat
    buffer array of TrainInterface inputs then outputs, caller-owned, on the
    caller's stream — the XLA custom-call ABI scripts/jax_train.py uses.
    The observation rows and the lidar are written by k_obs / k_lidar
    straight into the call's buffers (engine.h OutTab): two caller buffer
    sets alternate step by step (XLA hands out fresh result buffers), every
    output of the set a step used equals the oracle, and the captured step
    graph is not re-captured for them.  Afterwards a plain step() writes the
    engine's own exports again (the table is off outside the call)."""
    import ctypes as C
    import torch

    ts, W = 2, 16
    A = W * 2 * ts
    lib = T.lib_mpenv()
    lib.mpenv_gpu_stream_init.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]
    lib.mpenv_gpu_stream_step.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]
    lib.mpenv_train_interface_entry.argtypes = [C.c_int32, C.c_int32, C.POINTER(C.c_char_p),
                                                C.POINTER(C.c_int32)]
    e = T.Engine(W, ts)
    o = T.Oracle(W, ts)
    ni, no = C.c_int32(), C.c_int32()
    assert lib.mpenv_train_interface_size(C.byref(ni), C.byref(no)) == 0
    if groups > 1:
        lib.mpenv_set_world_groups.argtypes = [C.c_void_p, C.c_int32]
        assert lib.mpenv_set_world_groups(e.h, groups) == 0
    names, sets = [], [[], []]
    inv = {v: k for k, v in T.EXPORT.items()}
    for io, n in ((0, ni.value), (1, no.value)):
        for k in range(n):
            nm, eid = C.c_char_p(), C.c_int32()
            assert lib.mpenv_train_interface_entry(io, k, C.byref(nm), C.byref(eid)) == 0
            _, dt, shape = e.desc(inv[eid.value])
            tdt = {np.int32: torch.int32, np.float32: torch.float32}[dt]
            names.append((io, nm.value.decode(), inv[eid.value]))
            for bs in sets:  # outputs not zeros: every byte must be written
                bs.append(torch.full(shape, 7 if io == 1 else 0, dtype=tdt, device="cuda"))
    arrs = [(C.c_void_p * len(bs))(*[b.data_ptr() for b in bs]) for bs in sets]
    idx = {nm: i for i, (io, nm, _) in enumerate(names)}
    for bs in sets:
        bs[idx["simCtrl"]].copy_(torch.tensor([0, 1, 1], dtype=torch.int32).view_as(bs[idx["simCtrl"]]))
    o.put_ctrl([0, 1, 1])
    stream = torch.cuda.Stream()
    e.put_ctrl([0, 1, 1])
    assert lib.mpenv_gpu_stream_init(e.h, C.c_void_p(stream.cuda_stream), arrs[0]) == 0
    o.init()
    stream.synchronize()
    lib.mpenv_graph_captures.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    caps = []
    for s in range(40):
        bufs = sets[s % 2]
        acts = T.mpenv_tape.tape_actions(1234, s, 0, A)
        bufs[idx["discrete"]].copy_(torch.from_numpy(acts[:, :4].copy()).view_as(bufs[idx["discrete"]]))
        bufs[idx["aim"]].copy_(torch.from_numpy(acts[:, 4:6].copy()).view_as(bufs[idx["aim"]]))
        torch.cuda.synchronize()
        assert lib.mpenv_gpu_stream_step(e.h, C.c_void_p(stream.cuda_stream), arrs[s % 2]) == 0
        o.set_actions(acts)
        o.step()
        stream.synchronize()
        for (io, nm, ename), b in zip(names, bufs):
            if io == 1:
                T.compare(b.cpu().numpy(), o.get(ename), f"{nm} @ {s}")
        n = C.c_int64()
        assert lib.mpenv_graph_captures(e.h, C.byref(n)) == 0
        caps.append(n.value)
    assert caps[1] >= 1 and caps[-1] == caps[1], caps  # one capture serves both buffer sets
    # a plain step afterwards: the engine's own exports are written again
    acts = T.mpenv_tape.tape_actions(1234, 40, 0, A)
    e.set_actions(acts)
    e.step()
    o.set_actions(acts)
    o.step()
    for (io, nm, ename) in names:
        if io == 1 and nm != "unmasked_agent_map" and nm != "agent_map":
            T.compare(e.get(ename), o.get(ename), f"engine export {nm} after the stream steps")


def test_jax_custom_call_targets_match_gpu_stream_step():
    """SimManager.jax() (JAXInterface::buildEntry, bindings.cpp:149-158): the
    XLA GPU custom-call targets as PyCapsules named xla._CUSTOM_CALL_TARGET
    plus the opaque bytes naming the manager.  Called as XLA would -- the
    function pointer taken out of the capsule, (stream, operands + results,
    opaque, len) -- on one manager, and gpu_stream_step on a twin with the
    same inputs: every output buffer equal byte for byte.  Also: a short
    buffer list is refused (ValueError); the status-returning twin
    (API_VERSION_STATUS_RETURNING) runs every other step and gives the same
    bytes.  A foreign opaque aborts the v1 target (the reference's FATAL):
    that is tested on the CPU, in a subprocess (tests/test_abi.py)."""
    import ctypes as C

    import torch
    import madrona_mp_env as m

    ts, W, steps = 3, 32, 30
    A = W * 2 * ts

    def mk():
        return m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                            auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                            team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE)

    a, b = mk(), mk()
    reg = a.jax(True)
    assert reg["platform"] == "ROCM" and reg["api_version"] == 1
    get_ptr = C.pythonapi.PyCapsule_GetPointer
    get_ptr.restype = C.c_void_p
    get_ptr.argtypes = [C.py_object, C.c_char_p]
    XlaFn = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_size_t)
    init_fn = XlaFn(get_ptr(reg["init"], b"xla._CUSTOM_CALL_TARGET"))
    step_fn = XlaFn(get_ptr(reg["step"], b"xla._CUSTOM_CALL_TARGET"))
    assert reg["status_api_version"] == 2
    XlaFnS = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_size_t, C.c_void_p)
    step_status_fn = XlaFnS(get_ptr(reg["step_status"], b"xla._CUSTOM_CALL_TARGET"))
    opaque = reg["opaque"]
    ti = a.train_interface()
    names = list(reg["input_names"]) + list(reg["output_names"])
    assert list(reg["input_names"]) == list(ti["inputs"]) and list(reg["output_names"]) == list(ti["outputs"])
    ref = {**{k: v.to_torch() for k, v in ti["inputs"].items()}, **{k: v.to_torch() for k, v in ti["outputs"].items()}}
    bufs_a = [torch.zeros_like(ref[n]) for n in names]
    bufs_b = [torch.zeros_like(ref[n]) for n in names]
    arr_a = (C.c_void_p * len(names))(*[t.data_ptr() for t in bufs_a])
    ptrs_b = [t.data_ptr() for t in bufs_b]
    ni = len(reg["input_names"])
    idx = {n: i for i, n in enumerate(names)}
    for bufs in (bufs_a, bufs_b):
        bufs[idx["simCtrl"]].copy_(torch.tensor([0, 1, 1], dtype=torch.int32).view_as(bufs[idx["simCtrl"]]))
    with pytest.raises(ValueError):
        b.gpu_stream_step(0, ptrs_b[:-1])
    lib = T.lib_mpenv()
    lib.mpenv_xla_errors.restype = C.c_int64
    errs0 = lib.mpenv_xla_errors()
    stream = torch.cuda.Stream()
    # the reference's ordering: gpuStreamInit's forced reset reads simCtrl
    # from the engine, so set it there as Manager::init callers do
    for sim in (a, b):
        c = sim.sim_control_tensor().to_torch()
        c.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device=c.device).view_as(c))
    torch.cuda.synchronize()
    init_fn(C.c_void_p(stream.cuda_stream), arr_a, opaque, len(opaque))
    b.gpu_stream_init(stream.cuda_stream, ptrs_b)
    stream.synchronize()
    for s in range(steps):
        acts = torch.from_numpy(T.mpenv_tape.tape_actions(1234, s, 0, A))
        for bufs in (bufs_a, bufs_b):
            bufs[idx["discrete"]].copy_(acts[:, :4].contiguous().view_as(bufs[idx["discrete"]]))
            bufs[idx["aim"]].copy_(acts[:, 4:6].contiguous().view_as(bufs[idx["aim"]]))
        torch.cuda.synchronize()
        if s % 2:
            step_status_fn(C.c_void_p(stream.cuda_stream), arr_a, opaque, len(opaque), None)
        else:
            step_fn(C.c_void_p(stream.cuda_stream), arr_a, opaque, len(opaque))
        b.gpu_stream_step(stream.cuda_stream, ptrs_b)
        stream.synchronize()
        for k in range(ni, len(names)):
            x, y = bufs_a[k], bufs_b[k]
            assert torch.equal(x.view(torch.uint8), y.view(torch.uint8)), (names[k], s)
    assert lib.mpenv_xla_errors() == errs0
    assert int(bufs_a[idx["hp"]].ne(0).sum()) > 0


_edge_aimed_rays = T.edge_aimed_rays


def test_bvh_traversal_matches_oracle_on_edge_cases():
    """GPU closest-hit traversal (inlined and out-of-line) vs the oracle's
    restatement of MeshBVH::traceRay, on random rays and on rays aimed
    exactly at shared edges/vertices (where triangles tie)."""
    import ctypes as C
    import torch

    lib = T.lib_mpenv()
    lib.mpenv_debug_trace_rays.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                           C.c_void_p, C.c_void_p, C.c_void_p]
    e = T.Engine(1, 1)
    o = T.Oracle(1, 1)
    nodes, verts, _ = T.scene_bvh()
    rng = np.random.default_rng(11)
    ro = rng.uniform([-2000, -2000, -150], [2000, 2000, 600], (200000, 3)).astype(np.float32)
    rd = rng.normal(size=(200000, 3))
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    eo, ed = _edge_aimed_rays(verts, 40, 12)
    ro = np.concatenate([ro, eo])
    rd = np.concatenate([rd, ed])
    n = len(ro)
    od = torch.from_numpy(ro).cuda()
    dd = torch.from_numpy(rd).cuda()
    res = []
    for mode in (0, 1):
        t = torch.zeros(n, dtype=torch.float32, device="cuda")
        h = torch.zeros(n, dtype=torch.int32, device="cuda")
        assert lib.mpenv_debug_trace_rays(e.h, od.data_ptr(), dd.data_ptr(), n, mode, t.data_ptr(),
                                          h.data_ptr(), None) == 0
        res.append((t.cpu().numpy(), h.cpu().numpy()))
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][0], res[1][0])
    # oracle (reference order on the CPU) on a subset incl. all edge-aimed rays
    idx = np.concatenate([np.arange(0, 200000, 97), np.arange(200000, n)])
    for i in idx:
        tt = C.c_float(0)
        hit = o.lib.oracle_trace_ray(o.h, T.fptr(ro[i]), T.fptr(rd[i]), C.byref(tt))
        assert hit == res[1][1][i], i
        if hit:
            assert tt.value == res[1][0][i], (i, tt.value, res[1][0][i])


def test_world_groups_on_streams_match_oracle(monkeypatch):
    """Worlds split into 3 uneven groups stepped on concurrent streams
    (MPENV_WORLD_GROUPS) give the oracle's results for worlds at the group
    boundaries."""
    monkeypatch.setenv("MPENV_WORLD_GROUPS", "3")
    ts, W, steps = 2, 2050, 60
    N = 2 * ts
    e = T.Engine(W, ts, sim_flags=1)
    e.put_ctrl([0, 1, 1])
    e.init()
    probes = [0, 682, 683, 1366, 1367, W - 2]
    oracles = []
    for w0 in probes:
        o = T.Oracle(2, ts, sim_flags=1, world_id_offset=w0)
        o.put_ctrl([0, 1, 1])
        o.init()
        oracles.append(o)
    for s in range(steps):
        e.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, W * N))
        e.step()
        for w0, o in zip(probes, oracles):
            o.set_actions(T.mpenv_tape.tape_actions(1234, s, w0 * N, 2 * N))
            o.step()
        if s % 7 == 0 or s == steps - 1:
            for w0, o in zip(probes, oracles):
                for n in T.STEP_OUTPUTS:
                    _, _, shape = e.desc(n)
                    k = shape[0] // W
                    r0, r1 = w0 * k, (w0 + 2) * k
                    T.compare(e.get_rows(n, r0, r1), o.get(n), f"{n} worlds {w0}.. @ {s}")


def test_step_graph_captures_every_fork_layout(monkeypatch):
    """Round-4 review: a capture of the lidar branch stream crashed the
    process.  The capture is now checked (capture status before it ends,
    every capture call's return) and a failed one is abandoned for direct
    launches with the reason kept (mpenv_graph_status).  Here every fork
    layout is captured -- 1-4 world groups (4 is capped at 3), and one
    group with k_lidar on a branch stream beside k_vis -> k_obs -- and its
    replay must equal kernel-by-kernel launches bit for bit, with the graph
    on (no abandoned capture)."""
    import ctypes as C

    ts, W, steps = 3, 3000, 12
    N = 2 * ts
    monkeypatch.setenv("MPENV_STEP_GRAPH", "0")
    monkeypatch.setenv("MPENV_WORLD_GROUPS", "1")
    ref = T.Engine(W, ts)
    monkeypatch.setenv("MPENV_STEP_GRAPH", "1")
    layouts = [(1, False), (1, True), (2, False), (3, False), (4, False)]
    engines = []
    for groups, branch in layouts:
        e = T.Engine(W, ts)
        e.set_world_groups(groups)
        e.lib.mpenv_set_lidar_branch.argtypes = [C.c_void_p, C.c_int32]
        assert e.lib.mpenv_set_lidar_branch(e.h, int(branch)) == 0
        engines.append(e)
    for e in [ref] + engines:
        e.put_ctrl([0, 1, 1])
        e.init()
    for s in range(steps):
        acts = T.mpenv_tape.tape_actions(1234, s, 0, W * N)
        for e in [ref] + engines:
            e.set_actions(acts)
            e.step()
        if s % 4 == 3:
            for (groups, branch), e in zip(layouts, engines):
                for n in T.STEP_OUTPUTS:
                    T.compare(e.get(n), ref.get(n), f"{n} graph ({groups} groups, branch {branch}) vs direct @ {s}")
    for (groups, branch), e in zip(layouts, engines):
        on, why = C.c_int32(-1), C.create_string_buffer(512)
        e.lib.mpenv_graph_status.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_char_p, C.c_int32]
        assert e.lib.mpenv_graph_status(e.h, C.byref(on), why, 512) == 0
        assert on.value == 1 and why.value == b"", (groups, branch, why.value)
        n_cap = C.c_int64(-1)
        e.lib.mpenv_graph_captures.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
        assert e.lib.mpenv_graph_captures(e.h, C.byref(n_cap)) == 0 and n_cap.value == 1, (groups, branch, n_cap.value)
        e.close()
    ref.close()


def test_step_graph_replay_equals_direct_launches(monkeypatch):
    """The Step graph replayed as a captured HIP graph (the default) equals
    kernel-by-kernel launches (MPENV_STEP_GRAPH=0) bit for bit, including
    across re-captures: world groups 2 -> 3 -> 1 -> 2, the stats buffer
    switched on and off (kernel arguments change), and timed steps (which
    bypass the graph) in between; plus oracle slices at the group borders."""
    ts, W, steps = 3, 3000, 48
    N = 2 * ts
    monkeypatch.setenv("MPENV_WORLD_GROUPS", "2")
    monkeypatch.setenv("MPENV_STEP_GRAPH", "0")
    ref = T.Engine(W, ts)
    monkeypatch.setenv("MPENV_STEP_GRAPH", "1")
    g = T.Engine(W, ts)
    probes = [0, 999, 1499, 1999, W - 2]
    oracles = []
    for e in (ref, g):
        e.put_ctrl([0, 1, 1])
        e.init()
    for w0 in probes:
        o = T.Oracle(2, ts, world_id_offset=w0)
        o.put_ctrl([0, 1, 1])
        o.init()
        oracles.append(o)
    for s in range(steps):
        if s == 8:
            g.set_world_groups(3)
        elif s == 16:
            g.enable_stats(True)
        elif s == 20:
            g.enable_stats(False)
            g.set_world_groups(1)
        elif s == 28:
            g.set_world_groups(2)
        elif s == 34:
            assert g.lib.mpenv_enable_kernel_timing(g.h, 1) == 0
        elif s == 38:
            assert g.lib.mpenv_enable_kernel_timing(g.h, 0) == 0
        acts = T.mpenv_tape.tape_actions(1234, s, 0, W * N)
        for e in (ref, g):
            e.set_actions(acts)
            e.step()
        for w0, o in zip(probes, oracles):
            o.set_actions(T.mpenv_tape.tape_actions(1234, s, w0 * N, 2 * N))
            o.step()
        if s % 4 == 3:
            for n in T.STEP_OUTPUTS:
                T.compare(g.get(n), ref.get(n), f"{n} graph vs direct @ {s}")
            for w0, o in zip(probes, oracles):
                for n in T.STEP_OUTPUTS:
                    _, _, shape = g.desc(n)
                    k = shape[0] // W
                    T.compare(g.get_rows(n, w0 * k, (w0 + 2) * k), o.get(n), f"{n} worlds {w0}.. @ {s}")
    # one capture per argument change and none otherwise: steps 0 (first),
    # 8 (3 groups), 16 (stats on), 20 (stats off + 1 group), 28 (2 groups);
    # the timed steps 34-37 bypass the graph and 38 replays the step-28 graph
    import ctypes as C
    n_cap = C.c_int64(-1)
    g.lib.mpenv_graph_captures.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    assert g.lib.mpenv_graph_captures(g.h, C.byref(n_cap)) == 0
    assert n_cap.value == 5, n_cap.value
    # a re-capture right after an asynchronous launch (the previous exec may
    # still run): groups 2 -> 3 with no sync between, then both engines agree
    g.lib.mpenv_step_async.argtypes = [C.c_void_p, C.c_void_p]
    acts = T.mpenv_tape.tape_actions(1234, steps, 0, W * N)
    for e in (ref, g):
        e.set_actions(acts)
    ref.step()
    assert g.lib.mpenv_step_async(g.h, None) == 0
    g.set_world_groups(3)
    acts = T.mpenv_tape.tape_actions(1234, steps + 1, 0, W * N)
    for e in (ref, g):
        e.set_actions(acts)
        e.step()
    for n in T.STEP_OUTPUTS:
        T.compare(g.get(n), ref.get(n), f"{n} graph vs direct after an async re-capture")


def test_logs_record_and_events_match_oracle(tmp_path):
    """record_log_path + event_log_path: the engine's StepLog file,
    events.bin and steps.bin equal, byte for byte, what the oracle's buffers
    give for the same run (mgr.cpp:104-116, sim.cpp:23-106, 4750-4792)."""
    W, ts, steps = 12, 3, 250
    rec = str(tmp_path / "rec.bin")
    e = T.Engine(W, ts, sim_flags=1, record=rec, events=str(tmp_path))
    o = T.Oracle(W, ts, sim_flags=1)
    o.lib.oracle_set_log_modes(o.h, 1, 0, 1)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    exp_rec, exp_ev, exp_steps = [], [], []
    for s in range(steps):
        acts = T.combat_actions(o, s)
        e.set_actions(acts)
        o.set_actions(acts)
        e.step()
        o.step()
        exp_rec.append(o.get("RECORD_LOG").astype("<i4").tobytes())
        rows = o.get("EVENT_LOG").reshape(-1, 6)
        exp_ev.append(rows[rows[:, 0] != 0].astype("<i4").tobytes())
        sn, wr = o.get("PACKED_STEP_SNAPSHOT"), o.get("SNAPSHOT_WRITTEN").ravel()
        exp_steps.append(sn[wr != 0].astype("<i4").tobytes())
        if s % 25 == 0:
            _compare_all(e, o, f"step {s}")
    e.close()  # flushes the files
    got_rec = open(rec, "rb").read()
    assert got_rec == b"".join(exp_rec)
    got_ev = open(tmp_path / "events.bin", "rb").read()
    assert len(got_ev) > 24 * 20
    assert got_ev == b"".join(exp_ev)
    assert open(tmp_path / "steps.bin", "rb").read() == b"".join(exp_steps)


def test_logs_replay_matches_oracle(tmp_path):
    """replay_log_path: the engine replays a recorded match (pvpReplayLogic)
    exactly as the oracle does from the same StepLogs."""
    W, ts, steps = 8, 2, 200
    rec = str(tmp_path / "rec.bin")
    src = T.Engine(W, ts, sim_flags=1, record=rec)
    src.put_ctrl([0, 1, 1])
    src.init()
    for s in range(steps):
        src.set_actions(T.mpenv_tape.tape_actions(1234, s, 0, W * 2 * ts))
        src.step()
    src.close()
    logs = np.fromfile(rec, dtype=np.int32).reshape(steps, W, 217)
    e = T.Engine(W, ts, sim_flags=1, replay=rec)
    o = T.Oracle(W, ts, sim_flags=1)
    o.lib.oracle_set_log_modes(o.h, 0, 1, 0)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    zero = np.zeros((W * 2 * ts, 6), np.int32)
    for s in range(steps):
        o.view("REPLAY_LOG")[:] = logs[s]
        for sim in (e, o):
            sim.set_actions(zero)
            sim.step()
        _compare_all(e, o, f"replay step {s}")
    fin = C.c_int32(0)
    assert e.lib.mpenv_is_replay_finished(e.h, C.byref(fin)) == 0 and fin.value == 1
