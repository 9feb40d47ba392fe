"""Generate tests/golden/*.json: per-step state hashes of oracle rollouts.

SURVEY.md §8c: the reference cannot be built or imported here, so golden
vectors come from the CPU restatement (oracle/) in this container.  Each
fixture records a config, the action tape seed, and for every step the
sha256 of every compared export (tests/mpenv_testlib.py STEP_OUTPUTS +
DEBUG_OUTPUTS), plus a few float tensors of the final step in full.  The
GPU parity tests check the engine against these files as well as against a
live oracle run.

Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import mpenv_testlib as T  # noqa: E402

CASES = {
    "1v1_w2": dict(team_size=1, worlds=2, steps=200, sim_flags=0, ctrl=[0, 1, 1]),
    "3v3_w2": dict(team_size=3, worlds=2, steps=200, sim_flags=0, ctrl=[0, 1, 1]),
    "6v6_w2": dict(team_size=6, worlds=2, steps=200, sim_flags=0, ctrl=[0, 1, 1]),
    # RandomizeHPMagazine | NoRespawn | StaggerStarts, no auto flip
    "2v2_flags": dict(team_size=2, worlds=3, steps=150, sim_flags=(1 << 1) | (1 << 3) | (1 << 4),
                      ctrl=[0, 0, 0]),
    # SpawnInMiddle (+ RandomizeHPMagazine) with the aim-bot action source:
    # contact, kills, respawns, combat rewards
    "3v3_mid_combat": dict(team_size=3, worlds=4, steps=300, sim_flags=1 | (1 << 1), ctrl=[0, 1, 1],
                           policy="combat"),
    "6v6_mid_combat": dict(team_size=6, worlds=2, steps=300, sim_flags=1, ctrl=[0, 1, 1],
                           policy="combat"),
    # team 1 as A* bots (AgentPolicy = -1, planAStarAISystem)
    "3v3_bots": dict(team_size=3, worlds=3, steps=250, sim_flags=1, ctrl=[0, 1, 1], bots="team1"),
    # HardcodedSpawns | SpawnInMiddle | RandomizeHPMagazine, random team sides
    "3v3_hardcoded": dict(team_size=3, worlds=3, steps=200, sim_flags=1 | 2 | (1 << 6), ctrl=[0, 1, 1],
                          policy="combat"),
    # SubZones | SpawnInMiddle with policies cycling over the sub-zones
    "3v3_subzones": dict(team_size=3, worlds=4, steps=250, sim_flags=1 | (1 << 11), ctrl=[0, 1, 1],
                         policy="combat", bots="cycle"),
    # ZoneCaptureDefend as scripts/jax_train.py configures it (HardcodedSpawns,
    # StaggerStarts, RandomFlipTeams), 6v6 on a four-zone scene
    "6v6_capture_defend": dict(team_size=6, worlds=3, steps=300, sim_flags=1 | (1 << 6) | (1 << 4),
                               ctrl=[0, 1, 1], policy="combat", task=T.TASK_ZONE_CAPTURE_DEFEND,
                               scene="four_zones"),
    # NavmeshSpawn | EnableCurriculum (LearnShooting rewards)
    "2v2_navmesh_curriculum": dict(team_size=2, worlds=4, steps=200, sim_flags=(1 << 2) | (1 << 5),
                                   ctrl=[0, 1, 1], policy="combat"),
}
TAPE_SEED = 1234
_SCENES = {}


def make_sim(cls, case):
    """T.Oracle or T.Engine for a case (task and scene are optional keys;
    scene "four_zones" is simple_map plus a fourth zone, generated on first
    use)."""
    kw = dict(sim_flags=case["sim_flags"], task=case.get("task", T.TASK_ZONE))
    if case.get("scene") == "four_zones":
        if "four_zones" not in _SCENES:
            import tempfile
            _SCENES["four_zones"] = T.four_zone_scene(tempfile.mkdtemp(prefix="mpenv_scene_"))
        kw["scene"] = _SCENES["four_zones"]
    return cls(case["worlds"], case["team_size"], **kw)
FINAL_TENSORS = ["SELF_OBSERVATION", "REWARD", "HP", "FWD_LIDAR"]


def step_hashes(sim):
    h = {}
    for name in T.STEP_OUTPUTS + T.DEBUG_OUTPUTS:
        h[name] = hashlib.sha256(np.ascontiguousarray(sim.get(name)).tobytes()).hexdigest()[:16]
    return h


def rollout(sim, case, record=None):
    """Drive an Oracle or Engine through a case; yields (step, sim)."""
    sim.put_ctrl(np.array(case["ctrl"], np.int32))
    A = case["worlds"] * 2 * case["team_size"]
    sim.init()
    if case.get("bots"):
        set_bots(sim, case)
    yield -1
    for s in range(case["steps"]):
        if case.get("policy") == "combat":
            sim.set_actions(T.combat_actions(sim, s, TAPE_SEED))
        else:
            sim.set_actions(T.mpenv_tape.tape_actions(TAPE_SEED, s, 0, A))
        sim.step()
        yield s


def set_bots(sim, case):
    """AgentPolicy = -1 (consts::aStarPolicyID) for team 1 ("team1") or
    everyone ("all"); "cycle" assigns (agent % 10) - 1, i.e. -1 (bot) .. 8,
    which SubZones clamps to sub-zones 0..7."""
    W, ts = case["worlds"], case["team_size"]
    pol = np.zeros((W, 2, ts), np.int32)
    if case["bots"] == "all":
        pol[:] = -1
    elif case["bots"] == "cycle":
        pol = (np.arange(W * 2 * ts, dtype=np.int32) % 10) - 1
    else:
        pol[:, 1, :] = -1
    if hasattr(sim, "view"):
        sim.view("AGENT_POLICY")[:] = pol.reshape(-1, 1)
    else:
        sim.put("AGENT_POLICY", pol.reshape(-1, 1))


def make(name, case):
    o = make_sim(T.Oracle, case)
    hashes = []
    for _ in rollout(o, case):
        hashes.append(step_hashes(o))
    final = {n: o.get(n).ravel().tolist() for n in FINAL_TENSORS}
    o.close()
    return dict(case=case, tape_seed=TAPE_SEED, hashes=hashes, final=final)


if __name__ == "__main__":
    for name, case in CASES.items():
        out = make(name, case)
        path = os.path.join(HERE, f"{name}.json")
        with open(path, "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print(path, os.path.getsize(path))
