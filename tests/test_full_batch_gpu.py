"""Whole-batch parity at the benchmark configurations.

* Every world of the driver's timed regime: the C3 batch (6v6 x 16,384
  worlds) and the C2 batch (3v3 x 4,096), stepped exactly as bench.py steps
  them (Manager::init with simCtrl [0, 1, 1], the hash tape copied each step
  from a 64-step ring resident in HBM, two world groups on concurrent
  streams), against the oracle over the SAME batch (oracle_run_threaded, the
  restatement of the reference's ThreadPoolExecutor path, worlds partitioned
  over the usable CPUs) -- every STEP_OUTPUT and internal-state export of
  every world, bit-exact.
* Config C4 on one GPU: the eight 16,384-world shards of 131,072 worlds
  (world_id_offset r·16,384, ≈49 GB of HBM), team 1 of every even global
  world an A* bot (C5's nav-mesh pathing), everyone else the zone-seeking
  aim-bot over the global tape; oracle slices straddling every shard boundary
  compared every 25 steps; the outputs then assembled through the learner
  exchange's flat layout (mpenv_dist) in global world order.
* Config C5's loop on one GPU: team 1 A* bots in every world, team 0 driven
  by bench.py's policy MLP reading the previous step's observations; oracle
  slices fed the same policy actions.
"""
import time

import numpy as np
import pytest

import mpenv_testlib as T

pytestmark = pytest.mark.gpu

RING = 64
SEED = 1234
ALL = T.STEP_OUTPUTS + T.DEBUG_OUTPUTS

FULL = [
    # team_size, worlds, warmup, timed steps, compare every
    (6, 16384, 5, 20, 5),     # C3: the driver's window (5 warmup + 20 timed)
    (3, 4096, 5, 300, 25),    # C2
]


@pytest.mark.parametrize("ts,W,warmup,steps,every", FULL, ids=["C3_6v6x16384", "C2_3v3x4096"])
def test_every_world_of_the_bench_window_matches_oracle(ts, W, warmup, steps, every):
    t_start = time.time()
    N = 2 * ts
    A = W * N
    e = T.Engine(W, ts)
    e.set_world_groups(1)  # as bench.py's timed pass (multi-group parity: test_parity_gpu)
    o = T.Oracle(W, ts)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    ring = T.mpenv_tape.tape_ring(SEED, 0, A, RING)
    dev_ring = e.mem.upload(ring)
    threads = T.usable_cpus()

    def compare_all(where):
        for n in ALL:
            T.compare(e.get(n), o.get(n), f"{n} @ {where}")

    compare_all("init")
    t_oracle = 0.0
    total = warmup + steps
    for s in range(total):
        row = np.ascontiguousarray(ring[s % RING])
        e.copy_actions(dev_ring + (s % RING) * A * 24)
        e.step()
        t_oracle += o.lib.oracle_run_threaded(o.h, 1, threads, row.ctypes.data, 1)
        if (s + 1) % every == 0 or s == total - 1:
            compare_all(f"step {s}")
        else:
            for n in ("REWARD", "DONE", "HP", "SELF_OBSERVATION"):
                T.compare(e.get(n), o.get(n), f"{n} @ step {s}")
    e.mem.free(dev_ring)
    if W * N <= 65536:  # the expanded grid is 26 KB per agent on each side
        T.compare(T.explore_visited(e), T.explore_visited(o), "explore cells @ end")
    alive = o.get("ALIVE")
    print(f"\n{ts}v{ts} x {W}: {total} steps, every world compared ({len(ALL)} exports every {every} steps); "
          f"oracle {t_oracle:.1f} s on {threads} threads, test {time.time() - t_start:.1f} s, "
          f"alive {alive.mean():.3f}")
    e.close()
    o.close()


LIDAR_EXPORTS = ("FWD_LIDAR", "REAR_LIDAR", "FULL_TEAM_FWD_LIDAR", "FULL_TEAM_REAR_LIDAR")


def compare_lidar_ulp(a, b, name):
    """Lidar rows [..., 4] (depth, wall, teammate, opponent): the three class
    channels byte-exact, the depth within one ulp (same sign, bit patterns
    at most 1 apart).  Returns the number of rays whose depth differs."""
    assert a.shape == b.shape and a.shape[-1] == 4, (name, a.shape, b.shape)
    T.compare(np.ascontiguousarray(a[..., 1:]), np.ascontiguousarray(b[..., 1:]), f"{name} (class channels)")
    da = np.ascontiguousarray(a[..., 0]).view(np.int32).astype(np.int64)
    db = np.ascontiguousarray(b[..., 0]).view(np.int32).astype(np.int64)
    diff = np.abs(da - db)
    same_sign = (da < 0) == (db < 0)
    bad = ~same_sign | (diff > 1)
    assert not bad.any(), f"{name}: {int(bad.sum())} depths beyond 1 ulp, first at {tuple(np.argwhere(bad)[0])}"
    return int((diff == 1).sum())


def test_bench_window_every_world_against_the_reference_slot_order():
    """The product's lidar walks each node's children in a per-octant order
    (DESIGN.md §2 definition 12); the reference walks them in slot order
    (mesh_bvh.inl:160-204).  Against an oracle built with the reference's
    slot order, over every world of the driver's C3 window (Manager::init,
    5 warm-up + 20 timed steps of the tape -- no bots, so lidar depth never
    feeds back into the state): every export byte-exact except the lidar
    depths, which may differ by one ulp where two coplanar triangles tie
    (class channels exact).  The count of 1-ulp rays is printed; the north
    star allows 1e-5 relative."""
    t_start = time.time()
    ts, W, total = 6, 16384, 25
    N = 2 * ts
    A = W * N
    e = T.Engine(W, ts)
    e.set_world_groups(1)
    o = T.Oracle(W, ts, lidar_order="slot")
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    ring = T.mpenv_tape.tape_ring(SEED, 0, A, RING)
    dev_ring = e.mem.upload(ring)
    threads = T.usable_cpus()
    ulp_rays, checked = 0, 0

    def compare_all(where):
        nonlocal ulp_rays, checked
        for n in ALL:
            if n in LIDAR_EXPORTS:
                a = e.get(n)
                ulp_rays += compare_lidar_ulp(a, o.get(n), f"{n} @ {where}")
                checked += a.size // 4
            else:
                T.compare(e.get(n), o.get(n), f"{n} @ {where}")

    compare_all("init")
    for s in range(total):
        row = np.ascontiguousarray(ring[s % RING])
        e.copy_actions(dev_ring + (s % RING) * A * 24)
        e.step()
        o.lib.oracle_run_threaded(o.h, 1, threads, row.ctypes.data, 1)
        if (s + 1) % 5 == 0 or s == total - 1:
            compare_all(f"step {s}")
    e.mem.free(dev_ring)
    print(f"\nC3 6v6 x {W}, init + {total} steps vs the reference's slot-order traversal: every export "
          f"byte-exact but lidar depth; {ulp_rays} of {checked} lidar rays compared differ by 1 ulp "
          f"({ulp_rays / max(checked, 1):.2e}); test {time.time() - t_start:.1f} s")
    e.close()
    o.close()


COMBAT = [
    # team_size, worlds, steps, compare every, kills required (C3's teams
    # first meet near the zone: 120 steps see ~25 agents hit and no kill
    # yet; C2's 300 steps ~700 kills)
    (6, 16384, 120, 20, False),   # C3
    (3, 4096, 300, 25, True),     # C2
]


@pytest.mark.parametrize("ts,W,steps,every,need_kills", COMBAT, ids=["C3_6v6x16384", "C2_3v3x4096"])
def test_every_world_in_the_combat_regime_matches_oracle(ts, W, steps, every, need_kills):
    """bench.py --actions combat, world by world: every step the device
    aim-bot (mpenv_combat_actions mode 1: fire at the first visible
    opponent, else turn and run toward the zone, reload an empty magazine)
    rewrites the tape row from the engine's observations; the same actions
    must come out of its numpy twin (seek_combat_actions) over the ORACLE's
    observations, and the oracle then steps the whole batch with them.  Every
    STEP_OUTPUT and debug export of every world is compared byte for byte
    (floats by bit pattern), so respawn scoring (utils.cpp:734-948), kill
    bookkeeping and last-known updates are checked at full batch."""
    t_start = time.time()
    N = 2 * ts
    A = W * N
    e = T.Engine(W, ts)
    e.set_world_groups(1)  # as bench.py's timed pass (multi-group parity: test_parity_gpu)
    o = T.Oracle(W, ts)
    for sim in (e, o):
        sim.put_ctrl([0, 1, 1])
        sim.init()
    ring = T.mpenv_tape.tape_ring(SEED, 0, A, RING)
    dev_ring = e.mem.upload(ring)
    dev_acts = e.mem.upload(np.zeros((A, 6), np.int32))
    threads = T.usable_cpus()
    e.enable_stats(True)

    def compare_all(where):
        for n in ALL:
            T.compare(e.get(n), o.get(n), f"{n} @ {where}")

    compare_all("init")
    t_oracle = 0.0
    acts = np.empty((A, 6), np.int32)
    for s in range(steps):
        if s % 5 == 0:  # progress (a long GPU test must not look hung)
            print(f"  step {s}: oracle {t_oracle:.0f} s, test {time.time() - t_start:.0f} s", flush=True)
        e.combat_actions(dev_ring + (s % RING) * A * 24, dev_acts, 1)
        e.mem.d2h(dev_acts, acts.nbytes, acts)
        twin = T.seek_combat_actions(o, s, base=ring[s % RING])
        T.compare(acts, twin, f"combat actions @ step {s}")
        e.copy_actions(dev_acts)
        e.step()
        t_oracle += o.lib.oracle_run_threaded(o.h, 1, threads, twin.ctypes.data, 1)
        if (s + 1) % every == 0 or s == steps - 1:
            compare_all(f"step {s}")
        else:
            for n in ("REWARD", "DONE", "HP", "ALIVE", "SELF_OBSERVATION"):
                T.compare(e.get(n), o.get(n), f"{n} @ step {s}")
    st = e.read_stats()
    e.mem.free(dev_ring)
    e.mem.free(dev_acts)
    print(f"\n{ts}v{ts} x {W} combat: {steps} steps, every world compared ({len(ALL)} exports every {every} "
          f"steps); {st['shot_rays']} shots, {st['hit_agents']} agents hit, {st['kills']} kills; oracle "
          f"{t_oracle:.1f} s on {threads} threads, test {time.time() - t_start:.1f} s")
    assert st["hit_agents"] > 0 and st["shot_rays"] > 0
    if need_kills:
        assert st["kills"] > 0
    e.close()
    o.close()


C4_SHARDS, C4_WORLDS, C4_TS, C4_STEPS = 8, 16384, 6, 300


def test_c4_shards_on_one_gpu_match_oracle_across_boundaries():
    import torch

    import madrona_mp_env as m
    from mpenv_dist import NOT_SHIPPED, flat_layout, pack_flat, unpack_flat

    R, W, ts = C4_SHARDS, C4_WORLDS, C4_TS
    N = 2 * ts
    A = W * N
    t_start = time.time()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    sims, rings, outs = [], [], []

    def policies(first_world, count):
        # team 1 of every even GLOBAL world is an A* bot (AgentPolicy -1)
        pol = np.zeros((count, 2, ts), np.int32)
        glob = np.arange(first_world, first_world + count)
        pol[glob % 2 == 0, 1, :] = -1
        return pol.reshape(-1, 1)

    for r in range(R):
        sim = m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                           auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                           team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE,
                           world_id_offset=r * W)
        ctrl = sim.sim_control_tensor().to_torch()
        ctrl.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device=dev).view_as(ctrl))
        torch.cuda.synchronize()
        sim.init()
        sim.policy_assignment_tensor().to_torch().copy_(torch.from_numpy(policies(r * W, W)).to(dev))
        torch.cuda.synchronize()
        sims.append(sim)
        rings.append(torch.from_numpy(T.mpenv_tape.tape_ring(SEED, r * A, A, RING)).to(dev))
        outs.append({n: t.to_torch() for n, t in sim.train_interface()["outputs"].items()
                     if n not in NOT_SHIPPED})
    assert set(outs[0]) == set(T.TRAIN_OUTPUTS)

    # oracle slices: the first two and last two worlds of the job, and
    # worlds r·W-2 .. r·W+1 across every shard boundary
    slices = [(0, 2)] + [(r * W - 2, 4) for r in range(1, R)] + [(R * W - 2, 2)]
    oracles = []
    for g0, nw in slices:
        o = T.Oracle(nw, ts, world_id_offset=g0)
        o.put_ctrl([0, 1, 1])
        o.init()
        o.view("AGENT_POLICY")[:] = policies(g0, nw)
        oracles.append(o)

    def engine_rows(name, g0, nw):
        parts = []
        for g in range(g0, g0 + nw):
            r, w = divmod(g, W)
            t = outs[r][name]
            rpw = t.shape[0] // W
            parts.append(t[w * rpw:(w + 1) * rpw].cpu().numpy())
        return np.concatenate(parts)

    def compare(where):
        torch.cuda.synchronize()
        for (g0, nw), o in zip(slices, oracles):
            for n, ex in T.TRAIN_OUTPUTS.items():
                T.compare(engine_rows(n, g0, nw), o.get(ex).reshape((-1,) + tuple(outs[0][n].shape[1:])),
                          f"{n} worlds {g0}.. @ {where}")

    compare("init")
    for sim in sims:
        sim.enable_stats(True)
    for s in range(C4_STEPS):
        for r in range(R):
            sims[r].combat_actions(rings[r][s % RING].data_ptr(), 0, 1, sptr)
            sims[r].step_async(sptr)
        for (g0, nw), o in zip(slices, oracles):
            base = T.mpenv_tape.tape_actions(SEED, s % RING, g0 * N, nw * N)
            o.set_actions(T.seek_combat_actions(o, s, base=base))
            o.step()
        if s % 25 == 24:
            compare(f"step {s}")
    torch.cuda.synchronize()
    kills = sum(sim.read_stats()["kills"] for sim in sims)

    # the learner exchange's layout: each shard's outputs packed into its row
    # of a [ranks, bytes] receive buffer, read back as [ranks, rows, ...]
    layout, nbytes = flat_layout(outs[0])
    recv = torch.empty((R, nbytes), dtype=torch.uint8, device=dev)
    for r in range(R):
        pack_flat(layout, [outs[r][n] for n, *_ in layout], recv[r])
    views = unpack_flat(layout, recv)
    torch.cuda.synchronize()
    for n, *_ in layout:
        for r in range(R):
            assert torch.equal(views[n][r], outs[r][n]), (n, r)
    for (g0, nw), o in zip(slices, oracles):
        for n, ex in T.TRAIN_OUTPUTS.items():
            v = views[n]
            rpw = v.shape[1] // W
            flat = v.reshape((-1,) + tuple(v.shape[2:]))
            T.compare(flat[g0 * rpw:(g0 + nw) * rpw].cpu().numpy(), o.get(ex).reshape((-1,) + tuple(v.shape[2:])),
                      f"gathered {n} worlds {g0}..")
    hp = torch.cat([outs[r]["hp"] for r in range(R)])
    assert bool(((hp >= 0) & (hp <= 100)).all())
    print(f"\nC4 on one GPU: {R} shards x {W} worlds {ts}v{ts}, {C4_STEPS} steps, {len(slices)} boundary "
          f"slices bit-exact every 25 steps; {kills} kills in the whole job; gathered layout {nbytes / 1e6:.1f} MB per rank; test {time.time() - t_start:.1f} s")
    assert kills > 0
    for o in oracles:
        o.close()


def test_c5_policy_loop_with_bots_matches_oracle():
    """Config C5's shape on one GPU: 6v6 x 16,384 worlds, team 1 of every
    world an A* bot (AgentPolicy -1, planAStarAISystem over the nav mesh),
    team 0 driven by a closed policy loop -- bench.py's random-init bf16 MLP
    reads every trainInterface observation of the previous step and its
    argmax actions are the next step's inputs (the engine side of the
    jax_train self-play loop; JAX itself is absent from the image).  Oracle
    slices of the same global worlds are fed the very actions the policy
    produced and compared on every trainInterface output every 25 steps."""
    import sys

    import torch

    import madrona_mp_env as m

    sys.path.insert(0, T.ROOT)
    from bench import make_policy

    W, ts, steps = 16384, 6, 300
    N = 2 * ts
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sim = m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=0, num_worlds=W, rand_seed=5,
                       auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                       team_size=ts, num_pbt_policies=0, policy_history_size=0, scene_path=T.SCENE)
    ctrl = sim.sim_control_tensor().to_torch()
    ctrl.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device=dev).view_as(ctrl))
    torch.cuda.synchronize()
    sim.init()
    pol = np.zeros((W, 2, ts), np.int32)
    pol[:, 1, :] = -1
    sim.policy_assignment_tensor().to_torch().copy_(torch.from_numpy(pol.reshape(-1, 1)).to(dev))
    torch.cuda.synchronize()
    policy = make_policy(sim, 512, dev)
    outs = {n: t.to_torch() for n, t in sim.train_interface()["outputs"].items()}
    slices = [(0, 3), (5000, 3), (W - 3, 3)]
    oracles = []
    for g0, nw in slices:
        o = T.Oracle(nw, ts, world_id_offset=g0)
        o.put_ctrl([0, 1, 1])
        o.init()
        o.view("AGENT_POLICY")[:] = pol[g0:g0 + nw].reshape(-1, 1)
        oracles.append(o)
    sim.enable_stats(True)
    for s in range(steps):
        ptr = policy()
        sim.copy_actions(ptr, stream.cuda_stream)
        sim.step_async(stream.cuda_stream)
        for (g0, nw), o in zip(slices, oracles):
            o.set_actions(policy.actions[g0 * N:(g0 + nw) * N].cpu().numpy())
            o.step()
        if s % 25 == 24:
            for (g0, nw), o in zip(slices, oracles):
                for n, ex in T.TRAIN_OUTPUTS.items():
                    t = outs[n]
                    rpw = t.shape[0] // W
                    T.compare(t[g0 * rpw:(g0 + nw) * rpw].cpu().numpy(),
                              o.get(ex).reshape((-1,) + tuple(t.shape[1:])), f"{n} worlds {g0}.. @ {s}")
    torch.cuda.synchronize()
    st = sim.read_stats()
    print(f"\nC5 loop on one GPU: {W} worlds {ts}v{ts}, {steps} policy steps, team 1 A* bots; "
          f"{len(slices)} slices bit-exact every 25 steps; pairs seen {st['los_seen']}, shots {st['shot_rays']}, "
          f"hits {st['hit_agents']}, kills {st['kills']}")
    assert st["los_seen"] > 0 and st["shot_rays"] > 0  # the bots see and fire on the policy team
    for o in oracles:
        o.close()
