"""Headline benchmark: agent-steps/s of the world-batched Zone step.

Metric (BASELINE.json): env steps/sec x agents, simple_map 6v6 @ 16384 worlds
per GPU (config C3 at N=1; C4 = 8 x 16384 worlds sharded one process per
GPU, weak scaling).  One "step" = one full Step graph (sim.cpp:5299-5320
setupStepTasks, Task::Zone) over every world of the rank, preceded by the
TrainInterface input copy of gpuStreamStep (mgr.cpp:625): the actions of
step s are copied device-to-device from a 64-step ring of synthetic action
tapes resident in HBM.  Inputs are resident before the timed
region; nothing is skipped inside it.

Also reported (one JSON line on rank 0):
  roofline     -- dominant kernel's algorithmic HBM bytes / its average
                  duration (HIP events on the engine's stream, timed
                  region), against the 8 TB/s HBM3E peak; `traffic` = PMC
                  HBM bytes per launch from profiles/ when a matching
                  rocprofv3 --pmc summary exists (else null).
  cpu_baseline -- the CPU oracle (a restatement of the reference's
                  ThreadPoolExecutor path, oracle/) timed on this host on a
                  bounded sample of the same workload, rank 0, N=1 only.

Launch: python bench.py [--gpus 1 --steps 1000 --warmup 100]
        N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "madrona-mp-env_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md §HBM)
RING = 64
TAPE_SEED = 1234

# Algorithmic HBM bytes per agent-step for each kernel: the
# unique bytes the kernel must read or write, no re-reads counted.
#   k_move : actions 24 r; 20 movement columns (pos, vel, rot, aim yaw/pitch/
#            quat, pose x3, maxVel, aim velocities) x 4 B r+w (160)  = 184
#   k_sim  : 20 combat/bookkeeping columns r+w (160); pos/rot/alive r (32);
#            DamageDealt 6 x 4 r+w (48); hp/magazine r+w (24); reward+done
#            w (8); explore tile cache (tile, 64-bit word) r+w (24);
#            rewardCoefs r (4)                                      = 300
#   k_vis  : pos 12 + aim rot 16 + pose 4 + alive 4 r; mask w 1   = 37
#   k_obs  : state r ~124; self 172 + teammates 640 + opponents 768 w;
#            positions 12+60+72 w; masks 24 + filters 4 w; vis 1 r;
#            full-team player 112 + enemy 132 + last-known 96 w  = 2213,
#            plus 140 B (a 128-B row + its 12-B position) per last-known row
#            written (when the team knows the opponent, or it died), counted
#            per step by the workload counter lk_rows (rounds 1-3 charged
#            every row every step, read and written: 3,893 B)
#   k_lidar: pos 12 + rot 16 + aim rot 16 + pose 4 r; 80 rays x 16 B w;
#            previous rays 80 x 16 B r + full-team copy 80 x 16 B w = 3888
# plus per world-step: 32 singleton columns x 4 B r+w (256), full-team
# reward/done 16 w and the live breadcrumbs r+w (32 B each; 18.8 per world
# at steady state under the tape, oracle rollout of 256 worlds, steps
# 100-1100: 1,203 B) in k_sim; full-team global 2 x 64 w in k_obs.
KERNEL_BYTES_PER_AGENT = {"k_move": 184, "k_sim": 300, "k_vis": 37, "k_obs": 2213, "k_lidar": 3888}
LK_ROW_BYTES = 140  # k_obs, per last-known row written (counter lk_rows)
KERNEL_BYTES_PER_WORLD = {"k_move": 0, "k_sim": 1475, "k_vis": 0, "k_obs": 128, "k_lidar": 0}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--worlds", type=int, default=16384, help="worlds per GPU")
    ap.add_argument("--team-size", type=int, default=6)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "simple_map"))
    ap.add_argument("--world-groups", type=int, default=1,
                    help="world ranges stepped on concurrent streams in the timed pass (engine option); "
                         "the profile pass always runs one group so kernel times are exclusive")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline timed budget")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the CPUs this process may use")
    ap.add_argument("--exchange", choices=["auto", "none", "gather", "wire", "local"], default="auto",
                    help="learner exchange over RCCL (named in config.parallelism): wire = every "
                         "trainInterface output to rank 0 each step in the compact wire format, rebuilt "
                         "there bit for bit (config C4 as named; the default for N>1; at N=1 a loopback: "
                         "pack + unpack into a shadow on the same GPU); gather = the same outputs as "
                         "exported (3,924 B per agent); local = each rank's learner keeps its shard, a "
                         "gradient-sized all-reduce every --update-every steps; none = simulators only "
                         "(the default at N=1)")
    ap.add_argument("--gather", action="store_true", help="alias of --exchange gather")
    ap.add_argument("--grad-mb", type=float, default=16.0, help="local exchange: all-reduced gradient MB")
    ap.add_argument("--update-every", type=int, default=50,
                    help="local exchange: steps per policy update (jax_train.py --steps-per-update)")
    ap.add_argument("--actions", choices=["tape", "combat", "policy"], default="tape",
                    help="tape = the hash action tape (headline); combat = the tape overridden on the "
                         "device by the zone-seeking aim-bot (mpenv_combat_actions mode 1), so agents "
                         "meet, fight, die and respawn inside the timed window; policy = a closed "
                         "loop: a random-init bf16 MLP reads every trainInterface observation each step "
                         "and its argmax actions are the next step inputs (the env side of a "
                         "jax_train-style self-play loop; the policy forward is inside the timed window)")
    ap.add_argument("--path", choices=["step", "stream"], default="step",
                    help="step = copy_actions + step_async (the headline: outputs stay in the engine's "
                         "zero-copy tensors); stream = Manager::gpuStreamStep (mgr.cpp:614-645), the XLA "
                         "custom-call path of scripts/jax_train.py: every trainInterface input copied from "
                         "caller buffers, the step, every output copied into caller buffers")
    ap.add_argument("--policy-hidden", type=int, default=512, help="policy MLP width (--actions policy)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--learner-dedicated", choices=["auto", "on", "off"], default="auto",
                    help="--exchange wire at N > 1: rank 0 is a learner that simulates nothing -- it only "
                         "receives and unpacks ranks 1..N-1's messages into their shadows (C4 as 7 "
                         "simulators + 1 learner); value counts the simulator ranks' agent-steps.  auto: "
                         "from 4 ranks up (below that a learner that also simulates carries more)")
    ap.add_argument("--share-device", action="store_true",
                    help="debug: map every rank to GPU 0 (rehearse N>1 on a one-GPU box; no --gather)")
    ap.add_argument("--wire-serial", action="store_true",
                    help="--exchange wire: the learner unpacks on the step stream (back to back with its own "
                         "step) instead of its own unpack stream")
    ap.add_argument("--no-profile-pass", action="store_true",
                    help="skip the second (kernel-timing + workload-counter) pass")
    ap.add_argument("--bots", choices=["none", "team1", "all"], default="none",
                    help="A* scripted bots (AgentPolicy -1, planAStarAISystem) for team 1 / everyone "
                         "(config C5's nav-mesh pathing); the headline C3 line uses none")
    return ap.parse_args()


def cpu_share():
    """CPUs this process may use: affinity, capped by a cgroup v2 CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args):
    """Oracle (test infrastructure, a restatement of the reference's CPU
    executor, whose ThreadPoolExecutor partitions worlds over threads,
    mgr.cpp:1863-1871) on the same batch as the GPU line: every world of the
    configuration, one std::thread per usable CPU, steps until
    --cpu-seconds elapse (at least 2 after 1 untimed)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import mpenv_testlib as T

    threads = args.cpu_threads or cpu_share()
    W = args.worlds
    N = 2 * args.team_size
    A = W * N
    o = T.Oracle(W, args.team_size, scene=args.scene)
    o.put_ctrl([0, 1, 1])
    o.init()
    ring_len = 8
    ring = np.ascontiguousarray(T.mpenv_tape.tape_ring(TAPE_SEED, 0, A, ring_len))
    row = A * 6 * 4
    o.lib.oracle_run_threaded(o.h, 1, threads, ring.ctypes.data, 1)
    secs, steps = 0.0, 0
    while (secs < args.cpu_seconds or steps < 2) and steps < 1000:
        s = 1 + steps
        secs += o.lib.oracle_run_threaded(o.h, 1, threads, ring.ctypes.data + (s % ring_len) * row, 1)
        steps += 1
    o.close()
    return {
        "value": A * steps / secs,
        "unit": "agent-steps/s",
        "cores": threads,
        "kind": "port",
        "host_cpus": os.cpu_count(),
        "sample": f"the GPU line's batch ({W} worlds {args.team_size}v{args.team_size} simple_map), "
                  f"{steps} steps after 1 untimed, {threads} std::threads (static world partition; "
                  f"{threads} = CPUs usable by this process, of {os.cpu_count()} on the host), {secs:.1f} s",
    }


VALU_PEAK = 256 * 4 * 0.5 * 2.4e9  # wave-instr/s: 256 CUs x 4 SIMD32 x 1/2 per clock x 2.4 GHz
# What bounds each kernel: the ray kernels issue VALU
# instructions over divergent traversals; k_obs streams observation rows.
KERNEL_BOUND = {"k_move": "valu", "k_sim": "latency", "k_vis": "valu", "k_obs": "hbm", "k_lidar": "valu"}


def load_profile(path, workload):
    """profiles/pmc_traffic.json (tools/pmc_summary.py) if it was collected
    on this workload: HBM bytes and VALU instructions per launch per kernel."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    if "workloads" in d:
        e = d["workloads"].get(workload, {})
        return dict(e, by_window=e.get("by_window", {}))
    return d if d.get("workload") == workload else {}


# Action heads of the discrete policy (PvPDiscreteAction + discrete aim,
# jax_policy.py actions_config): move amount, move angle, fire, stand, yaw, pitch.
POLICY_HEADS = (3, 8, 3, 3, 13, 7)


def make_policy(sim, hidden, dev):
    """A random-init two-layer bf16 MLP over every observation tensor of the
    trainInterface (jax_policy.py's encoder widths, no LSTM), one argmax per
    action head.  Returns a callable that runs it on the engine's current
    outputs (zero-copy views) and returns the device pointer of an [A][6]
    int32 action buffer for copy_actions."""
    import torch

    outs = sim.train_interface()["outputs"]
    names = ["self", "teammates", "opponents", "opponents_last_known", "self_pos", "teammate_positions",
             "opponent_positions", "opponent_last_known_positions", "opponent_masks", "fwd_lidar",
             "rear_lidar", "hp", "magazine", "alive", "filters_state"]
    views = [outs[n].to_torch() for n in names]
    A = views[0].shape[0]
    flat = [v.reshape(A, -1) for v in views]
    width = sum(v.shape[1] for v in flat)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    w1 = (torch.randn(width, hidden, device=dev, generator=g) / width ** 0.5).to(torch.bfloat16)
    w2 = (torch.randn(hidden, hidden, device=dev, generator=g) / hidden ** 0.5).to(torch.bfloat16)
    wh = (torch.randn(hidden, sum(POLICY_HEADS), device=dev, generator=g) / hidden ** 0.5).to(torch.bfloat16)
    x = torch.empty(A, width, dtype=torch.bfloat16, device=dev)
    act = torch.empty(A, 6, dtype=torch.int32, device=dev)
    splits = list(POLICY_HEADS)

    def run():
        col = 0
        for v in flat:
            x[:, col:col + v.shape[1]].copy_(v)
            col += v.shape[1]
        h = torch.relu(x @ w1)
        h = torch.relu(h @ w2)
        logits = h @ wh
        for k, part in enumerate(torch.split(logits, splits, dim=1)):
            act[:, k] = part.argmax(dim=1).to(torch.int32)
        return act.data_ptr()

    run.actions = act
    return run


def stream_buffers(sim, ring, dev):
    """Caller-owned buffers for Manager::gpuStreamStep, ordered as the
    trainInterface (inputs then outputs, mgr.cpp:2383-2431), the layout an
    XLA custom call hands over.  The action inputs of step s point into the
    HBM ring (split into the discrete [A][4] and discrete-aim [A][2]
    tensors); the other inputs hold the engine's values after Manager::init,
    so copying them in every step changes nothing; outputs are fresh
    buffers.  Returns one pointer list per ring slot, the bytes each step
    copies, and the tensors to keep alive."""
    import torch

    ti = sim.train_interface()
    ins = {n: t.to_torch() for n, t in ti["inputs"].items()}
    outs = {n: t.to_torch() for n, t in ti["outputs"].items()}
    A = ring.shape[1]
    disc = ring[:, :, :4].contiguous()
    aim = ring[:, :, 4:6].contiguous()
    keep = [disc, aim]
    fixed = {}
    for n, t in ins.items():
        if n not in ("discrete", "aim"):
            fixed[n] = t.clone()
            keep.append(fixed[n])
    obufs = [torch.empty_like(t) for t in outs.values()]
    keep += obufs
    ptrs = []
    for k in range(ring.shape[0]):
        row = []
        for n, t in ins.items():
            if n == "discrete":
                row.append(disc[k].data_ptr())
            elif n == "aim":
                row.append(aim[k].data_ptr())
            else:
                row.append(fixed[n].data_ptr())
        row += [b.data_ptr() for b in obufs]
        ptrs.append(row)
    nbytes = sum(t.numel() * t.element_size() for t in ins.values()) + \
        sum(t.numel() * t.element_size() for t in outs.values())
    assert disc[0].numel() == A * 4
    return ptrs, nbytes, keep


def main():
    args = parse()
    # stdout carries the one JSON line only: native libraries print to fd 1
    # (RCCL's version banner at communicator init), so fd 1 is pointed at
    # stderr for the run and the line goes to a copy of the original.
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}")
    gpu = 0 if args.share_device else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    exchange = "gather" if args.gather else args.exchange
    if exchange == "auto":
        exchange = "wire" if world_size > 1 and not args.share_device else "none"
    dedicated = exchange == "wire" and world_size > 1 and (
        args.learner_dedicated == "on" or (args.learner_dedicated == "auto" and world_size >= 4))
    learner_only = dedicated and rank == 0  # this rank simulates nothing
    sims = world_size - 1 if dedicated else world_size  # simulator ranks
    si = rank - 1 if dedicated else rank  # this rank's shard (simulator ranks)
    if exchange != "none":
        # the step, the pack / unpack and the transfers on one explicit
        # stream (the default stream's handle, 0, means each manager's own
        # internal stream at the C ABI)
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    xgroup = None
    if world_size > 1:
        # Control plane (barriers, max-over-ranks time) on gloo: the step has
        # no data-path collective.  The learner exchange runs on RCCL.
        dist.init_process_group("gloo")
        if exchange != "none":
            if args.share_device:
                raise SystemExit("--exchange gather/local needs one GPU per rank")
            xgroup = dist.new_group(backend="nccl")
    elif exchange != "none":
        # one rank, exchange asked for explicitly: a one-rank RCCL group, so
        # the line carries the exchange's per-rank cost (pack copy + the RCCL
        # launch; nothing crosses xGMI)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)

    import madrona_mp_env as m
    from mpenv_dist import make_exchange
    import mpenv_tape

    W, ts = args.worlds, args.team_size
    N = 2 * ts
    A = W * N
    offset = si * W  # weak scaling: each simulator rank owns W global worlds
    sim = None
    if not learner_only:
        sim = m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=gpu, num_worlds=W, rand_seed=5,
                           auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                           team_size=ts, num_pbt_policies=0, policy_history_size=0,
                           scene_path=args.scene, world_id_offset=offset)
        sim.set_world_groups(args.world_groups)
    groups = sim.world_groups() if sim is not None else 0
    ctrl = sim.sim_control_tensor().to_torch() if sim is not None else None

    def start_episode():
        # Manager::init -- a forced reset of every world (simCtrl [0, 1, 1]:
        # random start step and team sides, scripts/jax_train.py:377)
        if sim is None:
            return
        ctrl.copy_(torch.tensor([0, 1, 1], dtype=torch.int32, device=dev).view_as(ctrl))
        torch.cuda.synchronize()
        sim.init()
        if args.bots != "none":
            pol = torch.zeros((W, 2, ts), dtype=torch.int32)
            if args.bots == "all":
                pol[:] = -1
            else:
                pol[:, 1, :] = -1
            sim.policy_assignment_tensor().to_torch().copy_(pol.view(-1, 1).to(dev))
        torch.cuda.synchronize()

    start_episode()
    ring = torch.from_numpy(mpenv_tape.tape_ring(TAPE_SEED, offset * N, A, RING)).to(dev) if sim is not None else None
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    def make_shadow(r):
        # the learner's copy of rank r's engine: same configuration, rank r's
        # worlds (wire.hip rebuilds r's outputs into it)
        return m.SimManager(exec_mode=m.madrona.ExecMode.CUDA, gpu_id=gpu, num_worlds=W, rand_seed=5,
                            auto_reset=True, sim_flags=int(m.SimFlags.Default), task_type=m.Task.Zone,
                            team_size=ts, num_pbt_policies=0, policy_history_size=0,
                            scene_path=args.scene, world_id_offset=(r - 1 if dedicated else r) * W)

    if exchange == "local":
        learner = make_exchange(exchange, sim, group=xgroup, grad_bytes=int(args.grad_mb * (1 << 20)),
                                update_every=args.update_every)
    elif exchange == "wire":
        learner = make_exchange(exchange, sim, group=xgroup, make_shadow=make_shadow, overlap=not args.wire_serial,
                                dedicated=dedicated, unpack_streams=4 if dedicated else 1)
    else:
        learner = make_exchange(exchange, sim, group=xgroup)

    policy = make_policy(sim, args.policy_hidden, dev) if args.actions == "policy" and sim is not None else None
    stream_ptrs = None
    if args.path == "stream" and sim is not None:
        if args.actions != "tape":
            raise SystemExit("--path stream runs the tape actions only")
        stream_ptrs, stream_bytes, _keep = stream_buffers(sim, ring, dev)

    def one_step(s, exchange_on=True):
        if learner_only:
            # the dedicated learner: receive this step's messages, unpack the
            # previous step's into the shadows (LearnerWire.submit)
            if exchange_on:
                learner.submit(sptr)
            return
        if stream_ptrs is not None:
            # gpuStreamStep: inputs from the caller's buffers (the step's
            # actions straight from the ring), the step, outputs copied out
            # -- the whole step (no step_async after it)
            sim.gpu_stream_step(sptr, stream_ptrs[s % RING])
        else:
            if policy is not None:
                # actions from the observations the previous step left (no tape)
                sim.copy_actions(policy(), sptr)
            elif args.actions == "combat":
                # the aim-bot reads the previous step's observations and writes
                # the step inputs directly (replaces the input copy)
                sim.combat_actions(ring[s % RING].data_ptr(), 0, 1, sptr)
            else:
                sim.copy_actions(ring[s % RING].data_ptr(), sptr)
            sim.step_async(sptr)
        if learner is not None and exchange_on:
            learner.submit(sptr)

    # ---- timed pass: W warmup steps, then K steps, no events or counters
    for s in range(args.warmup):
        one_step(s)
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        one_step(args.warmup + s)
    if learner is not None:
        learner.drain()
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_agent_steps = sims * A * args.steps
    value = total_agent_steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # ---- profile passes (not part of `value`): the same episode window
    # again (Manager::init, W warmup steps, K steps) with ONE world group, so
    # every kernel runs alone and its HIP-event duration is exclusive; then
    # once more with the kernels' workload counters on (their atomics slow
    # the kernels, so counters and timings never share a pass).
    # The exchange is not part of these passes (their windows restart the
    # episode; the learner's shadows are left as the timed pass left them).
    prof_pass = None
    if not args.no_profile_pass and not learner_only:
        if learner is not None:
            learner.drain()
        sim.set_world_groups(1)

        def window(timing, stats):
            start_episode()
            for s in range(args.warmup):
                one_step(s, exchange_on=False)
            torch.cuda.synchronize()
            sim.enable_kernel_timing(timing)
            sim.enable_stats(stats)
            for s in range(args.steps):
                one_step(args.warmup + s, exchange_on=False)
            torch.cuda.synchronize()
            out = sim.kernel_timings() if timing else sim.read_stats()
            sim.enable_kernel_timing(False)
            sim.enable_stats(False)
            return out

        timings = window(True, False)  # {name: (avg ms, launches)}
        counts = window(False, True)
        sim.set_world_groups(groups)
        prof_pass = (timings, counts)

    workload = f"simple_map {ts}v{ts} x {W} worlds/GPU" + ("" if args.bots == "none" else f" + A* bots ({args.bots})") \
        + {"tape": "", "combat": " + combat actions", "policy": f" + MLP policy loop (bf16, {args.policy_hidden} wide)"}[args.actions] \
        + ("" if args.path == "step" else " + gpuStreamStep buffer copies")
    result = {
        "metric": f"env steps/sec x agents (whole node), simple_map {ts}v{ts} @ {W} worlds"
                  + ("" if world_size == 1 else f"/GPU x {sims} GPUs")
                  + (" + 1 dedicated learner GPU" if dedicated else ""),
        "value": round(value, 1),
        "unit": "agent-steps/s",
        "n_gpus": world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": {"tape": "synthetic (hash action tape, seed 1234; 64-step ring resident in HBM)",
                 "combat": "synthetic (hash action tape, seed 1234; 64-step ring resident in HBM; overridden on "
                           "the device by the zone-seeking aim-bot)",
                 "policy": "synthetic (actions = argmax of a random-init bf16 MLP over every trainInterface "
                           "observation of the previous step)"}[args.actions],
        "config": {
            "workload": workload,
            "worlds_per_gpu": W,
            "agents_per_gpu": A,
            "total_worlds": W * sims,
            "task": "Zone",
            "sim_flags": "Default",
            "sim_control": [0, 1, 1],
            "bots": args.bots,
            "rand_seed": 5,
            "world_groups": groups,
            "actions": args.actions,
            "parallelism": f"world-sharded x{sims}" + ("" if learner is None else
                                                       f" + RCCL learner exchange ({exchange}"
                                                       + (", dedicated learner rank 0)" if dedicated else ")")),
            "exchange": exchange,
        },
        "world_steps_per_s": round(value / N, 1),
    }
    if learner is not None:
        result["exchange_bytes_per_step"] = learner.bytes_per_step()
        if exchange == "wire":
            result["wire_unpack"] = "step stream" if args.wire_serial else "own stream (overlaps the step)"
        if exchange in ("wire", "gather"):
            result["exchange_bytes_per_agent"] = round(result["exchange_bytes_per_step"]["sent_per_rank"] / A, 1)
    if stream_ptrs is not None:
        result["config"]["path"] = "gpuStreamStep (mgr.cpp:614-645)"
        result["stream_copy_bytes_per_step"] = stream_bytes
    if prof_pass is not None:
        timings, counts = prof_pass
        steps = args.steps
        dom = max(timings, key=lambda k: timings[k][0])
        dom_ms = timings[dom][0]
        lk_bytes = LK_ROW_BYTES * counts.get("lk_rows", 0) / steps  # k_obs's conditional rows, per step
        alg = KERNEL_BYTES_PER_AGENT[dom] * A + KERNEL_BYTES_PER_WORLD[dom] * W + (lk_bytes if dom == "k_obs" else 0)
        achieved = alg / (dom_ms * 1e-3) / 1e9
        prof = load_profile(args.traffic, workload)
        # the PMC pass of this very window when one was collected
        prof = prof.get("by_window", {}).get(f"{args.warmup}x{args.steps}", prof)
        traffic = prof.get("per_kernel", {}).get(dom)
        valu = prof.get("valu_insts_per_launch", {}).get(dom)
        step_bytes = sum(KERNEL_BYTES_PER_AGENT.values()) * A + sum(KERNEL_BYTES_PER_WORLD.values()) * W + lk_bytes
        kern_ms = sum(v[0] for v in timings.values())
        result["roofline"] = {
            "bound": KERNEL_BOUND[dom],
            "kernel": dom,
            "note": "profile pass (same episode window, one world group, whole batch per launch): "
                    "exclusive HIP-event time per launch",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": alg,
            "launch_ms": round(dom_ms, 4),
            # the limiter of the ray kernels: VALU issue (PMC instructions
            # per launch from profiles/, same workload) over the launch time
            "valu_issue": None if not valu else {
                "window": f"PMC instructions from {os.path.basename(args.traffic)} (tag {prof.get('tag')}: its "
                          f"profile pass, one world group); launch time from this run's profile pass "
                          f"(steps {args.warmup}..{args.warmup + args.steps - 1})",
                "same_window": prof.get("bench_window") == [args.warmup, args.steps],
                "insts_per_launch": valu,
                "achieved_per_s": round(valu / (dom_ms * 1e-3), 1),
                "peak_per_s": VALU_PEAK,
                "frac": round(valu / (dom_ms * 1e-3) / VALU_PEAK, 4),
                "lane_efficiency": prof.get("lane_efficiency", {}).get(dom),
            },
        }
        result["kernels_ms"] = {k: round(v[0], 4) for k, v in timings.items()}
        result["step_hbm"] = {
            "note": "sum of the kernels' algorithmic bytes (state each kernel reads counted per kernel); "
                    "survey_8d_bytes_per_step = SURVEY.md 8(d)'s whole-step definition, A x 4,468 + W x 512",
            "algorithmic_bytes_per_step": round(step_bytes),
            "survey_8d_bytes_per_step": 4468 * A + 512 * W,
            "lk_rows_per_step": round(counts.get("lk_rows", 0) / steps, 1),
            "kernel_ms_per_step": round(kern_ms, 4),
            "achieved_GBps_over_kernels": round(step_bytes / (kern_ms * 1e-3) / 1e9, 2),
        }
        lidar_rays = 80 * A * steps
        rays = lidar_rays + counts["los_rays"] + counts["shot_rays"]
        result["workload"] = {
            "note": f"per step, averaged over the counter pass's {steps} steps (same episode window)",
            "alive_agents": round(counts["alive_agents"] / steps, 1),
            "alive_frac": round(counts["alive_agents"] / steps / A, 4),
            "los_pairs": round(counts["los_pairs"] / steps, 1),
            "los_rays": round(counts["los_rays"] / steps, 1),
            "los_seen": round(counts["los_seen"] / steps, 1),
            "los_traced": round(counts.get("los_traced", 0) / steps, 1),
            "lidar_rays": 80 * A,
            "shot_rays": round(counts["shot_rays"] / steps, 1),
            "hit_agents": round(counts["hit_agents"] / steps, 1),
            "kills": round(counts["kills"] / steps, 2),
            "sphere_casts": round(counts["sphere_casts"] / steps, 1),
            "rays_per_s": round(rays / steps / (ms_per_step * 1e-3), 1),
            "bvh_queries_per_s": round((rays + counts["sphere_casts"]) / steps / (ms_per_step * 1e-3), 1),
        }
    if dedicated:
        # the learner rank simulates nothing: the first simulator rank's
        # profile pass stands for the step kernels
        obj = [{k: result[k] for k in ("roofline", "kernels_ms", "step_hbm", "workload") if k in result}]
        dist.broadcast_object_list(obj, src=1)
        if rank == 0:
            result.update(obj[0])
            result["profile_rank"] = 1
    if rank == 0 and world_size == 1 and args.cpu_baseline == "auto":
        result["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(result), file=line_out, flush=True)
    if learner is not None:
        learner.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
