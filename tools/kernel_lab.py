"""Kernel lab: build variants of libmpenv.so with extra -D switches and time
their step kernels on the C3 workload (development tool; variants that
switch parts of a kernel off give wrong results by design and are never
used outside this tool).

  python tools/kernel_lab.py build NAME [--patch tools/lab/X.patch ...] [--sub 'FILE:OLD|||NEW' ...] [-DFOO=1 ...]
                                                        (here, cross-compiles)
  python tools/kernel_lab.py run NAME [NAME ...]        (on the GPU box)

Instrumentation and switched-off parts live in patches under tools/lab/
(the overlay): a build copies csrc/ into lab/NAME/src, applies the patches
there and compiles that copy, so no lab hook sits in the shipped sources.

  tools/lab/lab_hooks.patch   the round-1..5 switches (-DMPENV_LAB_MOVE_SKIP=,
                              _NO_TRI, _NO_BVH, _NO_CAPSULE, ...) and dropped
                              variants: retired in round 6 (every kernel change
                              had to re-merge it); it is in git history, before
                              the commit "retire lab_hooks.patch"
  k_sim's -DMPENV_LAB_PHASE_T / _SIM_SKIP= / MPENV_SIM_WPE= hooks are inserted
  by text (ksim_hooks below), not by a patch
e.g. build phase -DMPENV_LAB_PHASE_T
(tests/test_abi.py checks that every patch still applies to csrc/).
"""
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "madrona-mp-env_amd")
LAB = os.path.join(PKG, "lab")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))


# k_sim's lab hooks, inserted by text into the lab copy (k_sim changes too
# often for a patch): a phase timer after every block barrier
# (-DMPENV_LAB_PHASE_T, k_sim per-phase block cycles in stats slots 10..),
# -DMPENV_LAB_SIM_SKIP=bits to switch phases off (wrong results by design),
# -DMPENV_SIM_WPE=n for the waves-per-SIMD target, -DMPENV_SIM_BLOCK=n for
# the block size.
KSIM_SKIP = [("fireD(", 1), ("spawnAgentsD(", 2), ("zoneMatchInfoD(", 8), ("goalRegionsD(", 16),
             ("resetSystemD(", 128), ("appendCrumbsD(", 256), ("crumbRoundsD(", 512),
             ("exploreVisitedD(", 1024)]


def ksim_hooks(path):
    s = open(path).read()
    s = s.replace("constexpr int kSimBlock = 128;",
                  "#ifndef MPENV_SIM_BLOCK\n#define MPENV_SIM_BLOCK 128\n#endif\nconstexpr int kSimBlock = MPENV_SIM_BLOCK;")
    s = s.replace("#define MP_SIM_ATTR __attribute__((amdgpu_waves_per_eu(4)))",
                  "#ifndef MPENV_SIM_WPE\n#define MPENV_SIM_WPE 4\n#endif\n"
                  "#define MP_SIM_ATTR __attribute__((amdgpu_waves_per_eu(MPENV_SIM_WPE)))")
    head = "k_sim(DevState S, SceneDev sc)\n{"
    a = s.index(head) + len(head) - 1
    d, k = 0, a
    while True:
        d += {"{": 1, "}": -1}.get(s[k], 0)
        if d == 0:
            break
        k += 1
    body = s[a + 1:k]
    body = body.replace("__syncthreads();", "__syncthreads(); MP_PT();")
    for name, bit in KSIM_SKIP:
        body = body.replace(name, f"(MPENV_LAB_SIM_SKIP & {bit}) ? (void)0 : (void){name}")
    prelude = """
#ifndef MPENV_LAB_SIM_SKIP
#define MPENV_LAB_SIM_SKIP 0
#endif
#ifdef MPENV_LAB_PHASE_T
    uint64_t pt_prev = clock64();
    int pt_k = 0;
    auto PT = [&]() {
        if (threadIdx.x == 0 && S.stats) {
            const uint64_t t = clock64();
            atomicAdd(&S.stats[10 + pt_k], (unsigned long long)(t - pt_prev));
            pt_prev = t;
        }
        pt_k++;
    };
#define MP_PT() PT()
#else
#define MP_PT() ((void)0)
#endif
"""
    s = s[:a + 1] + prelude + body + s[k:]
    open(path, "w").write(s)


def build(name, args):
    import shutil

    import build_native as B

    out = os.path.join(LAB, name)
    os.makedirs(out, exist_ok=True)
    patches, defines, subs = [], [], []
    it = iter(args)
    for a in it:
        if a == "--patch":
            patches.append(os.path.abspath(next(it)))
        elif a == "--sub":  # "FILE:OLD|||NEW", a literal text substitution in the lab copy
            subs.append(next(it))
        else:
            defines.append(a)
    src_dir = os.path.join(out, "src")
    shutil.rmtree(src_dir, ignore_errors=True)
    shutil.copytree(B.CSRC, src_dir)
    for pf in patches:
        subprocess.run(["patch", "-s", "-p1", "-d", src_dir, "-i", pf], check=True)
    for sub in subs:
        fname, rest = sub.split(":", 1)
        old, new = rest.split("|||", 1)
        fp = os.path.join(src_dir, fname)
        text = open(fp).read()
        assert old in text, f"--sub: {old!r} not in {fname}"
        open(fp, "w").write(text.replace(old, new))
    if any(d.startswith(("-DMPENV_LAB_PHASE_T", "-DMPENV_LAB_SIM_SKIP", "-DMPENV_SIM_WPE", "-DMPENV_SIM_BLOCK"))
           for d in defines):
        ksim_hooks(os.path.join(src_dir, "kernels.hip"))
    common = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"-I{src_dir}",
              f"-I{B.INCLUDE}"] + list(defines)
    objs = []
    for src in B.LIB_SOURCES:
        s = os.path.join(src_dir, src)
        o = os.path.join(out, src + ".o")
        if src.endswith(".hip"):
            cmd = [B.HIPCC, "-x", "hip", f"--offload-arch={B.ARCH}", "-c", s, "-o", o] + common
        else:
            cmd = [B.HIPCC, "-x", "c++", "-c", s, "-o", o] + common + ["-D__HIP_PLATFORM_AMD__",
                                                                      "-I/opt/rocm/include"]
        subprocess.run(cmd, check=True)
        objs.append(o)
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o",
                    os.path.join(out, "libmpenv.so")] + objs, check=True)
    json.dump({"defines": defines, "patches": [os.path.relpath(p, ROOT) for p in patches], "subs": subs},
              open(os.path.join(out, "variant.json"), "w"))
    print("built", name, defines)


def time_one(name, worlds=int(os.environ.get("LAB_WORLDS", 16384)), team=int(os.environ.get("LAB_TEAM", 6)),
             warm=int(os.environ.get("LAB_WARM", 100)), steps=int(os.environ.get("LAB_STEPS", 200)), label=None):
    import mpenv_testlib as T

    path = os.path.join(LAB, name, "libmpenv.so") if name != "main" else os.path.join(PKG, "libmpenv.so")
    lib = C.CDLL(path)
    lib.mpenv_create.argtypes = [C.POINTER(T.MpenvConfig), C.POINTER(C.c_void_p)]
    lib.mpenv_last_error.restype = C.c_char_p
    for f in ("mpenv_init", "mpenv_step"):
        getattr(lib, f).argtypes = [C.c_void_p]
    lib.mpenv_enable_kernel_timing.argtypes = [C.c_void_p, C.c_int32]
    lib.mpenv_kernel_timings.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_char_p),
                                         C.POINTER(C.c_float), C.POINTER(C.c_int32)]
    cfg = T.MpenvConfig(1, 0, worlds, 5, 1, 0, 2, team, 0, 0, T.SCENE.encode(), 0, None, None, None,
                        None, 0)
    h = C.c_void_p()
    assert lib.mpenv_create(C.byref(cfg), C.byref(h)) == 0, lib.mpenv_last_error()
    # simCtrl [0, 1, 1] as bench.py (random start step and team sides)
    lib.mpenv_export_tensor.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
    hip0 = C.CDLL("libamdhip64.so")
    p, dt, nd, gid = C.c_void_p(), C.c_int32(), C.c_int32(), C.c_int32()
    dims = (C.c_int64 * 8)()
    assert lib.mpenv_export_tensor(h, 64, C.byref(p), C.byref(dt), C.byref(nd), dims, C.byref(gid)) == 0
    ctrl = (C.c_int32 * 3)(0, 1, 1)
    assert hip0.hipMemcpy(p, ctrl, C.c_size_t(12), 1) == 0
    assert lib.mpenv_init(h) == 0
    # 16-step action ring in device memory (hash tape, as bench.py)
    ring = T.mpenv_tape.tape_ring(1234, 0, worlds * 2 * team, 16)
    hip = C.CDLL("libamdhip64.so")
    dptr = C.c_void_p()
    assert hip.hipMalloc(C.byref(dptr), C.c_size_t(ring.nbytes)) == 0
    assert hip.hipMemcpy(dptr, ring.ctypes.data_as(C.c_void_p), C.c_size_t(ring.nbytes), 1) == 0
    lib.mpenv_copy_actions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    per = ring[0].nbytes

    lib.mpenv_combat_actions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    combat = os.environ.get("LAB_ACTIONS", "tape") == "combat"

    def step(s):
        if combat:
            # bench.py --actions combat: the device aim-bot over the tape
            lib.mpenv_combat_actions(h, C.c_void_p(dptr.value + (s % 16) * per), None, 1, None)
        else:
            lib.mpenv_copy_actions(h, C.c_void_p(dptr.value + (s % 16) * per), None)
        lib.mpenv_step(h)

    lib.mpenv_set_world_groups.argtypes = [C.c_void_p, C.c_int32]
    for s in range(warm):
        step(s)
    # step time with the default world groups, no timing hooks
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        step(warm + s)
    hip.hipDeviceSynchronize()
    el_groups = time.perf_counter() - t0
    # per-kernel times with one group (kernels alone on the GPU)
    lib.mpenv_set_world_groups(h, 1)
    for s in range(5):
        step(warm + steps + s)
    lib.mpenv_enable_kernel_timing(h, 1)
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        step(warm + steps + 5 + s)
    hip.hipDeviceSynchronize()
    el = time.perf_counter() - t0
    names = (C.c_char_p * 16)()
    ms = (C.c_float * 16)()
    ln = (C.c_int32 * 16)()
    n = lib.mpenv_kernel_timings(h, 16, names, ms, ln)
    res = {names[i].decode(): round(ms[i], 4) for i in range(n)}
    # Output digest: variants that keep the arithmetic must agree bit-for-bit.
    import hashlib

    lib.mpenv_export_tensor.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
    hip.hipDeviceSynchronize()
    dig = hashlib.sha1()
    pex = {}
    for eid in (6, 10, 12, 13, 18, 19, 20, 23, 24, 65, 66, 67, 11, 14, 15, 16, 17, 27, 28, 29, 30, 31, 32):
        p, dt, nd, gid = C.c_void_p(), C.c_int32(), C.c_int32(), C.c_int32()
        dims = (C.c_int64 * 8)()
        assert lib.mpenv_export_tensor(h, eid, C.byref(p), C.byref(dt), C.byref(nd), dims, C.byref(gid)) == 0
        nbytes = 4
        for i in range(nd.value):
            nbytes *= dims[i]
        buf = (C.c_char * nbytes)()
        assert hip.hipMemcpy(buf, p, C.c_size_t(nbytes), 2) == 0
        if eid in (6, 10, 12, 13, 18, 19, 20, 23, 24, 65, 66, 67):
            dig.update(bytes(buf))
        pex[eid] = hashlib.sha1(bytes(buf)).hexdigest()[:6]
        if str(eid) in os.environ.get("LAB_DUMP", "").split(","):
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            open(os.path.join(ROOT, "gpurun_out", f"dump_{label or name}_{eid}.bin"), "wb").write(bytes(buf))
    phases = None
    if os.environ.get("LAB_STATS"):
        # lab_hooks.patch builds with -DMPENV_LAB_PHASE_T: k_sim per-phase block cycles
        lib.mpenv_enable_stats.argtypes = [C.c_void_p, C.c_int32]
        lib.mpenv_read_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
        lib.mpenv_enable_stats(h, 1)
        ns = int(os.environ.get("LAB_STATS_STEPS", 50))
        for s in range(ns):
            step(s)
        st = (C.c_uint64 * 64)()
        n = lib.mpenv_read_stats(h, st, 64)
        lib.mpenv_enable_stats(h, 0)
        phases = [round(st[k] / ns / 1e6, 2) for k in range(10, n)]
    timeline = None
    if hasattr(lib, "mpenv_lab_wave"):
        # lab_hooks.patch with -DMPENV_LAB_WAVE_HIST=k: per-wave start / end of one kernel in one
        # step (100 MHz wall clock), the default world groups
        import numpy as np

        nw = 1 << 16
        tb = np.zeros(2 * nw, np.uint64)
        lib.mpenv_lab_wave.argtypes = [C.c_void_p, C.c_int32]
        lib.mpenv_set_world_groups(h, 1)
        hip.hipDeviceSynchronize()
        lib.mpenv_lab_wave(tb.ctypes.data, nw)  # clears
        step(1)
        hip.hipDeviceSynchronize()
        assert lib.mpenv_lab_wave(tb.ctypes.data, nw) == 0
        tt = tb.reshape(nw, 2)
        tt = tt[tt[:, 1] > 0].astype(np.float64)
        t0 = tt[:, 0].min()
        st_, en = (tt[:, 0] - t0) / 100.0, (tt[:, 1] - t0) / 100.0
        dur = en - st_
        span = en.max()
        timeline = {"waves": int(len(tt)), "span_us": round(span, 1), "mean_wave_us": round(dur.mean(), 1),
                    "dur_pct_us": [round(float(np.percentile(dur, q)), 1) for q in (10, 50, 90, 99, 100)],
                    "start_pct_us": [round(float(np.percentile(st_, q)), 1) for q in (10, 50, 90, 99, 100)],
                    "end_pct_us": [round(float(np.percentile(en, q)), 1) for q in (10, 50, 90, 99, 100)],
                    # busy fraction: wave-time integral over (span x max concurrent waves)
                    "waves_alive_at_pct_of_span": [int(((st_ <= f * span) & (en > f * span)).sum())
                                                   for f in (0.1, 0.25, 0.5, 0.75, 0.9)]}
    work = None
    if hasattr(lib, "mpenv_lab_work"):
        # lab_hooks.patch with -DMPENV_LAB_WORK: per-thread sphere-cast work of one step's k_move
        import numpy as np

        nthr = 1 << 18
        buf = np.zeros(11 * nthr, np.uint32)
        lib.mpenv_lab_work.argtypes = [C.c_void_p, C.c_int32]
        hip.hipDeviceSynchronize()
        lib.mpenv_lab_work(buf.ctypes.data, nthr)  # clears
        step(0)
        hip.hipDeviceSynchronize()
        assert lib.mpenv_lab_work(buf.ctypes.data, nthr) == 0
        a = worlds * 2 * team
        wv = buf.reshape(11, nthr)[:, :a].reshape(11, -1, 64).astype(np.float64)
        work = {}
        sites = ("ground0", "fwd_low", "fwd_high", "slide", "ground_chk", "stuck4", "stuck_ground", "fall")
        for k, nm in enumerate(("casts", "nodes", "tris") + tuple("nodes@" + x for x in sites)):
            lane_mean = wv[k].mean()
            wmax = wv[k].max(1)
            work[nm] = {"lane_mean": round(lane_mean, 2), "wave_max_mean": round(wmax.mean(), 2),
                        "simd_eff": round(lane_mean / max(wmax.mean(), 1e-9), 3),
                        "wave_max_pct": [round(float(np.percentile(wmax, q)), 1) for q in (10, 50, 90, 99, 100)],
                        "lane_pct": [round(float(np.percentile(wv[k], q)), 1) for q in (50, 90, 99, 99.9, 100)],
                        "lanes_active": round(float((wv[k] > 0).mean()), 4)}
    fan = None
    if hasattr(lib, "mpenv_lab_fan"):
        # tools/lab/fan_phases.patch: per forward-fan task, mean wave cycles
        # per phase and mean work counts (each read: the last launch's
        # per-wave sums; 5 steps)
        import numpy as np

        lib.mpenv_lab_fan.argtypes = [C.c_void_p, C.c_int32]
        acc = np.zeros(13, np.float64)
        fb = np.zeros(13, np.uint64)
        for s in range(5):
            step(s)
            hip.hipDeviceSynchronize()
            assert lib.mpenv_lab_fan(fb.ctypes.data, 13) == 0
            acc += fb
        nt = max(acc[5], 1.0)
        fan = {k: round(float(acc[i]) / nt, 2) for i, k in enumerate(
            ("cyc_pre", "cyc_cull", "cyc_masks", "cyc_walk", "cyc_post", "tasks", "survivors", "entries_walked",
             "entries_tested", "lane_tests")) if i != 5}
        fan["tasks_per_step"] = nt / 5
        nr = max(acc[12], 1.0)
        fan["rear_cyc_trace"] = round(float(acc[10]) / nr, 2)
        fan["rear_cyc_post"] = round(float(acc[11]) / nr, 2)
        fan["rear_tasks_per_step"] = nr / 5
    print(json.dumps({"variant": label or name, "fan": fan, "work": work, "timeline": timeline, "ms_per_step": round(1e3 * el_groups / steps, 4), "phases_mcyc": phases,
                      "ms_per_step_1group": round(1e3 * el / steps, 4), "kernels_1group": res,
                      "digest": dig.hexdigest()[:16], "per_export": pex}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3:])
    elif sys.argv[1] == "run":
        for spec in sys.argv[2:]:
            # NAME[@ENV=VAL,ENV=VAL]: a variant library plus runtime settings
            name, _, envs = spec.partition("@")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            subprocess.run([sys.executable, __file__, "_one", name, spec], check=True, env=env)
    elif sys.argv[1] == "_one":
        time_one(sys.argv[2], label=sys.argv[3] if len(sys.argv) > 3 else None)
