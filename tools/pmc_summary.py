"""Condense a tools/profile_round.sh run into tracked files under profiles/.

  profiles/<tag>_kernel_stats.csv  -- rocprofv3 --kernel-trace --stats summary of
                                      the default bench command (every launch)
  profiles/<tag>_kernels.json      -- per kernel, over the bench command's
                                      exclusive-timing window (its profile pass:
                                      whole-batch launches, warmup excluded):
                                      rocprof average duration next to the bench
                                      line's launch time, and per whole-batch
                                      launch from the --pmc passes: HBM bytes,
                                      VALU / SALU / LDS instructions, VALU issue
  profiles/pmc_traffic.json        -- what bench.py reads for roofline.traffic /
                                      valu_issue

VALU issue: SQ_INSTS_VALU per launch (wave instructions) against the chip's
issue peak of 256 CUs x 4 SIMDs x 1/2 wave-instruction per clock x 2.4 GHz
= 1.229e12 /s (a wave64 VALU op takes 2 cycles on a SIMD32,
MI355X_MICROARCH.md), over the kernel's average duration.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are KB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads (MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact for
streaming stores.  Each counter comes from its own rocprofv3 --pmc pass.

    python tools/pmc_summary.py TAG [SRC_DIR]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU_PEAK = 256 * 4 * 0.5 * 2.4e9  # wave-instructions per second


def short(name):
    n = name.split("(")[0].replace("mpenv::", "").replace("void ", "").strip()
    # the templated observation kernel: the step's and the learner's
    return {"k_obs<false>": "k_obs", "k_obs<true>": "k_obs_wire"}.get(n, n)


def counters(path):
    """{counter: {kernel: mean value per dispatch}} over k_* dispatches."""
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k.startswith("k_"):
                acc[row["Counter_Name"]][k].append(float(row["Counter_Value"]))
    return {c: {k: sum(v) / len(v) for k, v in d.items()} for c, d in acc.items()}


def main(tag, src):
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = json.load(open(os.path.join(src, "trace_bench.json")))
    warm, steps = bench["warmup"], bench["steps"]
    disp = defaultdict(list)  # kernel -> [(dispatch id, grid, ns)]
    with open(os.path.join(src, "trace", "run_kernel_trace.csv")) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k.startswith("k_"):
                disp[k].append((int(row["Dispatch_Id"]), int(row["Grid_Size_X"]),
                                int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    pmc = {}
    for sub in ("fetch", "write", "sq", "lanes"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            pmc.update(counters(p))
    out = {"tag": tag, "workload": bench["config"]["workload"], "bench_command_window":
           f"profile pass of `bench.py --cpu-baseline off`: whole-batch launches {warm}..{warm + steps - 1}",
           "kernels": {}}
    for k, lst in sorted(disp.items()):
        lst.sort()
        big = max(g for _, g, _ in lst)
        whole = [ns for _, g, ns in lst if g == big]
        window = whole[:warm + steps][warm:]  # the timing pass; the counter pass follows it
        if not window:
            continue
        avg = sum(window) / len(window)
        fetch = pmc.get("FETCH_SIZE", {}).get(k)
        write = pmc.get("WRITE_SIZE", {}).get(k)
        valu = pmc.get("SQ_INSTS_VALU", {}).get(k)
        r = {"rocprof_avg_ms": round(avg / 1e6, 4), "launches": len(window),
             "bench_launch_ms": bench.get("kernels_ms", {}).get(k)}
        if fetch is not None and write is not None:
            r["hbm_bytes_per_launch"] = int((2 * fetch + write) * 1024)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES",
                  "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in pmc and k in pmc[c]:
                r[c.lower()] = int(pmc[c][k])
        if valu:
            r["valu_issue_frac"] = round(valu / (avg * 1e-9) / VALU_PEAK, 4)
        # active lanes per VALU instruction over the wave size (the
        # "VALU thread utilisation" of the gfx9 SQ counters)
        tcv = pmc.get("SQ_THREAD_CYCLES_VALU", {}).get(k)
        aiv = pmc.get("SQ_ACTIVE_INST_VALU", {}).get(k)
        if tcv is not None and aiv:
            r["sq_thread_cycles_valu"] = int(tcv)
            r["sq_active_inst_valu"] = int(aiv)
            r["valu_lane_efficiency"] = round(tcv / (aiv * 64), 4)
        out["kernels"][k] = r
    # k_lidar runs as k_lidar_fan (forward fans) + k_lidar_rear (rear fans)
    # on scenes of <= 255 triangles; bench.py times the pair as "k_lidar"
    ks = out["kernels"]
    if "k_lidar_fan" in ks and "k_lidar_rear" in ks and "k_lidar" not in ks:
        a, b = ks["k_lidar_fan"], ks["k_lidar_rear"]
        comb = {"parts": ["k_lidar_fan", "k_lidar_rear"],
                "rocprof_avg_ms": round(a["rocprof_avg_ms"] + b["rocprof_avg_ms"], 4),
                "launches": a["launches"], "bench_launch_ms": bench.get("kernels_ms", {}).get("k_lidar")}
        for c in ("hbm_bytes_per_launch", "sq_insts_valu", "sq_insts_salu", "sq_insts_lds", "sq_waves",
                  "sq_wave_cycles", "sq_busy_cycles", "sq_wait_inst_any", "sq_active_inst_any"):
            if c in a and c in b:
                comb[c] = a[c] + b[c]
        if "sq_insts_valu" in comb:
            comb["valu_issue_frac"] = round(comb["sq_insts_valu"] / (comb["rocprof_avg_ms"] * 1e-3) / VALU_PEAK, 4)
        ks["k_lidar"] = comb
    with open(os.path.join(prof, f"{tag}_kernels.json"), "w") as f:
        json.dump(out, f, indent=1)
    traffic = {"tag": tag, "workload": out["workload"], "bench_window": [warm, steps],
               "per_kernel": {k: v.get("hbm_bytes_per_launch") for k, v in ks.items()},
               "valu_insts_per_launch": {k: v.get("sq_insts_valu") for k, v in ks.items()},
               "lane_efficiency": {k: v.get("valu_lane_efficiency") for k, v in ks.items()
                                   if v.get("valu_lane_efficiency") is not None},
               "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per whole-batch launch, separate --pmc passes"}
    # one entry per workload (bench.py picks the one it runs)
    path = os.path.join(prof, "pmc_traffic.json")
    try:
        allw = json.load(open(path))
    except (OSError, ValueError):
        allw = {}
    if "workloads" not in allw:
        allw = {"workloads": {allw["workload"]: allw} if "workload" in allw else {}}
    # per workload: every measured window under by_window ("WARMUPxSTEPS",
    # bench.py prefers the one it runs), the longest one at the top level
    prev = allw["workloads"].get(traffic["workload"], {})
    by_window = dict(prev.get("by_window", {}))
    if "bench_window" in prev and "per_kernel" in prev:
        pw = prev["bench_window"]
        by_window.setdefault(f"{pw[0]}x{pw[1]}", {k: v for k, v in prev.items() if k != "by_window"})
    by_window[f"{warm}x{steps}"] = traffic
    top = max(by_window.values(), key=lambda e: e["bench_window"][1])
    allw["workloads"][traffic["workload"]] = dict(top, by_window=by_window)
    with open(path, "w") as f:
        json.dump(allw, f, indent=1)
    for k, v in ks.items():
        print(k, v)


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    main(tag, src)
