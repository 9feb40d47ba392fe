"""Condense a tools/profile_round.sh run into tracked files under profiles/.

  profiles/<tag>_kernel_stats.csv  -- rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv           -- per kernel: launches, avg ns, VGPR/SGPR/LDS/
                                      scratch, FETCH_SIZE / WRITE_SIZE (KB per
                                      launch, raw) and corrected HBM bytes
  profiles/pmc_traffic.json        -- the dominant kernel's HBM bytes per launch,
                                      read by bench.py for roofline.traffic

VALU issue: SQ_INSTS_VALU per launch (wave instructions) against the chip's
issue peak of 256 CUs x 4 SIMDs x 1/2 wave-instruction per clock x 2.4 GHz
= 1.229e12 /s (a wave64 VALU op takes 2 cycles on a SIMD32,
MI355X_MICROARCH.md), over the kernel's average duration.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are KB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads (MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact for
streaming stores.  Each counter comes from its own rocprofv3 --pmc pass.
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
    return name.split("(")[0].replace("mpenv::", "")


def counters(path, counter):
    acc = defaultdict(list)
    meta = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            acc[k].append(float(row["Counter_Value"]))
            meta[k] = dict(vgpr=int(row["VGPR_Count"]), agpr=int(row["Accum_VGPR_Count"]),
                           sgpr=int(row["SGPR_Count"]), lds=int(row["LDS_Block_Size"]),
                           scratch=int(row["Scratch_Size"]), wg=int(row["Workgroup_Size"]),
                           grid=int(row["Grid_Size"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, meta


def main(tag, src, workload):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats_src = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_src, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    stats = {}
    with open(stats_src) as f:
        for row in csv.DictReader(f):
            stats[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]))
    fetch, meta = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, _ = counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    sqf = os.path.join(src, "sq", "run_counter_collection.csv")
    valu = counters(sqf, "SQ_INSTS_VALU")[0] if os.path.exists(sqf) else {}
    waves = counters(sqf, "SQ_WAVES")[0] if os.path.exists(sqf) else {}
    rows = []
    for k, (calls, avg) in sorted(stats.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        if k not in fetch:
            continue
        hbm = (2 * fetch[k] + write.get(k, 0.0)) * 1024
        v = valu.get(k, 0.0)
        rows.append(dict(kernel=k, launches=calls, avg_ns=round(avg), **meta.get(k, {}),
                         fetch_kb=round(fetch[k], 1), write_kb=round(write.get(k, 0.0), 1),
                         hbm_bytes_per_launch=int(hbm), waves=int(waves.get(k, 0)),
                         valu_insts_per_launch=int(v),
                         valu_issue_frac=round(v / (avg * 1e-9) / VALU_PEAK, 4) if avg else 0.0))
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    mpenv = [r for r in rows if r["kernel"].startswith("k_")]
    dom = max(mpenv, key=lambda r: r["avg_ns"])
    out = dict(tag=tag, workload=workload, kernel=dom["kernel"],
               hbm_bytes_per_launch=dom["hbm_bytes_per_launch"],
               per_kernel={r["kernel"]: r["hbm_bytes_per_launch"] for r in mpenv},
               valu_insts_per_launch={r["kernel"]: r["valu_insts_per_launch"] for r in mpenv},
               valu_issue_frac={r["kernel"]: r["valu_issue_frac"] for r in mpenv},
               formula="(2*FETCH_SIZE + WRITE_SIZE) * 1024, separate --pmc passes")
    with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    for r in rows:
        print(r)


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    main(tag, src, "simple_map 6v6 x 16384 worlds/GPU")
