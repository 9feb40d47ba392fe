"""Per-kernel averages from rocprofv3 outputs under a directory (kernel
trace: duration; counter collection: counters per dispatch), one line per
(run, kernel).    python tools/kstats.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*"))):
    if not os.path.isdir(d):
        continue
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    dur = defaultdict(list)
    for f in tr:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("mpenv::", "")
            if k.startswith("k_"):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ctr = defaultdict(lambda: defaultdict(list))
    for f in cc:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("mpenv::", "")
            if k.startswith("k_"):
                ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(dur):
        v = dur[k][len(dur[k]) // 3:]  # drop the warm-up third
        line = f"{os.path.basename(d):18s} {k:14s} avg {sum(v) / len(v):.4f} ms ({len(v)} launches)"
        for c, vals in sorted(ctr[k].items()):
            line += f" {c}={sum(vals) / len(vals) / 1e6:.2f}M"
        print(line)
