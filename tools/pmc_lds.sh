#!/bin/bash
# LDS bank-conflict counters per kernel (run under gpurun): one --pmc pass
# over a one-group bench window; per-dispatch rows under gpurun_out/pmc_lds_<tag>/.
set -o pipefail
TAG=${1:-r03}
ARGS=${PMC_ARGS:---steps 60 --warmup 20 --world-groups 1 --no-profile-pass --cpu-baseline off}
OUT=gpurun_out/pmc_lds_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py $ARGS > $OUT/bench.json && \
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("mpenv::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / max(1, n[(k, c)]) / 1e6, 3) for c, v in d.items()}, "(M per dispatch)")
PY
