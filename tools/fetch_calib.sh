#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (run under gpurun):
# one --pmc pass per counter over tools/fetch_calib; per-kernel values into
# gpurun_out/calib/summary.txt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/calib
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/calib/$c -o run -- \
        ./tools/fetch_calib > gpurun_out/calib/$c.log 2>&1 || exit 1
done
python3 - <<'PY' > gpurun_out/calib/summary.txt
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(c, r["Kernel_Name"].split("(")[0], float(r["Counter_Value"]) * 1024, "bytes")
PY
cat gpurun_out/calib/FETCH_SIZE.log gpurun_out/calib/summary.txt
