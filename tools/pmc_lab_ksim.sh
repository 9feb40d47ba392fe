#!/bin/bash
# k_sim HBM bytes with and without the explore-grid update (lab variants
# `cur` and `sk1024`), one --pmc pass per counter (run under gpurun).
set -o pipefail
OUT=gpurun_out/pmc_lab_ksim
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export LAB_WARM=50 LAB_STEPS=50
for v in cur sk1024; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/${v}_$c -o run -- \
        python3 tools/kernel_lab.py _one $v > $OUT/${v}_$c.json 2> $OUT/${v}_$c.err || exit 1
  done
done
echo done
