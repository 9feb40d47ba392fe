#!/bin/bash
# Profiles the bench workload on the GPU box (run under gpurun).  Every pass
# runs the bench command itself (default window unless ARGS is set), so the
# rocprof averages describe the same launches as the bench line:
#   1. rocprofv3 --kernel-trace --stats      -> per-kernel durations
#   2. rocprofv3 --pmc FETCH_SIZE (own pass) -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE (own pass) -> HBM write bytes per dispatch
#   4. rocprofv3 --pmc SQ_* (own pass)        -> VALU/SALU/LDS instructions per dispatch
# Outputs under gpurun_out/prof_<tag>/; tools/pmc_summary.py condenses them.
set -o pipefail
TAG=${1:-r02}
ARGS=${ARGS:-}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --cpu-baseline off $ARGS > $OUT/trace_bench.json && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --cpu-baseline off $ARGS > $OUT/fetch_bench.json && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --cpu-baseline off $ARGS > $OUT/write_bench.json && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $OUT/sq -o run -- \
    python3 bench.py --cpu-baseline off $ARGS > $OUT/sq_bench.json && \
find $OUT -name "*.csv"
