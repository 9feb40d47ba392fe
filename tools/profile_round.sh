#!/bin/bash
# Profiles the bench workload on the GPU box (run under gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench command itself
#      (its profile pass launches every kernel over the whole batch; the
#      summary tool averages those launches for comparison with the bench
#      line's launch_ms)
#   2-4. --pmc passes (each counter set in its own run) over a one-group
#      window (every launch covers the whole batch):
#      FETCH_SIZE, WRITE_SIZE, SQ instruction counters.
# Outputs under gpurun_out/prof_<tag>/; tools/pmc_summary.py condenses them.
set -o pipefail
TAG=${1:-r02}
# BENCH_ARGS: extra bench.py flags for every pass (e.g. "--actions combat")
PMC_ARGS="${PMC_ARGS:---steps 200 --warmup 100 --world-groups 1 --no-profile-pass --cpu-baseline off} $BENCH_ARGS"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --cpu-baseline off $BENCH_ARGS > $OUT/trace_bench.json && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py $PMC_ARGS > $OUT/fetch_bench.json && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
    python3 bench.py $PMC_ARGS > $OUT/write_bench.json && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $OUT/sq -o run -- \
    python3 bench.py $PMC_ARGS > $OUT/sq_bench.json || exit $?
# VALU lane utilisation, when gfx950's counter list has the thread-cycle
# counters (rocprofv3 --list-avail): active lanes per VALU instruction
timeout -k 10 120 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1
if grep -q SQ_THREAD_CYCLES_VALU $OUT/list_avail.txt; then
    timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv \
        -d $OUT/lanes -o run -- python3 bench.py $PMC_ARGS > $OUT/lanes_bench.json || exit $?
fi
find $OUT -name "*.csv"
