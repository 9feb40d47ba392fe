#!/bin/bash
# Instruction-fetch counters per kernel (run under gpurun; one --pmc pass per
# counter group, each under its own kill timeout).
set -o pipefail
OUT=gpurun_out/prof_icache
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
ARGS="--steps 50 --warmup 20 --world-groups 1 --no-profile-pass --cpu-baseline off"
timeout -s KILL 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_ANY\|SQ_INST_CYCLES_[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt || true
cat $OUT/names.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $OUT/a -o run -- \
    python3 bench.py $ARGS > $OUT/a.json 2> $OUT/a.err && \
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --kernel-trace --output-format csv -d $OUT/b -o run -- \
    python3 bench.py $ARGS > $OUT/b.json 2> $OUT/b.err
echo rc=$?
