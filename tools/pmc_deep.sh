#!/bin/bash
# Extra PMC passes (LDS / VALU / wait breakdown) over a short bench run.
set -e
OUT=gpurun_out/pmc_deep
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $OUT/p1 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/p1.json
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
    SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_ADDR_CONFLICT --kernel-trace --output-format csv -d $OUT/p2 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/p2.json
