#!/bin/bash
# One SQ counter pass per kernel_lab variant (run under gpurun after
# `python tools/kernel_lab.py build NAME ...` here):
#   bash tools/pmc_lab.sh main packet
# Outputs under gpurun_out/pmc_<variant>/ (per-dispatch counters of every kernel).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for v in "${@:-main}"; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES \
        SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv \
        -d gpurun_out/pmc_$v -o run -- python3 tools/kernel_lab.py _one $v > gpurun_out/pmc_$v.log 2>&1 || exit 1
done
