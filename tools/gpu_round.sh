#!/bin/bash
# The round's GPU measurements, one parameterised driver (run under gpurun):
#   TAG=r05x tools/gpu_round.sh bench   bench lines: driver window (20 steps
#                                       after 5), steady (1,000 after 100),
#                                       combat, gpuStreamStep path, wire loopback
#   TAG=r05x tools/gpu_round.sh prof    rocprof kernel trace + PMC passes of the
#                                       tape and combat workloads, and a trace of
#                                       the gpuStreamStep path
#   TAG=r05x tools/gpu_round.sh all     both
# Outputs under gpurun_out/; tools/pmc_summary.py condenses the profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:?set TAG}
WHAT=${1:-all}
B="timeout -k 10 300 python3 bench.py"
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    $B --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_bench_short.json && \
    $B > gpurun_out/${TAG}_bench.json && \
    $B --actions combat --cpu-baseline off > gpurun_out/${TAG}_bench_combat.json && \
    $B --path stream --cpu-baseline off > gpurun_out/${TAG}_bench_stream.json && \
    $B --exchange wire --cpu-baseline off > gpurun_out/${TAG}_bench_wire.json || exit $?
    for f in bench_short bench bench_combat bench_stream bench_wire; do
        python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('kernels_ms'))" $f
    done
fi
if [ "$WHAT" = prof ] || [ "$WHAT" = all ]; then
    bash tools/profile_round.sh ${TAG} > /dev/null && \
    BENCH_ARGS="--actions combat" bash tools/profile_round.sh ${TAG}_combat > /dev/null && \
    (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
     timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_stream -o run -- \
        python3 bench.py --path stream --steps 50 --warmup 10 --cpu-baseline off --no-profile-pass \
        > gpurun_out/prof_${TAG}_stream.json) && echo profiles done
fi
