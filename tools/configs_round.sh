#!/bin/bash
# Bench lines for the other BASELINE.json configurations and an N=2
# rehearsal on one GPU (run under gpurun; outputs under gpurun_out/configs_<tag>/).
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/configs_$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
run() { # name, timeout, args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAILED $name"; exit 1; }
    cat $OUT/$name.json
}
run c3_groups1 240 python -u bench.py --cpu-baseline off --world-groups 1
run c2_3v3_4096 240 python -u bench.py --worlds 4096 --team-size 3 --cpu-baseline off
run c1_1v1_64 240 python -u bench.py --worlds 64 --team-size 1 --steps 300 --warmup 30
run c5_bots_team1 240 python -u bench.py --bots team1 --cpu-baseline off
run c3_share2 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --share-device --steps 300 --warmup 30 --cpu-baseline off
