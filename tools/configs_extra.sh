#!/bin/bash
# Extra bench lines (run under gpurun after tools/configs_round.sh): world
# group sweep in both windows and the closed policy loop.
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/configs_$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
run() { # name, timeout, args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAILED $name"; exit 1; }
    cat $OUT/$name.json
}
run c3_groups3 240 python -u bench.py --cpu-baseline off --world-groups 3 --no-profile-pass
run c3_short_groups1 240 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --world-groups 1 --no-profile-pass
run c3_short_groups2 240 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --world-groups 2 --no-profile-pass
run c3_short_groups3 240 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --world-groups 3 --no-profile-pass
run c3_policy_loop 300 python -u bench.py --actions policy --cpu-baseline off --no-profile-pass
