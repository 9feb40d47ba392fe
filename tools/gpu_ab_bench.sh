#!/bin/bash
# A/B of bench.py settings on one GPU (each output line: the label, then the
# bench JSON line).  usage: tools/gpu_ab_bench.sh OUT "LABEL|ENV=V ...|ARGS" ...
# e.g. tools/gpu_ab_bench.sh gpurun_out/ab.jsonl "g1||--world-groups 1" "br|MPENV_LIDAR_BRANCH=1|--steps 20 --warmup 5"
out=$1; shift
mkdir -p "$(dirname "$out")"
: > "$out"
for spec in "$@"; do
    IFS='|' read -r label envs args <<< "$spec"
    line=$(eval "$envs timeout -k 10 240 python3 bench.py --cpu-baseline off --no-profile-pass $args" 2>>"$out.err") || { echo "bench failed: $label" >&2; exit 1; }
    echo "{\"label\": \"$label\", \"bench\": $line}" >> "$out"
done
