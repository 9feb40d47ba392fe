#!/bin/bash
# A/B of bench.py settings on one GPU (each line: the label, then the bench
# JSON line).  usage: tools/gpu_ab_bench.sh OUT "LABEL:ARGS" ...
# e.g. tools/gpu_ab_bench.sh gpurun_out/ab.jsonl "g1:--world-groups 1" "g2:--world-groups 2"
out=$1; shift
mkdir -p "$(dirname "$out")"
: > "$out"
for spec in "$@"; do
    label=${spec%%:*}; args=${spec#*:}
    line=$(timeout -k 10 240 python3 bench.py --cpu-baseline off --no-profile-pass $args 2>>"$out.err") || { echo "bench failed: $label" >&2; exit 1; }
    echo "{\"label\": \"$label\", \"bench\": $line}" >> "$out"
done
