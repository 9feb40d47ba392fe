# round-6 measurement pass: rocprof + PMC of the C3 tape / combat / stream
# workloads, the C2 (3v3 x 4,096) and C1 (1v1 x 64) bench lines with their
# own rocprof traces, and the list of gfx950 PMC counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:?}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/${T}_list_avail.txt 2>&1
TAG=$T bash tools/gpu_round.sh prof && \
timeout -k 10 300 python3 bench.py --team-size 3 --worlds 4096 > gpurun_out/${T}_c2_3v3_4096.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_c2 -o run -- \
    python3 bench.py --team-size 3 --worlds 4096 --cpu-baseline off > gpurun_out/prof_${T}_c2.json && \
timeout -k 10 300 python3 bench.py --team-size 1 --worlds 64 > gpurun_out/${T}_c1_1v1_64.json && \
python3 -c "import json
for f in ('c2_3v3_4096','c1_1v1_64'):
    d=json.load(open('gpurun_out/${T}_'+f+'.json')); print(f, d['value'], d['ms_per_step'], d.get('kernels_ms'), d.get('cpu_baseline'))"
