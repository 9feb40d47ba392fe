set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:?}
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 600 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --team-size 3 --worlds 4096 > gpurun_out/${T}_c2_3v3_4096.json && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${T}_bench_short.json && \
timeout -k 10 300 python3 bench.py --actions combat --cpu-baseline off > gpurun_out/${T}_bench_combat.json && \
python3 -c "import json
for f in ('c2_3v3_4096','bench_short','bench_combat'):
    d=json.load(open('gpurun_out/${T}_'+f+'.json')); print(f, d['value'], d['ms_per_step'], d.get('kernels_ms'))"
