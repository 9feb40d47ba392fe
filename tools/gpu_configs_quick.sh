# C2/C1/C3 bench lines without CPU baseline (run under gpurun), after a parity subset
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
    -k "${TESTS:-1v1x64 or 3v3x7 or 6v6x16_f0 or C2}" > gpurun_out/gpu_quick.log 2>&1 && \
timeout -k 10 200 python -u bench.py --worlds 4096 --team-size 3 --cpu-baseline off > gpurun_out/c2.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --worlds 64 --team-size 1 --steps 300 --warmup 30 --cpu-baseline off > gpurun_out/c1.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --cpu-baseline off > gpurun_out/c3.json 2>/dev/null
rc=$?
tail -1 gpurun_out/gpu_quick.log
for f in c2 c1 c3; do python3 -c "
import json; d=json.load(open('gpurun_out/$f.json')); print('$f', round(d['value']/1e6,2), 'M', d['ms_per_step'], d.get('kernels_ms'))" 2>/dev/null; done
exit $rc
