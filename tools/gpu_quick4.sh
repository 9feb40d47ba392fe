# Round 4 quick loop (run under gpurun): parity subset, then bench lines
# (driver window, steady, combat).  TAG names the outputs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "${K:-golden or live or edge_cases or smoke}" > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_bench_short.json && \
timeout -k 10 300 python3 bench.py --cpu-baseline off > gpurun_out/${TAG}_bench.json && \
timeout -k 10 300 python3 bench.py --actions combat --cpu-baseline off > gpurun_out/${TAG}_bench_combat.json
rc=$?
for f in bench_short bench bench_combat; do python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('kernels_ms'))" $f; done
exit $rc
