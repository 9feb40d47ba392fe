# Final-tree check in one call: the whole GPU suite (both halves), smoke, and
# the driver's two bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04ak}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -1 gpurun_out/${TAG}_smoke.log && \
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_bench_short.json && \
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_short.json')); print('short', d['value'], d['ms_per_step'])"
[ -n "$WITH_BENCH" ] || exit 0
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json && \
timeout -k 10 300 python3 bench.py --actions combat --cpu-baseline off > gpurun_out/${TAG}_bench_combat.json && \
for f in bench bench_combat; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('kernels_ms'))" $f || exit 1
done
