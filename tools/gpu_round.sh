# GPU round check (run under gpurun): GPU tests, default bench, then the driver's short window.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-baseline ${CPU:-auto} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err && \
cat gpurun_out/bench.json gpurun_out/bench_short.json
rc=$?
tail -3 gpurun_out/gpu_tests.log
exit $rc
