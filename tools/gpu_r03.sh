# Round-3 GPU check (run under gpurun): GPU tests (optionally -k filter), then
# the default bench, the driver's short window and the combat line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 ${TEST_LIMIT:-1000} python -u -m pytest tests -m gpu -v -s ${XFLAG:--x} --timeout 400 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ -n "$NOBENCH" ] && exit $rc
timeout -k 10 300 python -u bench.py --cpu-baseline ${CPU:-off} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_bench_short.json 2> gpurun_out/${TAG}_bench_short.err && \
timeout -k 10 300 python -u bench.py --actions combat --cpu-baseline off > gpurun_out/${TAG}_bench_combat.json 2> gpurun_out/${TAG}_bench_combat.err
rc2=$?
cat gpurun_out/${TAG}_bench*.json
exit $(( rc | rc2 ))
