# Quick GPU check of the captured-graph step (run under gpurun): the graph
# test, the smoke, then bench lines with the graph on and off.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r03w}
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -v -s -x --timeout 300 --timeout-method thread \
    -k "graph or world_groups or python_module or stream_step" > gpurun_out/${TAG}_graph_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
MPENV_STEP_GRAPH=0 timeout -k 10 300 python -u bench.py --cpu-baseline off --no-profile-pass > gpurun_out/${TAG}_bench_nograph.json 2> gpurun_out/${TAG}_bench_nograph.err && \
timeout -k 10 300 python -u bench.py --cpu-baseline off --no-profile-pass > gpurun_out/${TAG}_bench_graph.json 2> gpurun_out/${TAG}_bench_graph.err && \
MPENV_STEP_GRAPH=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --no-profile-pass > gpurun_out/${TAG}_bench_short_nograph.json 2>> gpurun_out/${TAG}_bench_nograph.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --no-profile-pass > gpurun_out/${TAG}_bench_short_graph.json 2>> gpurun_out/${TAG}_bench_graph.err
rc=$?
tail -3 gpurun_out/${TAG}_graph_tests.log
cat gpurun_out/${TAG}_smoke.log gpurun_out/${TAG}_bench*.json
exit $rc
