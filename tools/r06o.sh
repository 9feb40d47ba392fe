set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:?}
timeout -k 10 600 python -u -m pytest "tests/test_parity_gpu.py::test_gpu_stream_step_buffers_abi" "tests/test_parity_gpu.py::test_jax_custom_call_targets_match_gpu_stream_step" -x -q --timeout 500 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --path stream --cpu-baseline off > gpurun_out/${T}_bench_stream.json && \
python3 -c "import json
d=json.load(open('gpurun_out/${T}_bench_stream.json')); print(d['value'], d['ms_per_step'], d.get('kernels_ms'))"
