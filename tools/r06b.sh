set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r06c}
timeout -k 10 900 python -u -m pytest tests/test_wire_gpu.py tests/test_exchange_gpu.py "tests/test_parity_gpu.py::test_gpu_stream_step_buffers_abi" "tests/test_parity_gpu.py::test_jax_custom_call_targets_match_gpu_stream_step" -x -v --timeout 500 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/wire_timing.py > gpurun_out/${T}_wire_timing.json && cat gpurun_out/${T}_wire_timing.json && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${T}_bench_short.json && \
timeout -k 10 300 python3 bench.py --path stream --cpu-baseline off > gpurun_out/${T}_bench_stream.json && \
python3 -c "import json,sys
for f in ('bench_short','bench_stream'):
    d=json.load(open('gpurun_out/${T}_'+f+'.json')); print(f, d['value'], d['ms_per_step'], d.get('kernels_ms'))"
