# Full-batch GPU tests + the stream-path bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04t}
timeout -k 10 200 python3 bench.py --path stream --cpu-baseline off > gpurun_out/${TAG}_bench_stream.json && \
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_stream.json')); print('stream', d['value'], d['ms_per_step'])" || exit $?
timeout -k 10 900 python -u -m pytest tests/test_full_batch_gpu.py tests/test_wire_gpu.py -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
exit $rc
