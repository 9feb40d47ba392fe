# Lidar default A/B in the driver's window and steady, lists tests, wire timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04q}
timeout -k 10 300 python -u -m pytest tests/test_lidar_paths_gpu.py -v -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_lidar_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_lidar_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_lidar_tests.log
timeout -k 10 200 python3 tools/wire_timing.py > gpurun_out/${TAG}_wire_timing.json && cat gpurun_out/${TAG}_wire_timing.json && \
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_short_bvh.json && \
MPENV_LIDAR_FAN=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_short_fan.json && \
timeout -k 10 200 python3 bench.py --cpu-baseline off > gpurun_out/${TAG}_steady_bvh.json && \
MPENV_LIDAR_FAN=1 timeout -k 10 200 python3 bench.py --cpu-baseline off > gpurun_out/${TAG}_steady_fan.json || exit $?
for f in short_bvh short_fan steady_bvh steady_fan; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('kernels_ms'))" $f
done
