# Forward-fan lidar lab (run under gpurun): parity subset on the in-tree
# build, then kernel_lab timings -- fan vs BVH (MPENV_LIDAR_FAN=0), tape and
# combat -- and the fanph overlay's per-phase wave cycles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04h}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "${K:-golden or live or lidar}" > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 tools/kernel_lab.py run main main@LAB_ACTIONS=combat main@MPENV_LIDAR_FAN=0 \
    main@MPENV_LIDAR_FAN=0,LAB_ACTIONS=combat ${VARIANTS:-fanph fanph@LAB_ACTIONS=combat} > gpurun_out/${TAG}_lab.jsonl
