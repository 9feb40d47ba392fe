# The whole GPU suite (run under gpurun), log under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:?set TAG}
timeout -k 10 1100 python -u -m pytest tests -m gpu ${XFLAG:--x} -v -s --timeout 600 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_gpu_tests.log
exit $rc
