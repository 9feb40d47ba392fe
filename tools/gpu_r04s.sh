# GPU tests (all but the full-batch file) + the bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04s}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -k "not full_batch" > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
NOPROF=1 TAG=$TAG bash tools/gpu_bench_all.sh
