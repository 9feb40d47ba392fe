# Round 4: GPU suite (byte-exact compare, combat every-world test) + the
# gpuStreamStep bench line.  Run under gpurun; logs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04b}
timeout -k 10 240 python3 bench.py --path stream --cpu-baseline off > gpurun_out/${TAG}_bench_stream.json 2> gpurun_out/${TAG}_bench_stream.err && \
timeout -k 10 1500 python -u -m pytest tests -m gpu ${XFLAG:--x} -v -s --timeout 600 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_gpu_tests.log
exit $rc
