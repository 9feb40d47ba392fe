# Round-3 full GPU pass (run under gpurun): GPU tests, bench lines (default,
# driver window, combat), then the rocprof trace + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r03} XFLAG="${XFLAG:--x}" K="$K" bash tools/gpu_r03.sh
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ -n "$NOPROF" ] && exit $rc
bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1
rc2=$?
tail -3 gpurun_out/${TAG}_prof.log
exit $(( rc | rc2 ))
