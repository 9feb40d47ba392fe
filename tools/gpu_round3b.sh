# GPU tests + bench lines + profile + LDS counters (run under gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03} XFLAG="${XFLAG:--x}" K="$K" NOPROF=1 bash tools/gpu_round3.sh
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 && \
bash tools/pmc_lds.sh $TAG > gpurun_out/${TAG}_lds.log 2>&1
rc2=$?
tail -8 gpurun_out/${TAG}_lds.log
exit $(( rc | rc2 ))
