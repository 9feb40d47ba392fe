# Round 4, combat attribution (run under gpurun): combat bench lines, lab
# variants in the combat regime, then the rocprof trace + PMC passes of
# `bench.py --actions combat`.  Outputs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04a}
timeout -k 10 240 python3 bench.py --actions combat --cpu-baseline off > gpurun_out/${TAG}_bench_combat.json && \
LAB_ACTIONS=combat VARIANTS="${VARIANTS:-main work skip2 skip8 nocap}" TAG=${TAG}_combat LIMIT=400 bash tools/gpu_lab.sh && \
BENCH_ARGS="--actions combat" bash tools/profile_round.sh ${TAG}_combat > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_prof.log
exit $rc
