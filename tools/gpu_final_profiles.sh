# Final-tree profiles in one call: rocprof trace + PMC passes of the tape and
# combat workloads (default windows), the gpuStreamStep kernel trace, and the
# driver's 20-step window (tape, combat) for the short-window PMC entries.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04ae}
TAG=$TAG bash tools/gpu_prof_final.sh && \
BENCH_ARGS="--steps 20 --warmup 5" PMC_ARGS="--steps 20 --warmup 5 --world-groups 1 --no-profile-pass --cpu-baseline off" \
  bash tools/profile_round.sh ${TAG}_short > /dev/null && \
BENCH_ARGS="--steps 20 --warmup 5 --actions combat" PMC_ARGS="--steps 20 --warmup 5 --world-groups 1 --no-profile-pass --cpu-baseline off --actions combat" \
  bash tools/profile_round.sh ${TAG}_short_combat > /dev/null && echo all profiles done
