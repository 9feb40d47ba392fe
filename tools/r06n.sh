# driver-window and stream-path profiles (rocprof trace + PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:?}
BENCH_ARGS="--steps 20 --warmup 5" PMC_ARGS="--steps 20 --warmup 5 --world-groups 1 --no-profile-pass --cpu-baseline off" \
    bash tools/profile_round.sh ${T}_short > /dev/null && \
BENCH_ARGS="--steps 20 --warmup 5 --actions combat" PMC_ARGS="--steps 20 --warmup 5 --world-groups 1 --no-profile-pass --cpu-baseline off --actions combat" \
    bash tools/profile_round.sh ${T}_short_combat > /dev/null && \
BENCH_ARGS="--path stream" bash tools/profile_round.sh ${T}_stream > /dev/null && echo profiles done
