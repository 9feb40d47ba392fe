# Driver-window PMC profile (tape and combat), then the graph A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BENCH_ARGS="--steps 20 --warmup 5" PMC_ARGS="--steps 20 --warmup 5 --world-groups 1 --no-profile-pass --cpu-baseline off" \
  bash tools/profile_round.sh r04z_short > /dev/null && \
BENCH_ARGS="--steps 20 --warmup 5 --actions combat" PMC_ARGS="--steps 20 --warmup 5 --world-groups 1 --no-profile-pass --cpu-baseline off --actions combat" \
  bash tools/profile_round.sh r04z_short_combat > /dev/null && echo profiles done && \
TAG=r04y bash tools/gpu_ab_graph.sh
