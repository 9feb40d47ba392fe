# Final-tree profiles: rocprof trace + PMC passes for the tape and combat
# workloads, and a kernel trace of the gpuStreamStep path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04u}
bash tools/profile_round.sh ${TAG} > /dev/null && \
BENCH_ARGS="--actions combat" bash tools/profile_round.sh ${TAG}_combat > /dev/null && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_stream -o run -- \
    python3 bench.py --path stream --steps 50 --warmup 10 --cpu-baseline off --no-profile-pass > gpurun_out/prof_${TAG}_stream.json && echo done
