set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:?}
TAG=$T bash tools/gpu_round.sh bench && \
timeout -k 10 300 python3 tools/wire_timing.py > gpurun_out/${T}_wire_timing.json && cat gpurun_out/${T}_wire_timing.json
