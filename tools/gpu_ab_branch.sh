# A/B: lidar branch streams launched directly (no graph) vs the serial
# per-group order replayed from the captured graph.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04x}
run() { timeout -k 10 200 python3 bench.py "$@" --cpu-baseline off --no-profile-pass; }
MPENV_LIDAR_BRANCH=0 run --steps 20 --warmup 5 > gpurun_out/${T}_short_serial_graph.json && \
MPENV_STEP_GRAPH=0 run --steps 20 --warmup 5 > gpurun_out/${T}_short_branch_nograph.json && \
MPENV_LIDAR_BRANCH=0 MPENV_STEP_GRAPH=0 run --steps 20 --warmup 5 > gpurun_out/${T}_short_serial_nograph.json && \
MPENV_LIDAR_BRANCH=0 run > gpurun_out/${T}_steady_serial_graph.json && \
MPENV_STEP_GRAPH=0 run > gpurun_out/${T}_steady_branch_nograph.json && \
MPENV_LIDAR_BRANCH=0 run --actions combat > gpurun_out/${T}_combat_serial_graph.json && \
MPENV_STEP_GRAPH=0 run --actions combat > gpurun_out/${T}_combat_branch_nograph.json || exit $?
for f in short_serial_graph short_branch_nograph short_serial_nograph steady_serial_graph steady_branch_nograph combat_serial_graph combat_branch_nograph; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" $f
done
