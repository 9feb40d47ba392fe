# A/B: captured step graph vs direct launches, alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04y}
run() { timeout -k 10 200 python3 bench.py "$@" --cpu-baseline off --no-profile-pass; }
for k in 1 2 3; do
  run --steps 20 --warmup 5 > gpurun_out/${T}_short_graph_$k.json && \
  MPENV_STEP_GRAPH=0 run --steps 20 --warmup 5 > gpurun_out/${T}_short_direct_$k.json && \
  run --steps 300 --warmup 100 > gpurun_out/${T}_steady_graph_$k.json && \
  MPENV_STEP_GRAPH=0 run --steps 300 --warmup 100 > gpurun_out/${T}_steady_direct_$k.json || exit $?
done
for f in gpurun_out/${T}_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'])" $f; done
