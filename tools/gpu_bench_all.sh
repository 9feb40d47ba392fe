# Round 4 bench lines + profiles (run under gpurun): default, driver window,
# combat, gpuStreamStep path, wire exchange (one-rank loopback), then the
# rocprof kernel trace + PMC passes for the tape and combat workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04m}
B="timeout -k 10 300 python3 bench.py"
$B --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/${TAG}_bench_short.json && \
$B > gpurun_out/${TAG}_bench.json && \
$B --actions combat --cpu-baseline off > gpurun_out/${TAG}_bench_combat.json && \
$B --path stream --cpu-baseline off > gpurun_out/${TAG}_bench_stream.json && \
$B --exchange wire --cpu-baseline off > gpurun_out/${TAG}_bench_wire.json && \
$B --actions combat --world-groups 3 --cpu-baseline off --no-profile-pass > gpurun_out/${TAG}_bench_combat_g3.json && \
$B --actions combat --world-groups 4 --cpu-baseline off --no-profile-pass > gpurun_out/${TAG}_bench_combat_g4.json || exit $?
for f in bench_short bench bench_combat bench_stream bench_wire bench_combat_g3 bench_combat_g4; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('kernels_ms'))" $f
done
[ -n "$NOPROF" ] && exit 0
bash tools/profile_round.sh ${TAG} > /dev/null && \
BENCH_ARGS="--actions combat" bash tools/profile_round.sh ${TAG}_combat > /dev/null && echo profiles done
