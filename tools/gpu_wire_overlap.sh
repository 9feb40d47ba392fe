# LearnerWire's unpack stream: the loopback parity test, then the one-rank
# wire line with the unpacks on their own stream and serial on the step stream.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04aj}
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -x -v -s --timeout 240 --timeout-method thread -k "loopback or rejects" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
B="timeout -k 10 300 python3 bench.py --exchange wire --cpu-baseline off"
$B > gpurun_out/${TAG}_bench_wire.json && \
$B --wire-serial --no-profile-pass > gpurun_out/${TAG}_bench_wire_serial.json && \
$B --steps 20 --warmup 5 --no-profile-pass > gpurun_out/${TAG}_bench_wire_short.json || exit $?
for f in bench_wire bench_wire_serial bench_wire_short; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" $f
done
