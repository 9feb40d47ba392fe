# Wire exchange check: the wire GPU tests (incl. LearnerWire loopback on an
# explicit stream), smoke, then the one-rank wire bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04ai}
timeout -k 10 400 python -u -m pytest tests/test_wire_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -2 gpurun_out/${TAG}_smoke.log && \
timeout -k 10 300 python3 bench.py --exchange wire --cpu-baseline off > gpurun_out/${TAG}_bench_wire.json && \
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_wire.json')); print('wire', d['value'], d['ms_per_step'])"
