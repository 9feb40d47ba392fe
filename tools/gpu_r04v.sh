# smoke() + the stream-path line after the bench fix.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04v}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -2 gpurun_out/${TAG}_smoke.log && \
timeout -k 10 200 python3 bench.py --path stream --cpu-baseline off > gpurun_out/${TAG}_bench_stream.json && \
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_stream.json')); print('stream', d['value'], d['ms_per_step'], d['kernels_ms'], d['workload']['alive_frac'])"
