# Quick GPU iteration (run under gpurun): a parity subset, then the default
# and the 20-step bench lines without the CPU baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread \
    -k "${TESTS:-6v6x16_f0 or 5v5x13 or bots_all or golden or bvh_traversal or C3}" > gpurun_out/gpu_quick.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-baseline off > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err
rc=$?
tail -2 gpurun_out/gpu_quick.log
python3 - <<'PY'
import json
for f in ("gpurun_out/bench.json", "gpurun_out/bench_short.json"):
    try:
        d = json.load(open(f))
        print(f, d["value"] / 1e6, "M", d["ms_per_step"], "ms", d.get("kernels_ms"))
    except Exception as e:
        print(f, "n/a", e)
PY
exit $rc
