# Bench lines (run under gpurun): default window, the driver's short window,
# and the same with three world groups.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err && \
timeout -k 10 300 python -u bench.py --world-groups 3 --cpu-baseline off > gpurun_out/bench_g3.json 2> gpurun_out/bench_g3.err && \
timeout -k 10 300 python -u bench.py --world-groups 3 --cpu-baseline off --steps 20 --warmup 5 > gpurun_out/bench_g3_short.json 2> gpurun_out/bench_g3_short.err && \
cat gpurun_out/bench*.json
