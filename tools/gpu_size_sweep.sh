# Per-kernel time against batch size (tail / wave-quantisation check): the
# bench's exclusive per-kernel times at 2/3 and 1/2 of the C3 batch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04al}
for W in 16384 10923 8192 12288; do
  timeout -k 10 200 python3 bench.py --worlds $W --steps 200 --warmup 100 --cpu-baseline off > gpurun_out/${TAG}_w$W.json || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_w'+sys.argv[1]+'.json')); print(sys.argv[1], d['ms_per_step'], d.get('kernels_ms'))" $W
done
