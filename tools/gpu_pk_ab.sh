# Parity subset + lab A/B of the k_vis agent stage (lab/main = csrc, lab/nopk = without it).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04ag}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "golden or live or edge_cases or world_groups or stream or flank" > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 tools/kernel_lab.py run main nopk main@LAB_WARM=5,LAB_STEPS=20 nopk@LAB_WARM=5,LAB_STEPS=20 \
  main@LAB_ACTIONS=combat nopk@LAB_ACTIONS=combat > gpurun_out/${TAG}_lab.jsonl && \
python3 -c "
import json
for l in open('gpurun_out/${TAG}_lab.jsonl'):
    d=json.loads(l); k=d['kernels_1group']; print(d['variant'], d['ms_per_step'], k['k_vis'], k['k_lidar'], d['digest'])"
