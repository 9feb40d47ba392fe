# Lab: k_lidar task quads per block (kLidarIters 4 / 5 / 6 / 8) with the agent stage.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04au}
timeout -k 10 900 python3 tools/kernel_lab.py run hk4 hk5 hk6 hk8 hk4@LAB_WARM=5,LAB_STEPS=20 hk5@LAB_WARM=5,LAB_STEPS=20 \
  hk6@LAB_WARM=5,LAB_STEPS=20 hk8@LAB_WARM=5,LAB_STEPS=20 hk4@LAB_ACTIONS=combat hk5@LAB_ACTIONS=combat \
  hk6@LAB_ACTIONS=combat > gpurun_out/${TAG}_lab.jsonl && \
python3 -c "
import json
for l in open('gpurun_out/${TAG}_lab.jsonl'):
    d=json.loads(l); k=d['kernels_1group']; print(d['variant'], d['ms_per_step'], k['k_lidar'], d['digest'])"
