set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:?}
timeout -k 10 600 python3 tools/kernel_lab.py run ${LAB_VARIANTS:?} > gpurun_out/${T}_lab.jsonl && \
python3 -c "import json
for l in open('gpurun_out/${T}_lab.jsonl'):
    d=json.loads(l); print(d['variant'], d['ms_per_step'], d['digest'], d['kernels_1group'])"
