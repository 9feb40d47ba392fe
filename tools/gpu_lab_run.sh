# kernel_lab variants only (run under gpurun): VARIANTS="name name@ENV=V ...",
# output gpurun_out/${TAG}_lab.jsonl
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04x}
timeout -k 10 ${LAB_TIMEOUT:-600} python3 tools/kernel_lab.py run $VARIANTS > gpurun_out/${TAG}_lab.jsonl
