# Forward-fan candidate lists lab (run under gpurun): kernel_lab timings of
# the tools/lab/fan_lists.patch build ("fanlists") against the product
# ("main"), tape and combat, plus VARIANTS (e.g. a fan_phases.patch build).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r04h}
timeout -k 10 600 python3 tools/kernel_lab.py run main main@LAB_ACTIONS=combat fanlists fanlists@LAB_ACTIONS=combat \
    ${VARIANTS:-} > gpurun_out/${TAG}_lab.jsonl
