# Kernel-lab timing on the GPU box (run under gpurun): VARIANTS (names of
# tools/kernel_lab.py builds) in the steady window, then in the driver's
# early window (5 warmup + 20 steps).  Lines into gpurun_out/${TAG}_lab.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-lab}
EARLY=""
for v in $VARIANTS; do EARLY="$EARLY $v@LAB_WARM=5,LAB_STEPS=20"; done
timeout -k 10 ${LIMIT:-500} python -u tools/kernel_lab.py run $VARIANTS $EARLY > gpurun_out/${TAG}_lab.jsonl 2> gpurun_out/${TAG}_lab.err
rc=$?
python3 - "$TAG" <<'PY'
import json, sys
for line in open(f"gpurun_out/{sys.argv[1]}_lab.jsonl"):
    d = json.loads(line)
    print(d["variant"], d["ms_per_step"], d["ms_per_step_1group"], d["kernels_1group"], d["digest"])
PY
exit $rc
