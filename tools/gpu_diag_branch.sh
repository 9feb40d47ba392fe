# Diagnose the lidar-branch crash: serial, branch without graph, branch with graph.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --no-profile-pass"
MPENV_LIDAR_BRANCH=0 $B > gpurun_out/diag_serial.json && echo serial ok && \
MPENV_STEP_GRAPH=0 $B > gpurun_out/diag_branch_nograph.json && echo branch-nograph ok && \
$B > gpurun_out/diag_branch_graph.json && echo branch-graph ok
