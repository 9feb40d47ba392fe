set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG}_o bash tools/r06o.sh && \
TAG=${TAG}_lab LAB_VARIANTS="base vislt base@LAB_ACTIONS=combat vislt@LAB_ACTIONS=combat" bash tools/r06g.sh
