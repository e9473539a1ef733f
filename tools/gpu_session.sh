set -o pipefail
cd $GRAFT_REPO_ROOT
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_round.sh && TAG=${TAG:-r02e} bash tools/gpu_pmc.sh
