set -o pipefail
cd $GRAFT_REPO_ROOT
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_round.sh && TAG=r02a bash tools/gpu_pmc.sh
