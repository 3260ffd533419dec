# Full GPU suite into gpurun_out/$1/pytest.log (run from the repo root on the GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$1; mkdir -p gpurun_out/$D
shift
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s "$@" > gpurun_out/$D/pytest.log 2>&1
