# usage: bash scripts/gpu_test_and_sweep.sh <tag> [sweep args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -2 gpurun_out/$tag/pytest.log
timeout -k 10 400 python -u scripts/sweep.py "$@" > gpurun_out/$tag/sweep.jsonl 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/$tag/sweep.jsonl; exit 1; }
