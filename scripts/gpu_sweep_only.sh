# usage: bash scripts/gpu_sweep_only.sh <tag> [sweep args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u scripts/sweep.py "$@" > gpurun_out/$tag/sweep.jsonl 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/$tag/sweep.jsonl; exit 1; }
