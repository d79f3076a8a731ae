# final set, part 1: skew + split GPU tests (incl. K1w (6, 4)), smoke, bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r3l.sh ${1:-r3final} && bash scripts/gpu_r3.sh ${1:-r3final} smoke bench
