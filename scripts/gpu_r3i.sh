set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3i}
bash scripts/pmc_skew.sh $out 65536x65536 65536x8192 16384x16384
