set -o pipefail
cd $GRAFT_REPO_ROOT
sed -n '/^cd \/tmp/,$p' scripts/gpu_r3f.sh > /tmp/r3g_body.sh
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3g}
mkdir -p $out
export out
bash -c "out=$out; $(cat /tmp/r3g_body.sh)"
