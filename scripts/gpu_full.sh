# usage: bash scripts/gpu_full.sh <tag>   (GPU parity tests, then the measurement set)
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -2 gpurun_out/$tag/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || { cat gpurun_out/$tag/smoke.log; exit 1; }
cat gpurun_out/$tag/smoke.log
timeout -k 10 60 bash scripts/box_info.sh > gpurun_out/$tag/box.txt 2>&1
bash scripts/gpu_measure.sh $tag
