# GPU tests from test_gpu_parity.py on (the files before it passed in r3k)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3l}
mkdir -p $out
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 1000 $PYT tests/test_gpu_skew.py tests/test_gpu_split.py -m gpu -x > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
