# full GPU suite with per-test durations (the suite's length)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3o}
mkdir -p $out
timeout -k 10 1120 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests -m gpu -x --durations=60 > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -80 $out/pytest_gpu.log; exit 1; }
tail -75 $out/pytest_gpu.log
