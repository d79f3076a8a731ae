# the resident-timeout tests, then the rest of the GPU suite after test_gpu_events.py
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3k}
mkdir -p $out
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 200 $PYT tests/test_gpu_events.py -k "persistent_timeout" -x > $out/pytest_timeout.log 2>&1 || { echo "timeout tests failed"; tail -30 $out/pytest_timeout.log; exit 1; }
tail -2 $out/pytest_timeout.log
timeout -k 10 1000 $PYT tests -m gpu -x --deselect tests/test_gpu_events.py > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
