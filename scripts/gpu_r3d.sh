set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3d}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_run.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_run.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_run.log; exit 1; }
tail -2 $out/pytest_run.log
bash scripts/gpu_r3c.sh ${1:-r3d}
timeout -k 10 300 python -u bench.py --workload 5120 --steps 3 > $out/bench_5120.json 2> $out/bench_5120.err || { tail $out/bench_5120.err; exit 1; }
cat $out/bench_5120.json
bash scripts/gpu_r3e.sh ${1:-r3d}
