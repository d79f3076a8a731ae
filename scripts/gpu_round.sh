#!/bin/bash
# One GPU call: the whole GPU suite, the default bench line (configs[2] +
# configs3 + cpu baseline) and the events line, into gpurun_out/<tag>/.
# usage: scripts/gpu_round.sh <tag> [pytest-args...]
tag=${1:-run}; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests "$@" > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --workload 5120 --steps 5 > $out/bench_5120.json 2> $out/bench_5120.err || { echo "bench 5120 failed"; exit 1; }
echo done
