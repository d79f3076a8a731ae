# 262144^2 on the final launch plan: bench line, kernel trace, PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3t}
mkdir -p $out
timeout -k 10 300 python -u bench.py --workload 262144 --steps 5 --no-cpu-baseline > $out/bench_262144.json 2> $out/bench_262144.err || { tail $out/bench_262144.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_262144.json')); print(d['value'], d['parity'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace_262144 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload 262144 --steps 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/trace_262144.log 2>&1) || { tail $out/trace_262144.log; exit 1; }
bash scripts/pmc_bench.sh $out 262144 || exit 1
