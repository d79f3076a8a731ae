# depth plan A/B at 262144^2 x 100 (exact plan of the last 12 caps vs the last 3); fullsize c3 test; bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3m}
mkdir -p $out
L=game-of-life-distributed_amd/golhip
for rep in 1 2 3; do
for lib in libgolhip.so libgolhip_plan3.so; do
  GOLHIP_LIB=$L/$lib timeout -k 10 200 python -u scripts/sweep_opts.py --no-timing --reps 1 --turns 100 --cases "262144x262144" --sets "skew=1" >> $out/ab_plan.txt 2>> $out/ab_plan.err || { tail $out/ab_plan.err; exit 1; }
done
done
grep '"gcups"' $out/ab_plan.txt | python3 -c "
import sys,json,collections
b=collections.defaultdict(list)
for l in sys.stdin:
    d=json.loads(l); b[(d['case'],d['lib'])].append((d['gcups'], d['launches']))
for k in sorted(b): print(k, b[k])
"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py -k "config3" -x > $out/pytest_c3.log 2>&1 || { tail -30 $out/pytest_c3.log; exit 1; }
tail -2 $out/pytest_c3.log
timeout -k 10 300 python -u bench.py --workload 262144 --steps 5 --no-cpu-baseline > $out/bench_262144.json 2> $out/bench_262144.err || { tail $out/bench_262144.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_262144.json')); print(d['value'], d['parity'], d['roofline']['avg_launch_ms'], d['roofline']['launches'])"
