# round 3, first K1w measurements: skew parity tests, bench lines skew on/off, strip shares
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3a}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_skew.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_skew.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_skew.log; exit 1; }
tail -2 $out/pytest_skew.log
B="timeout -k 10 200 python -u bench.py --steps 5 --no-cpu-baseline --warmup-seconds 1"
for args in "--workload 65536" "--workload 65536 --option skew=0" "--workload 16384 --steps 2" "--workload 16384 --steps 2 --option persistent=1" "--workload 262144" "--workload 262144 --option skew=0"; do
  tag=$(echo $args | tr ' =-' '___')
  $B $args > $out/bench$tag.json 2> $out/bench$tag.err || { tail $out/bench$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['parity'], r['kernel'], r['avg_launch_ms'], r['launches'], r['frac'])" $out/bench$tag.json "$args"
done
timeout -k 10 300 python -u scripts/bench_strip.py --strips 65536x8192,65536x16384,262144x32768 --persistent 0 --depths 20 > $out/strip_skew.jsonl 2> $out/strip_skew.err || { tail $out/strip_skew.err; exit 1; }
timeout -k 10 300 python -u scripts/bench_strip.py --strips 65536x8192,262144x32768 --persistent -1,0 --depths 20 --option skew=0 > $out/strip_noskew.jsonl 2> $out/strip_noskew.err || { tail $out/strip_noskew.err; exit 1; }
cat $out/strip_skew.jsonl $out/strip_noskew.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['strip'], d['persistent'], d['options'], round(d['gcups']), d['skew_launches'], d['persist_launches'], d['step_launches'])"
