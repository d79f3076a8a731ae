# skew tests, bench lines (no per-launch events), kernel traces, store policy A/B without events
set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3f}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_skew.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_skew.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_skew.log; exit 1; }
tail -2 $out/pytest_skew.log
for wl in 65536 16384 262144; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --no-cpu-baseline > $out/bench_$wl.json 2> $out/bench_$wl.err || { tail $out/bench_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['parity'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['launches'], r['frac'])" $out/bench_$wl.json $wl
done
cd /tmp && export TMPDIR=/tmp
for wl in 65536 16384; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 3 --warmup-seconds 0.5 --no-cpu-baseline > $out/trace_$wl.log 2>&1 || { tail $out/trace_$wl.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for lib in libgolhip.so libgolhip_sc1.so; do
    GOLHIP_LIB=$GRAFT_REPO_ROOT/game-of-life-distributed_amd/golhip/$lib timeout -k 10 200 python -u scripts/sweep_opts.py --no-timing --reps 1 --cases "65536x65536,16384x16384,65536x8192,65536x8192r,262144x32768r" --sets "skew=1" >> $out/storepol.txt 2>> $out/storepol.err || { tail $out/storepol.err; exit 1; }
  done
done
grep '^{' $out/storepol.txt | python3 -c "
import json,sys,collections
best=collections.defaultdict(float)
for l in sys.stdin:
    d=json.loads(l); k=(d['case'],d['lib']); best[k]=max(best[k],d['gcups'])
for k,v in sorted(best.items()): print(k, round(v,1))
"
