set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3j}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_skew.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_skew.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_skew.log; exit 1; }
tail -2 $out/pytest_skew.log
for wl in 65536 16384 262144; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --no-cpu-baseline > $out/bench_$wl.json 2> $out/bench_$wl.err || { tail $out/bench_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['parity'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['launches'], r['frac'])" $out/bench_$wl.json $wl
done
timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x65536,65536x8192r,65536x16384r,262144x32768r" --sets "skew=1;skew_hcap=8;skew_hcap=24" > $out/sweep.txt 2> $out/sweep.err || { tail $out/sweep.err; exit 1; }
grep -A100 "^# best" $out/sweep.txt
