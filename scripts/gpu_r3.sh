# usage: bash scripts/gpu_r3.sh <tag> [full|fullsize|smoke|bench|trace|pmc|strips]...
# GPU steps of a round-3 measurement session; each under its own time limit,
# chained: the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1
shift
out=gpurun_out/$tag
mkdir -p $out
PYT="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
  case $step in
    fullsize)
      timeout -k 10 600 $PYT tests/test_gpu_fullsize.py -m gpu -x > $out/pytest_fullsize.log 2>&1 || { echo "fullsize tests failed"; tail -40 $out/pytest_fullsize.log; exit 1; }
      tail -3 $out/pytest_fullsize.log ;;
    skew64)
      timeout -k 10 300 $PYT tests/test_gpu_skew.py -m gpu -x -k "6-4" > $out/pytest_skew64.log 2>&1 || { echo "skew (6,4) tests failed"; tail -40 $out/pytest_skew64.log; exit 1; }
      tail -2 $out/pytest_skew64.log ;;
    full)
      timeout -k 10 900 $PYT tests -m gpu -x > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
      tail -3 $out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
      cat $out/smoke.log ;;
    bench)
      timeout -k 10 300 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail $out/bench_default.err; cat $out/bench_default.json; exit 1; }
      cat $out/bench_default.json
      for wl in 16384 262144 5120; do
        timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --no-cpu-baseline > $out/bench_$wl.json 2> $out/bench_$wl.err || { tail $out/bench_$wl.err; cat $out/bench_$wl.json; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d.get('parity'), d['ms_per_step'])" $out/bench_$wl.json $wl
      done ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && for wl in 65536 16384 262144; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace_$wl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/trace_$wl.log 2>&1 || { tail $GRAFT_REPO_ROOT/$out/trace_$wl.log; exit 1; }
      done) || exit 1 ;;
    pmc)
      bash scripts/pmc_bench.sh $out || exit 1 ;;
    strips)
      timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x8192r,65536x16384r,65536x32768r,262144x32768r,16384x2048r" --sets "skew=1" > $out/strips.txt 2> $out/strips.err || { tail $out/strips.err; exit 1; }
      grep -A100 "^# best" $out/strips.txt ;;
    stripdiag)
      timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x8192,65536x8192r" --sets "skew=1;halo_skip=1;tb_depth=16;tb_depth=12;tb_depth=16,halo_skip=1" > $out/stripdiag.txt 2> $out/stripdiag.err || { tail $out/stripdiag.err; exit 1; }
      timeout -k 10 200 python -u scripts/sweep_opts.py --reps 1 --cases "65536x8192r,65536x8192" --sets "skew=1" > $out/stripdiag_timed.txt 2>> $out/stripdiag.err || { tail $out/stripdiag.err; exit 1; }
      grep -A100 "^# best" $out/stripdiag.txt; grep '^{' $out/stripdiag_timed.txt ;;
  esac
done
echo "gpu_r3 $tag done"
