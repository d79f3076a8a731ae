# One parameterised GPU-box runner (replaces round 3's one-off gpu_r3*.sh).
# usage: bash scripts/gpu_run.sh <tag> <step> [step ...]
#   tests[:<pytest -k expr>]   GPU suite (or a subset; commas stand for spaces), one process
#   smoke                      __graft_entry__.smoke()
#   bench[:<workload>]         bench.py line (default workload 65536) -> bench_<wl>.json
#   trace[:<workload>]         rocprofv3 --kernel-trace --stats of that bench command
#   pmc[:<workload>]           FETCH / WRITE / SQ passes (scripts/pmc_bench.sh)
#   stalls[:<workload>]        SQ wait / active / instruction-mix passes (scripts/pmc_stalls.sh)
#   selflaunch                 bench.py --gpus 2 on this box (fewer devices than ranks: JSON error, exit 2)
#   py:<script args...>        any repo script, e.g. py:scripts/bench_strip.py (commas in
#                              the argument list stand for spaces)
# Every GPU step runs under its own time limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1
shift
out=gpurun_out/$tag
mkdir -p $out
for st in "$@"; do
  name=${st%%:*}
  arg=""
  [ "$name" != "$st" ] && arg=${st#*:}
  echo "== $st $(date +%T)"
  case $name in
    tests)
      k=()
      [ -n "$arg" ] && k=(-k "${arg//,/ }")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${k[@]}" \
        > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
      tail -3 $out/pytest.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
        || { tail $out/smoke.log; exit 1; }
      cat $out/smoke.log ;;
    bench)
      wl=${arg:-65536}
      timeout -k 10 400 python -u bench.py --workload $wl > $out/bench_$wl.json 2> $out/bench_$wl.err \
        || { tail $out/bench_$wl.err; cat $out/bench_$wl.json; exit 1; }
      python3 -c "import json; d=json.load(open('$out/bench_$wl.json')); print('$wl', d['value'], d['parity'], d.get('roofline', {}).get('avg_launch_ms'), d.get('roofline', {}).get('frac'))" ;;
    trace)
      wl=${arg:-65536}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace_$wl -o run \
        --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 5 --no-cpu-baseline \
        > $GRAFT_REPO_ROOT/$out/trace_$wl.log 2>&1) || { tail $out/trace_$wl.log; exit 1; }
      f=$(find $out/trace_$wl -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && cp $f $out/trace_${wl}_kernel_stats.csv && head -4 $out/trace_${wl}_kernel_stats.csv ;;
    pmc)
      bash scripts/pmc_bench.sh $out ${arg:-65536} || exit 1 ;;
    stalls)
      bash scripts/pmc_stalls.sh $out gol_ --workload ${arg:-65536} || exit 1 ;;
    selflaunch)
      # bench.py --gpus 2 without a launcher on a 1-GPU box: must fail fast with a JSON error line (exit 2)
      timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > $out/selflaunch.json 2> $out/selflaunch.err; rc=$?
      cat $out/selflaunch.json; [ $rc -eq 2 ] || { echo "selflaunch exit $rc"; exit 1; } ;;
    py)
      a=${arg//,/ }
      timeout -k 10 600 python -u $a > $out/py_$(basename ${a%% *} .py).log 2>&1 \
        || { tail -20 $out/py_$(basename ${a%% *} .py).log; exit 1; }
      tail -20 $out/py_$(basename ${a%% *} .py).log ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
