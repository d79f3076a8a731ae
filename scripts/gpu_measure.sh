# Round measurements: bench lines, rocprofv3 kernel-trace summary, PMC traffic passes, event path.
# usage: bash scripts/gpu_measure.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail $out/bench_default.err; exit 1; }
cat $out/bench_default.json
timeout -k 10 300 python -u bench.py --workload 65536 --steps 5 --no-cpu-baseline > $out/bench_65536.json 2> $out/bench_65536.err || { tail $out/bench_65536.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload 262144 --steps 5 --no-cpu-baseline > $out/bench_262144.json 2> $out/bench_262144.err || { tail $out/bench_262144.err; exit 1; }
timeout -k 10 300 python -u scripts/bench_events.py > $out/events_5120.json 2> $out/events_5120.err || { tail $out/events_5120.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_default -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $out/trace_default.log 2>&1 || { tail $out/trace_default.log; exit 1; }
for wl in 65536 262144; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 5 --no-cpu-baseline > $out/trace_$wl.log 2>&1 || { tail $out/trace_$wl.log; exit 1; }
done
# the default step kernel of each size: resident K1p at 16384^2, per-launch paired K1 at 65536^2
for sz in 16384 65536 262144; do
  pers=$([ $sz -le 16384 ] && echo 1 || echo 0)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex gol_ -d $out/pmc_${sz}_$ctr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_step.py --size $sz --launches 5 --persistent $pers > $out/pmc_${sz}_$ctr.log 2>&1 || { tail $out/pmc_${sz}_$ctr.log; exit 1; }
  done
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex gol_ -d $out/pmc_${sz}_sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_step.py --size $sz --launches 10 --persistent $pers > $out/pmc_${sz}_sq.log 2>&1 || { tail $out/pmc_${sz}_sq.log; exit 1; }
done
echo measure-done
