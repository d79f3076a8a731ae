# PMC passes of the bench command itself (one counter group per pass), then the summary.
# usage: bash scripts/pmc_bench.sh <out dir under gpurun_out> [workloads...]
set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/$1
shift
wls=${@:-65536 16384 262144}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for wl in $wls; do
  # (--no-configs3: the default line's configs3 block would mix 262144^2 dispatches into 65536^2's)
  args="$GRAFT_REPO_ROOT/bench.py --workload $wl --steps 2 --warmup 1 --warmup-seconds 0 --no-cpu-baseline --no-configs3"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gol_ -d $out/pmc_${wl}_fetch -o run --output-format csv -- python3 $args > $out/pmc_${wl}_fetch.log 2>&1 || { tail $out/pmc_${wl}_fetch.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gol_ -d $out/pmc_${wl}_write -o run --output-format csv -- python3 $args > $out/pmc_${wl}_write.log 2>&1 || { tail $out/pmc_${wl}_write.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex gol_ -d $out/pmc_${wl}_sq -o run --output-format csv -- python3 $args > $out/pmc_${wl}_sq.log 2>&1 || { tail $out/pmc_${wl}_sq.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/scripts/pmc_bench.py $out $out/pmc_bench.json > $out/pmc_bench.log 2>&1 || { tail $out/pmc_bench.log; exit 1; }
echo pmc-done
