set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3h}
mkdir -p $out
timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x8192,65536x65536" \
  --sets "skew=1;wpl=4;tb_depth=12;tb_depth=16;skew_tx=2;skew_young=64;skew_young=72;skew_hcap=10;skew_hcap=20" > $out/sweep.txt 2> $out/sweep.err || { tail $out/sweep.err; exit 1; }
grep -A100 "^# best" $out/sweep.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_ring -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/sweep_opts.py --no-timing --reps 1 --cases 65536x8192r --sets skew=1 > $out/trace_ring.log 2>&1 || { tail $out/trace_ring.log; exit 1; }
cut -d, -f1-5 $out/trace_ring/run_kernel_stats.csv | head -12
