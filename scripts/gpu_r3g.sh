# kernel trace of an overlapped one-rank ring; instruction-fetch sharing probe (fewer CUs planned)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3g}
mkdir -p $out
timeout -k 10 300 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x65536,65536x32768,65536x16384" --sets "cu_count=0;cu_count=128;cu_count=64" > $out/cu_probe.txt 2> $out/cu_probe.err || { tail $out/cu_probe.err; exit 1; }
grep -A100 "^# best" $out/cu_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace_overlap -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/sweep_opts.py --no-timing --reps 1 --turns 400 --cases 65536x8192r --sets "overlap=1" > $out/trace_overlap.log 2>&1 || { tail $out/trace_overlap.log; exit 1; }
echo done
