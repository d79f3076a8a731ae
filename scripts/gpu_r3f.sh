# exchange overlap (option "overlap"): parity tests, A/B on one-rank-ring strips, kernel trace of an overlapped ring
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3f}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_skew.py -k "overlap or rccl_ring" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_overlap.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_overlap.log; exit 1; }
tail -2 $out/pytest_overlap.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "rccl_ring" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest_fullsize_ring.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_fullsize_ring.log; exit 1; }
tail -2 $out/pytest_fullsize_ring.log
timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 3 --cases "65536x8192r,65536x16384r,262144x32768r" --sets "overlap=0;overlap=1;halo_skip=1" > $out/overlap_ab.txt 2> $out/overlap_ab.err || { tail $out/overlap_ab.err; exit 1; }
grep -A100 "^# best" $out/overlap_ab.txt
timeout -k 10 200 python -u scripts/sweep_opts.py --reps 1 --cases "65536x8192r" --sets "overlap=0;overlap=1" > $out/overlap_timed.txt 2>> $out/overlap_ab.err || { tail $out/overlap_ab.err; exit 1; }
grep '^{' $out/overlap_timed.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace_overlap -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/sweep_opts.py --no-timing --reps 1 --turns 400 --cases 65536x8192r --sets "overlap=1" > $GRAFT_REPO_ROOT/$out/trace_overlap.log 2>&1 || { tail $GRAFT_REPO_ROOT/$out/trace_overlap.log; exit 1; }

# instruction-fetch sharing probe: the same per-wave work on all CUs vs half / a quarter of them
timeout -k 10 300 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x65536,65536x32768,65536x16384" --sets "cu_count=0;cu_count=128;cu_count=64" > $GRAFT_REPO_ROOT/$out/cu_probe.txt 2>> $GRAFT_REPO_ROOT/$out/overlap_ab.err || { tail $GRAFT_REPO_ROOT/$out/overlap_ab.err; exit 1; }
grep -A100 "^# best" $GRAFT_REPO_ROOT/$out/cu_probe.txt
echo done
