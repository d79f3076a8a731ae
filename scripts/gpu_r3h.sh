# half-wave tiles: parity tests, then 16384^2 / 5120^2 option sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3h}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_skew.py -k "half_tiles_rccl" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_half.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|assert" $out/pytest_half.log | tail -30; exit 1; }
tail -3 $out/pytest_half.log
timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --turns 2000 --cases "16384x16384" --sets "skew_half=-1;skew_half=1;skew_half=1,skew_nst=28;skew_half=1,skew_nst=28,skew_hcap=8;skew_half=1,skew_hcap=8;skew_half=-1,skew_hcap=8;skew_half=1,skew_nst=28,skew_hcap=4" > $out/half_16384.txt 2> $out/half.err || { tail $out/half.err; exit 1; }
grep -A100 "^# best" $out/half_16384.txt
timeout -k 10 300 python -u scripts/sweep_opts.py --no-timing --reps 2 --turns 2000 --cases "5120x5120" --sets "skew=1;skew=2,skew_half=-1,wpl=2;skew=2,skew_half=1,wpl=2" > $out/half_5120.txt 2>> $out/half.err || { tail $out/half.err; exit 1; }
grep -A100 "^# best" $out/half_5120.txt
