# half tiles with the corrected stack bound (16384^2 default vs forced variants); small boards: K1w vs the K1 fallback
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3i}
mkdir -p $out
timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --turns 2000 --cases "16384x16384" --sets "skew_half=0;skew_half=-1;skew_half=1,skew_nst=28;skew_half=1,skew_nst=30" > $out/half_16384.txt 2> $out/sweep.err || { tail $out/sweep.err; exit 1; }
grep -A100 "^# best" $out/half_16384.txt
timeout -k 10 400 python -u scripts/sweep_opts.py --no-timing --reps 2 --turns 2000 --cases "5120x5120,4096x4096,8192x8192,2048x2048" --sets "skew=1;skew=2;skew=2,wpl=2;skew=0,wpl=2;skew=0,wpl=1" > $out/small.txt 2>> $out/sweep.err || { tail $out/sweep.err; exit 1; }
grep -A100 "^# best" $out/small.txt
