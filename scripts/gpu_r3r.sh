# 16384^2 on half-wave tiles: depth and band-weight options
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3r}
mkdir -p $out
timeout -k 10 500 python -u scripts/sweep_opts.py --no-timing --reps 2 --turns 4000 --cases "16384x16384" --sets "skew=1;tb_depth=16;skew_young=60;skew_young=78;skew_hcap=20;skew_hcap=12;skew_tx=2" > $out/opts_16384.txt 2> $out/opts.err || { tail $out/opts.err; exit 1; }
grep -A100 "^# best" $out/opts_16384.txt
