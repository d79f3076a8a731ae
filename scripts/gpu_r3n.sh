# K1w options on the 8192-row share of configs[2] at 8 GPUs (one-rank ring)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3n}
mkdir -p $out
timeout -k 10 500 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x8192r" --sets "skew=1;skew_tx=2;skew_young=60;skew_young=78;skew_hcap=10;skew_hcap=20;tb_depth=16;skew_young=78,skew_hcap=20" > $out/strip_opts.txt 2> $out/strip_opts.err || { tail $out/strip_opts.err; exit 1; }
grep -A100 "^# best" $out/strip_opts.txt
