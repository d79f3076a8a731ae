set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3c}
mkdir -p $out
timeout -k 10 600 python -u scripts/sweep_opts.py --reps 2 --cases "65536x65536,65536x8192r,65536x8192,16384x16384" \
  --sets "skew=0;skew_young=62;skew_young=66;skew_young=70;skew_young=74;skew_young=78;skew_young=66,skew_hcap=8;skew_young=66,skew_hcap=24" \
  > $out/sweep2.txt 2> $out/sweep2.err || { tail $out/sweep2.err; exit 1; }
grep -A100 "^# best" $out/sweep2.txt
timeout -k 10 600 python -u scripts/sweep_opts.py --reps 2 --turns 100 --cases "262144x262144,262144x32768r" \
  --sets "skew=0;skew_young=70;skew_young=76;skew_young=82;skew_young=88" \
  > $out/sweep3.txt 2> $out/sweep3.err || { tail $out/sweep3.err; exit 1; }
grep -A100 "^# best" $out/sweep3.txt
