set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3b}
mkdir -p $out
timeout -k 10 500 python -u scripts/sweep_opts.py --reps 2 --cases "65536x65536,65536x8192r,16384x16384" \
  --sets "skew=0;skew=1;skew_young=85;skew_young=70;skew_prio=1;skew_prio=1,skew_young=115;skew_hcap=0;skew_hcap=30;skew_tx=2;tb_depth=16" \
  > $out/sweep1.txt 2> $out/sweep1.err || { tail $out/sweep1.err; exit 1; }
grep -A100 "^# best" $out/sweep1.txt
for c in 65536x65536 65536x8192r 16384x16384 262144x262144; do
  for o in "" "--opt skew_prio=1" "--opt skew_young=80"; do
    timeout -k 10 120 python -u scripts/trace_skew.py --case $c $o >> $out/trace_skew.jsonl 2>> $out/trace_skew.err || { tail $out/trace_skew.err; exit 1; }
  done
done
cat $out/trace_skew.jsonl
