# store-policy libs and timing-event cost (A/B, alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3e}
mkdir -p $out
for rep in 1 2; do
  for lib in libgolhip.so libgolhip_sc1.so libgolhip_nt.so; do
    GOLHIP_LIB=$GRAFT_REPO_ROOT/game-of-life-distributed_amd/golhip/$lib timeout -k 10 200 python -u scripts/sweep_opts.py --reps 1 --cases "65536x65536,16384x16384,65536x8192" --sets "skew_young=68" >> $out/storepol.txt 2>> $out/storepol.err || { tail $out/storepol.err; exit 1; }
  done
  timeout -k 10 200 python -u scripts/sweep_opts.py --reps 1 --no-timing --cases "65536x65536,16384x16384,65536x8192" --sets "skew_young=68" >> $out/notiming.txt 2>> $out/notiming.err || { tail $out/notiming.err; exit 1; }
done
grep '^{' $out/storepol.txt $out/notiming.txt | python3 -c "
import json,sys,collections
best=collections.defaultdict(float)
for l in sys.stdin:
    f,j=l.split(':',1); d=json.loads(j); k=(d['case'],d['lib'],'notiming' in f); best[k]=max(best[k],d['gcups'])
for k,v in sorted(best.items()): print(k, round(v,1))
"
