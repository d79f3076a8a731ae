set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3l}
mkdir -p $out
L=game-of-life-distributed_amd/golhip
for rep in 1 2; do
for lib in libgolhip.so libgolhip_8416.so libgolhip_020c.so; do
  GOLHIP_LIB=$L/$lib timeout -k 10 200 python -u scripts/sweep_opts.py --no-timing --reps 1 --turns 2000 --cases "262144x32768r,65536x65536,65536x8192r,16384x16384" --sets "skew=1" >> $out/ab.txt 2> $out/ab.err || { tail $out/ab.err; exit 1; }
done
done
grep '"gcups"' $out/ab.txt | python3 -c "
import sys,json,collections
b=collections.defaultdict(list)
for l in sys.stdin:
    d=json.loads(l); b[(d['case'],d['lib'])].append(d['gcups'])
for k in sorted(b): print(k, b[k])
"
