# final set, part 2: K1w (6, 4) tail A/B at 262144^2, strip shares, kernel traces, PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3final}
mkdir -p $out
L=game-of-life-distributed_amd/golhip
for rep in 1 2; do
for lib in libgolhip.so libgolhip_no64.so; do
  GOLHIP_LIB=$L/$lib timeout -k 10 200 python -u scripts/sweep_opts.py --no-timing --reps 1 --turns 100 --cases "262144x262144" --sets "skew=1" >> $out/ab64.txt 2>> $out/ab64.err || { tail $out/ab64.err; exit 1; }
done
done
grep '"gcups"' $out/ab64.txt | python3 -c "
import sys,json,collections
b=collections.defaultdict(list)
for l in sys.stdin:
    d=json.loads(l); b[(d['case'],d['lib'])].append(d['gcups'])
for k in sorted(b): print(k, b[k])
"
bash scripts/gpu_r3.sh ${1:-r3final} strips trace pmc
