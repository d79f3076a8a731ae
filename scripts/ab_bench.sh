# A/B of libgolhip builds on one box with whole bench.py lines (alternating, two rounds).
# usage: bash scripts/ab_bench.sh <out_dir> "<bench args>" <lib1> <lib2> ...
out=$1; args=$2; shift 2
mkdir -p $out
for round in 1 2; do
  for lib in "$@"; do
    GOLHIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $out/tmp.json 2> $out/tmp.err || { tail $out/tmp.err; exit 1; }
    python3 -c "
import json
d=json.load(open('$out/tmp.json')); r=d['roofline']
print(json.dumps(dict(lib='$lib', round=$round, args='$args', value=d['value'], ms_per_step=d['ms_per_step'], kernel=r['kernel'], avg_launch_ms=r['avg_launch_ms'], launches=r['launches'])))" | tee -a $out/ab.jsonl
  done
done
