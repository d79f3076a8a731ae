# A/B of libgolhip builds on one box: alternating sweeps of the default
# kernels per library (scripts/sweep.py), two rounds.
# usage: bash scripts/ab_libs.sh <out_dir> <sizes> <lib1> <lib2> ...
out=$1; sizes=$2; shift 2
mkdir -p $out
for round in 1 2; do
  for lib in "$@"; do
    GOLHIP_LIB=$lib timeout -k 10 200 python -u scripts/sweep.py --sizes $sizes --depths 16 --rpw 0 --variants "persistent=-1" --turns 2048 --repeats 2 > $out/tmp.jsonl 2>&1 || { cat $out/tmp.jsonl; exit 1; }
    python3 -c "
import json,sys
for l in open('$out/tmp.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); d['lib']='$(basename $lib)'; d['round']=$round; print(json.dumps(d))" >> $out/ab.jsonl
  done
done
