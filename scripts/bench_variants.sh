# Whole bench lines for several argument sets on one box (one JSON summary line each).
# usage: bash scripts/bench_variants.sh <out.jsonl> "<args 1>" "<args 2>" ...
out=$1; shift
mkdir -p $(dirname $out)
for args in "$@"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $out.tmp.json 2> $out.tmp.err || { tail $out.tmp.err; exit 1; }
  python3 - "$args" "$out.tmp.json" <<'PY' | tee -a $out
import json, sys
d = json.load(open(sys.argv[2])); r = d["roofline"]
print(json.dumps(dict(args=sys.argv[1], value=d["value"], parity=d["parity"], kernel=r["kernel"],
                      avg_launch_ms=r["avg_launch_ms"], launches=r["launches"], split=r.get("split_launches"),
                      frac=r["frac"], hbm=(r.get("hbm") or {}).get("frac"))))
PY
done
