# K5 PMC passes of the configs[4] bench command, merged into the PMC summary, then the bench line with traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3s}
mkdir -p $out
bash scripts/pmc_bench.sh $out 5120 || exit 1
python3 - "$out" <<'PY' || exit 1
import json, sys
out = sys.argv[1]
new = json.load(open(f"{out}/pmc_bench.json"))
cur = json.load(open("profiles/pmc_bench.json"))
cur.update({k: v for k, v in new.items() if k.startswith("5120:")})
json.dump(cur, open(f"{out}/pmc_bench_merged.json", "w"), indent=1, sort_keys=True)
print({k: v.get("hbm_bytes_per_launch") for k, v in new.items()})
PY
timeout -k 10 300 python -u bench.py --workload 5120 --steps 5 --no-cpu-baseline --pmc $out/pmc_bench_merged.json > $out/bench_5120.json 2> $out/bench_5120.err || { tail $out/bench_5120.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_5120.json')); print(d['value'], d['parity'], d['roofline'])"
