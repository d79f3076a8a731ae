# configs[4] A/B of K5r's copy-block groups (GOLHIP_FLIP_CP_GROUPS), alternating; bench lines into gpurun_out/<tag>/.
# usage: bash scripts/gpu_ab_cpg.sh <tag> <groups...>
set -o pipefail
out=gpurun_out/${1:-abcpg}
shift
mkdir -p $out
for i in 1 2; do
  for v in "$@"; do
    GOLHIP_TUNING=1 GOLHIP_FLIP_CP_GROUPS=$v timeout -k 10 300 python bench.py --workload 5120 --steps 10 --no-cpu-baseline --e2e-turns 0 > $out/bench_5120_g$v.$i.json 2> $out/bench_5120_g$v.$i.err || { tail $out/bench_5120_g$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/bench_5120_g$v.$i.json')); r=d['roofline']; print($v, d['value'], d['parity'], d['events_on']['turns_per_s'], r['avg_launch_ms'], r['frac'], r['frac_vs_list_size_probe'])"
  done
done
