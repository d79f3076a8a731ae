# configs[4] A/B: flip_overlap 2 (K5r) against 1, alternating; bench lines into gpurun_out/<tag>/.
set -o pipefail
out=gpurun_out/${1:-ab5120}
mkdir -p $out
for i in 1 2; do
  for v in 2 1; do
    GOLHIP_TUNING=1 timeout -k 10 300 python bench.py --workload 5120 --steps 10 --no-cpu-baseline --e2e-turns 0 --option flip_overlap=$v > $out/bench_5120_ov$v.$i.json 2> $out/bench_5120_ov$v.$i.err || { tail $out/bench_5120_ov$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/bench_5120_ov$v.$i.json')); r=d['roofline']; print($v, d['value'], d['parity'], d['events_on']['turns_per_s'], r['avg_launch_ms'], r['frac'], r['frac_vs_list_size_probe'])"
  done
done
