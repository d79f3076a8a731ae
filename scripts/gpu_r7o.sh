# 262144^2 (configs[3]): quads (the plan) against two words per lane on the pair rule, alternating.
set -o pipefail
out=gpurun_out/r7o
mkdir -p $out
for i in 1 2; do
  for w in 0 2; do
    timeout -k 10 300 python bench.py --workload 262144 --steps 10 --no-cpu-baseline --no-configs3 $( [ $w = 2 ] && echo --option wpl=2 ) > $out/b262144_wpl$w.$i.json 2> $out/b262144_wpl$w.$i.err || { tail $out/b262144_wpl$w.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b262144_wpl$w.$i.json')); r=d['roofline']; print('wpl$w', d['value'], d['parity'], r['words_per_lane'], r['turns_per_launch'], r['avg_launch_ms'], r['frac'])"
  done
done
