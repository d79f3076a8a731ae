#!/bin/bash
# A/B of a skew_pairs value against the default plan on one bench workload,
# alternating runs.
# usage: scripts/ab_pairs.sh [reps] [workload] [skew_pairs value]
reps=${1:-3}; wl=${2:-65536}; v=${3:-1}
mkdir -p gpurun_out/ab_pairs
for i in $(seq 1 $reps); do
  timeout -k 10 200 python bench.py --workload $wl --steps 10 --no-cpu-baseline --no-configs3 > gpurun_out/ab_pairs/base_$wl.$i.json || exit 1
  GOLHIP_TUNING=1 timeout -k 10 200 python bench.py --workload $wl --steps 10 --no-cpu-baseline --no-configs3 --option skew_pairs=$v > gpurun_out/ab_pairs/pairs${v}_$wl.$i.json || exit 1
done
for f in gpurun_out/ab_pairs/*_$wl.*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['parity'], d['roofline']['avg_launch_ms'])"; done
