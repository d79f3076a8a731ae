#!/bin/bash
# A/B of the pair rule (skew_pairs) on the default bench, alternating runs.
# usage: scripts/ab_pairs.sh [reps] [workload]
reps=${1:-3}; wl=${2:-65536}
mkdir -p gpurun_out/ab_pairs
for i in $(seq 1 $reps); do
  timeout -k 10 200 python bench.py --workload $wl --steps 10 --no-cpu-baseline --no-configs3 > gpurun_out/ab_pairs/base_$wl.$i.json || exit 1
  GOLHIP_TUNING=1 timeout -k 10 200 python bench.py --workload $wl --steps 10 --no-cpu-baseline --no-configs3 --option skew_pairs=1 > gpurun_out/ab_pairs/pairs_$wl.$i.json || exit 1
done
