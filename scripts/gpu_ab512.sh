# configs[0] and configs[4] end to end through the gol.Run mirror: flip_overlap 2 (K5r) against 1, alternating.
set -o pipefail
out=gpurun_out/${1:-ab512}
mkdir -p $out
for i in 1 2; do
  for v in 2 1; do
    GOLHIP_TUNING=1 GOLHIP_FLIP_OVERLAP=$v timeout -k 10 300 python bench.py --workload 512 --steps 3 --no-cpu-baseline > $out/b512_ov$v.$i.json 2> $out/b512_ov$v.$i.err || { tail $out/b512_ov$v.$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b512_ov$v.$i.json')); print('512', $v, d['value'], d['ms_per_step'], d['buffered_1000'])"
  done
done
