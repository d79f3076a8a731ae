set -o pipefail
mkdir -p gpurun_out/r7c
bash scripts/ab_pairs.sh 2 16384 5 > gpurun_out/r7c/ab_half.log 2>&1 || { tail gpurun_out/r7c/ab_half.log; exit 1; }
tail -4 gpurun_out/r7c/ab_half.log
for v in 1 0; do
  timeout -k 10 300 python scripts/bench_strip.py --turns 720 --strips 65536x8192,65536x16384,65536x32768,262144x32768 --persistent 0 --depths 20 --option skew_pairs=$v > gpurun_out/r7c/strip_pairs$v.jsonl 2> gpurun_out/r7c/strip_pairs$v.err || { tail gpurun_out/r7c/strip_pairs$v.err; exit 1; }
  cat gpurun_out/r7c/strip_pairs$v.jsonl | cut -c1-300
done
