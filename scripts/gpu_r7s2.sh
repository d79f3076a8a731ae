# strip shares (one-rank rings) on the tree's default plan: the pair drain (round 6), two repetitions
set -o pipefail
mkdir -p gpurun_out/r7s2
for i in 1 2; do
  timeout -k 10 300 python scripts/bench_strip.py --turns 720 --strips 65536x8192,65536x16384,65536x32768,262144x32768 \
    --persistent 0 --depths 20 >> gpurun_out/r7s2/strip_pairs_drain.jsonl 2>> gpurun_out/r7s2/strip.err \
    || { tail gpurun_out/r7s2/strip.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/r7s2/strip_pairs_drain.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['strip'], round(d['gcups']), d.get('tb_depth'), d.get('words_per_lane'))
"
