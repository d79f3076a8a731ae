# Round-4 K1w probe: per-wave load waits (diagnostic build) at three shapes, then the A/B of the candidate builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
AB=game-of-life-distributed_amd/golhip/ab
for c in 65536x65536 16384x16384 65536x8192r; do
  GOLHIP_LIB=$PWD/$AB/libgolhip_wt.so timeout -k 10 120 python -u scripts/trace_skew.py --case $c >> $out/wait_trace.jsonl 2> $out/wait_trace.err || { tail $out/wait_trace.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/wait_trace.jsonl'):
    d=json.loads(l); print(d['case'], d['span_us'], [(q['w'], q.get('dur_mean'), q.get('fill_us'), q.get('fill_wait_us'), q.get('main_us'), q.get('main_wait_us'), q.get('main_groups'), q.get('drain_us')) for q in d['positions']])"
bash scripts/gpu_ab.sh $(basename $out) "$@"
