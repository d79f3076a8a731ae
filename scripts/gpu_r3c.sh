# per-wave K1w traces at strip sizes vs the whole board; one-rank-ring timeout tests
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3c}
mkdir -p $out
for c in 65536x8192 65536x65536 16384x16384; do
  for o in ""; do
    timeout -k 10 120 python -u scripts/trace_skew.py --case $c $o >> $out/trace_skew.jsonl 2>> $out/trace_skew.err || { tail $out/trace_skew.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$out/trace_skew.jsonl'):
    d=json.loads(l); print(d['case'], d['opts'], round(d['launch_ms_event']*1e3,1), 'span', round(d['span_us'],1), 'start', round(d['start_spread_us'],1), 'idle', round(d['wg_idle_frac'],3), [(p['w'], p['dur_mean'], p.get('fill_us'), p.get('main_us'), p.get('drain_us')) for p in d['positions']])
"
