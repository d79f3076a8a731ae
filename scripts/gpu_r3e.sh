# exact K1w fill: skew parity tests, A/B against the phase-loop fill (alternating libraries), phase traces
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3e}
mkdir -p $out
L=game-of-life-distributed_amd/golhip
timeout -k 10 500 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_skew.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_skew.log; exit 1; }
tail -2 $out/pytest_skew.log
for rep in 1 2; do
for lib in libgolhip.so libgolhip_phfill.so; do
  GOLHIP_LIB=$L/$lib timeout -k 10 200 python -u scripts/sweep_opts.py --no-timing --reps 1 --turns 1000 --cases "65536x65536,65536x8192,65536x8192r,16384x16384,262144x32768r" --sets "skew=1" >> $out/ab.txt 2>> $out/ab.err || { tail $out/ab.err; exit 1; }
done
done
grep '"gcups"' $out/ab.txt | python3 -c "
import sys,json,collections
b=collections.defaultdict(list)
for l in sys.stdin:
    d=json.loads(l); b[(d['case'],d['lib'])].append(d['gcups'])
for k in sorted(b): print(k, b[k])
"
for c in 65536x8192 16384x16384; do
  timeout -k 10 120 python -u scripts/trace_skew.py --case $c >> $out/trace_skew.jsonl 2>> $out/trace_skew.err || { tail $out/trace_skew.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/trace_skew.jsonl'):
    d=json.loads(l); print(d['case'], round(d['launch_ms_event']*1e3,1), 'span', round(d['span_us'],1), [(p['w'], p['dur_mean'], p.get('fill_us'), p.get('main_us'), p.get('drain_us')) for p in d['positions']])
"
