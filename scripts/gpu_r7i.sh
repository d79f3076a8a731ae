# configs[4]: the flip-stream event tests and fixture, the K5 probe, bench A/B
# of flip_overlap 2 / 1, and a kernel timeline of K5r.
# usage: bash scripts/gpu_r7i.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r7i}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_events.py tests/test_gpu_fullsize.py -k "pinned or flip_stream" -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
K5_MODES=resident,overlap,no_entries timeout -k 10 300 python scripts/k5_overlap_probe.py > $out/k5.jsonl 2> $out/k5.err || { tail $out/k5.err; exit 1; }
cat $out/k5.jsonl
for v in 2 1 2 1; do
  GOLHIP_TUNING=1 timeout -k 10 300 python bench.py --workload 5120 --steps 5 --no-cpu-baseline --e2e-turns 0 --option flip_overlap=$v > $out/bench_5120_ov$v.json 2> $out/bench_5120_ov$v.err || { tail $out/bench_5120_ov$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_5120_ov$v.json')); print($v, d['value'], d['parity'], d['events_on'], d['roofline']['avg_launch_ms'])"
done
cd /tmp && export TMPDIR=/tmp
K5_MODES=resident K5_UNTIMED=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/trace_resident -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/k5_overlap_probe.py > $GRAFT_REPO_ROOT/$out/trace_resident.log 2>&1 || { tail $GRAFT_REPO_ROOT/$out/trace_resident.log; exit 1; }
grep '^{' $GRAFT_REPO_ROOT/$out/trace_resident.log
