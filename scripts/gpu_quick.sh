# usage: bash scripts/gpu_quick.sh <tag> [pytest -k expr]   (subset of GPU tests + the 65536/262144 bench lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1
out=gpurun_out/$tag
mkdir -p $out
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$2" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
fi
timeout -k 10 200 python -u bench.py --workload 65536 --steps 5 --no-cpu-baseline > $out/bench_65536.json 2> $out/bench_65536.err || { tail $out/bench_65536.err; exit 1; }
timeout -k 10 200 python -u bench.py --workload 262144 --steps 5 --no-cpu-baseline > $out/bench_262144.json 2> $out/bench_262144.err || { tail $out/bench_262144.err; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_default.json 2> $out/bench_default.err || { tail $out/bench_default.err; exit 1; }
python - $out <<'PY'
import json, sys
for f in ("bench_default", "bench_65536", "bench_262144"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["launches"], r["frac"])
PY
