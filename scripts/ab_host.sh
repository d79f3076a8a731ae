# A/B of host-mirror builds (libgolhost*.so via GOLHOST_LIB) on configs[0] end to end:
# alternating `bench.py --workload 512` runs, three rounds.
# usage: bash scripts/ab_host.sh <tag> <lib.so> <lib.so> ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
for r in 1 2 3; do
  for lib in "$@"; do
    GOLHOST_LIB=$GRAFT_REPO_ROOT/game-of-life-distributed_amd/golhip/$lib timeout -k 10 200 python -u bench.py --workload 512 \
      > gpurun_out/$tag/b_${lib}_$r.json 2> gpurun_out/$tag/b_${lib}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['ms_per_run_min'], d['buffered_1000']['ms_per_run'])" gpurun_out/$tag/b_${lib}_$r.json $lib
  done
done
