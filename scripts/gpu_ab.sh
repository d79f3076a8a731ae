# A/B of a candidate libgolhip build against the tree's build on one box:
# the candidate's K1w parity tests, alternating whole-case timings
# (scripts/ab_builds.py), and optionally its SQ stall passes.
# usage: bash scripts/gpu_ab.sh <tag> <candidate .so> [cases] [stalls]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1; cand=$(readlink -f $2); cases=${3:-65536x65536,16384x16384,65536x8192r}
out=gpurun_out/$tag
mkdir -p $out
base=$GRAFT_REPO_ROOT/game-of-life-distributed_amd/golhip/libgolhip.so
GOLHIP_LIB=$cand timeout -k 10 600 python -u -m pytest tests/test_gpu_skew.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/pytest_cand.log 2>&1 || { tail -30 $out/pytest_cand.log; exit 1; }
tail -2 $out/pytest_cand.log
timeout -k 10 900 python -u scripts/ab_builds.py --libs $base,$cand --cases $cases --rounds 3 > $out/ab.txt 2> $out/ab.err \
  || { tail -20 $out/ab.err; exit 1; }
grep -v "^{" $out/ab.txt
if [ "$4" = stalls ]; then
  GOLHIP_LIB=$cand bash scripts/pmc_stalls.sh $out/cand gol_skew --workload 65536 || exit 1
  python3 scripts/pmc_stalls_summary.py $out/cand > $out/cand/stalls_summary.json
fi
echo ab-done
