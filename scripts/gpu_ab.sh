# A/B of candidate libgolhip builds against the tree's build on one box:
# each candidate's K1w parity tests, alternating whole-case timings
# (scripts/ab_builds.py), and optionally the candidates' SQ stall passes.
# usage: bash scripts/gpu_ab.sh <tag> <cand.so[,cand2.so...]> [cases] [stalls]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1; cases=${3:-65536x65536,16384x16384,65536x8192r}
out=gpurun_out/$tag
mkdir -p $out
base=$GRAFT_REPO_ROOT/game-of-life-distributed_amd/golhip/libgolhip.so
libs=$base
for c in ${2//,/ }; do
  cand=$(readlink -f $c); n=$(basename $cand .so)
  GOLHIP_LIB=$cand timeout -k 10 600 python -u -m pytest tests/test_gpu_skew.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/pytest_$n.log 2>&1 || { tail -30 $out/pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 $out/pytest_$n.log)"
  libs=$libs,$cand
done
timeout -k 10 900 python -u scripts/ab_builds.py --libs $libs --cases $cases --rounds 3 > $out/ab.txt 2> $out/ab.err \
  || { tail -20 $out/ab.err; exit 1; }
grep -v "^{" $out/ab.txt
if [ "$4" = stalls ]; then
  for c in ${2//,/ }; do
    cand=$(readlink -f $c); n=$(basename $cand .so)
    GOLHIP_LIB=$cand bash scripts/pmc_stalls.sh $out/$n gol_skew --workload 65536 || exit 1
    python3 scripts/pmc_stalls_summary.py $out/$n > $out/$n/stalls_summary.json
  done
fi
echo ab-done
