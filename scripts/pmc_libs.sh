# rocprofv3 PMC passes (one counter group per pass) of prof_step.py per libgolhip build.
# usage: bash scripts/pmc_libs.sh <out_dir> <size> <depth> "<group1>" "<group2>" ... -- <lib1> <lib2> ...
out=$1; size=$2; depth=$3; shift 3
groups=(); while [ "$1" != "--" ]; do groups+=("$1"); shift; done; shift
mkdir -p $out
root=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename $lib .so)
  gi=0
  for g in "${groups[@]}"; do
    gi=$((gi+1))
    GOLHIP_LIB=$root/$lib timeout -s KILL 90 rocprofv3 --pmc $g --kernel-include-regex gol_ -d $out/pmc_${name}_$gi -o run --output-format csv -- python3 $root/scripts/prof_step.py --size $size --depth $depth --launches 5 --persistent 0 > $out/pmc_${name}_$gi.log 2>&1 || { tail $out/pmc_${name}_$gi.log; exit 1; }
  done
done
echo pmc-done
