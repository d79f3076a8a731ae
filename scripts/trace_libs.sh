# rocprofv3 kernel-trace summaries of one bench line per libgolhip build.
# usage: bash scripts/trace_libs.sh <out_dir> "<bench args>" <lib1> <lib2> ...
out=$1; args=$2; shift 2
mkdir -p $out
root=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename $lib .so)
  GOLHIP_LIB=$root/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace_$name -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline $args > $out/trace_$name.log 2>&1 || { tail $out/trace_$name.log; exit 1; }
  echo "== $name"; head -4 $(find $out/trace_$name -name "*kernel_stats.csv" | head -1) | cut -c1-160
done
