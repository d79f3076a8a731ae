# quads (4 words per lane, depth 9: taller bands, shorter fill) on the strip shares vs pairs (depth 20)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3p}
mkdir -p $out
timeout -k 10 500 python -u scripts/sweep_opts.py --no-timing --reps 2 --cases "65536x8192r,65536x16384r,65536x8192,65536x65536" --sets "skew=1;wpl=4;wpl=4,tb_depth=8" > $out/quads.txt 2> $out/quads.err || { tail $out/quads.err; exit 1; }
grep -A100 "^# best" $out/quads.txt
