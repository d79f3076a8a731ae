# waves per SIMD vs depth: paired-band K1 at depths 8/12/16/20 (4/3/2/2 waves per SIMD by VGPRs) and K1w
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3d}
mkdir -p $out
timeout -k 10 500 python -u scripts/sweep_opts.py --no-timing --reps 2 --turns 960 --cases "65536x65536,65536x8192" --sets "skew=1;skew=1,tb_depth=12;skew=0,split=0;skew=0,split=0,tb_depth=16;skew=0,split=0,tb_depth=12;skew=0,split=0,tb_depth=8" > $out/depth_waves.txt 2> $out/depth_waves.err || { tail $out/depth_waves.err; exit 1; }
grep -A100 "^# best" $out/depth_waves.txt
