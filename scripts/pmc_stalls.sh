# Where the step kernel's issue cycles go (65536^2 bench step): SQ wait/active
# breakdown and instruction mix, one counter group per rocprofv3 pass.
# usage: bash scripts/pmc_stalls.sh <out dir under gpurun_out> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/$1
shift
args="$GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --warmup-seconds 0 --no-cpu-baseline $@"
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --kernel-include-regex gol_tb_pair -d $out/pass_a -o run --output-format csv -- python3 $args > $out/pass_a.log 2>&1 || { tail $out/pass_a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --kernel-include-regex gol_tb_pair -d $out/pass_b -o run --output-format csv -- python3 $args > $out/pass_b.log 2>&1 || { tail $out/pass_b.log; exit 1; }
echo stalls-done
