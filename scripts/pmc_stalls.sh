# Where a step kernel's issue cycles go: SQ wait / active breakdown and the
# instruction mix of the bench command, one counter group per rocprofv3 pass.
# usage: bash scripts/pmc_stalls.sh <out dir under gpurun_out> <kernel regex> [bench args...]
#   e.g. bash scripts/pmc_stalls.sh gpurun_out/r4a gol_skew --workload 65536
#   or   bash scripts/pmc_stalls.sh <out> <regex> -- <script.py> [args...]   (any repo script instead of bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/$1
kre=$2
shift 2
if [ "$1" = "--" ]; then
  shift
  args="$GRAFT_REPO_ROOT/$*"
else
  args="$GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --warmup-seconds 0 --no-cpu-baseline --no-configs3 $@"
fi
tag=$(echo "$@" | tr -c 'a-zA-Z0-9\n' '_')
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
[ -s $out/counters_list.txt ] || timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $out/counters_list.txt && printf '%s ' "$c"; done; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
           "$(have SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SENDMSG)" \
           "$(have SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE)" \
           "$(have SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_LDS_MEM_VIOLATIONS)"; do
  i=$((i+1))
  [ -n "$(echo $grp)" ] || continue
  timeout -s KILL 120 rocprofv3 --pmc $grp GRBM_GUI_ACTIVE --kernel-include-regex $kre -d $out/stall_${tag}_$i -o run --output-format csv -- python3 $args > $out/stall_${tag}_$i.log 2>&1 || { tail $out/stall_${tag}_$i.log; exit 1; }
done
echo stalls-done
