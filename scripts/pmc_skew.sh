# rocprofv3 PMC passes of the K1w kernel on given cases (one counter group a pass)
# usage: bash scripts/pmc_skew.sh <out dir (absolute)> <case> [case ...]   (case as in sweep_opts.py)
set -o pipefail
out=$1; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  args="$GRAFT_REPO_ROOT/scripts/sweep_opts.py --no-timing --reps 1 --turns 200 --cases $c --sets skew=1"
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex gol_skew -d $out/pmc_${c}_$i -o run --output-format csv -- python3 $args > $out/pmc_${c}_$i.log 2>&1 || { tail $out/pmc_${c}_$i.log; exit 1; }
  done
done
python3 $GRAFT_REPO_ROOT/scripts/pmc_skew_summary.py $out
