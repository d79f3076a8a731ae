# K1r (resident LDS bands): parity tests, the phase probe (scripts/lds_probe.py)
# and SQ counter passes of one 8192^2 run.  usage: bash scripts/gpu_lds_probe.sh <tag> [sets]
set -o pipefail
tag=${1:-lds}
sets=${2:-"lds_depth=8;lds_depth=12"}
mkdir -p gpurun_out/$tag
echo "== lds tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_lds.log 2>&1; rc=$?
tail -3 gpurun_out/$tag/pytest_lds.log
[ $rc -eq 0 ] || exit $rc
echo "== probe $(date +%T)"
timeout -k 10 600 python -u scripts/lds_probe.py --reps 1 --cases 8192x8192,5120x5120 --sets "$sets" > gpurun_out/$tag/probe.log 2>&1; rc=$?
cut -c1-300 gpurun_out/$tag/probe.log
[ $rc -eq 0 ] || exit $rc
echo "== pmc $(date +%T)"
timeout -k 10 600 bash scripts/pmc_stalls.sh gpurun_out/$tag gol_lds_band -- scripts/lds_probe.py --reps 1 --turns 1000 --cases 8192x8192 --sets lds_depth=8 > gpurun_out/$tag/pmc.log 2>&1; rc=$?
tail -2 gpurun_out/$tag/pmc.log
python3 scripts/pmc_stalls_summary.py gpurun_out/$tag gol_lds_band > gpurun_out/$tag/stalls_summary.json && python3 -c "
import json;d=json.load(open('gpurun_out/$tag/stalls_summary.json'))
for k,v in d.items(): print(k, v.get('wave_cycle_split'), v.get('instruction_mix'), {c:round(x) for c,x in v['counters'].items() if 'LDS' in c or c in ('SQ_INSTS_VALU','SQ_WAVES')})"
exit $rc
