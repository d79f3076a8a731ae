# SQ counters of K5 (gol_flip_turn_kernel) with copy blocks (flip_overlap 1) and with no entries (flip_debug 2).
set -o pipefail
mkdir -p gpurun_out/r7j
K5_MODES=overlap bash scripts/pmc_stalls.sh gpurun_out/r7j/overlap gol_flip_turn -- scripts/k5_overlap_probe.py || exit 1
K5_MODES=no_entries bash scripts/pmc_stalls.sh gpurun_out/r7j/noent gol_flip_turn -- scripts/k5_overlap_probe.py || exit 1
python3 scripts/pmc_stalls_summary.py gpurun_out/r7j/overlap > gpurun_out/r7j/overlap_summary.json
python3 scripts/pmc_stalls_summary.py gpurun_out/r7j/noent > gpurun_out/r7j/noent_summary.json
cat gpurun_out/r7j/overlap_summary.json gpurun_out/r7j/noent_summary.json
