# Per-wave phase stamps of one K1w launch on the round-6 default plans (pair
# rule, 18 turns) and on the 9-LUT stages (skew_pairs 1: 16384^2 at 16).
set -o pipefail
mkdir -p gpurun_out/r7e
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python scripts/trace_skew.py "$@" > gpurun_out/r7e/trace_$tag.json 2> gpurun_out/r7e/trace_$tag.err || { tail gpurun_out/r7e/trace_$tag.err; exit 1; }
  cat gpurun_out/r7e/trace_$tag.json
}
run 16384 --case 16384x16384 --depth 18
run 16384_lut9 --case 16384x16384 --depth 16 --opt skew_pairs=1
run 8192r --case 65536x8192r --depth 18
run 8192r_lut9 --case 65536x8192r --depth 20 --opt skew_pairs=0
run 65536 --case 65536x65536 --depth 18
