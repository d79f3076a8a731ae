set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1
for d in 8 16 32; do
  timeout -k 10 120 python -u bench.py --steps 5 --tb-depth $d --no-cpu-baseline > gpurun_out/r1/bench16k_d$d.json 2> gpurun_out/r1/bench16k_d$d.err || exit 1
done
for d in 16 32; do
  timeout -k 10 120 python -u bench.py --workload 65536 --steps 3 --tb-depth $d --no-cpu-baseline > gpurun_out/r1/bench64k_d$d.json 2> gpurun_out/r1/bench64k_d$d.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r1/prof16k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r1/prof16k.log 2>&1 || exit 1
