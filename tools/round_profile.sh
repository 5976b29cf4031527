#!/bin/bash
# Round-end measurement on the GPU box: PMC traffic passes -> profiles/pmc_traffic.json (read by
# bench.py for roofline.traffic), kernel-trace stats, then the default bench line (with the CPU
# baseline).  Everything lands in gpurun_out/ (copied into profiles/ afterwards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_bench.sh || exit $?
python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_summary.csv profiles/pmc_traffic.json || exit $?
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_full.log
