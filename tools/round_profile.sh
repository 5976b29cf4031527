#!/bin/bash
# Round-end measurement on the GPU box.  For each config in CONFIGS (default: headline): PMC
# passes -> profiles/pmc_traffic.json[configs][cfg] (read by bench.py for that config's
# roofline.traffic / valu_busy), kernel-trace stats, and that config's bench line.  Everything
# lands in gpurun_out/ (copied into profiles/ afterwards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CONFIGS:-headline}; do
  CONFIG=$cfg bash tools/pmc_bench.sh || exit $?
  python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_summary_$cfg.csv \
    profiles/pmc_traffic.json $cfg || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats_$cfg -o run \
    -- python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-lane-occupancy --train-steps 5 \
    > gpurun_out/prof_bench_$cfg.log 2>&1 || exit $?
  python3 tools/rocpd_stats.py gpurun_out/prof_stats_$cfg/run_results.db \
    gpurun_out/kernel_stats_$cfg.csv || exit $?
  # only the summaries travel back (gpurun returns at most 64 MiB)
  rm -rf gpurun_out/pmc gpurun_out/prof_stats_$cfg
  timeout -k 10 600 python3 bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || exit $?
  tail -n 1 gpurun_out/bench_$cfg.log
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
