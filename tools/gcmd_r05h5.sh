# headline kernel durations, autograd vs direct step (rocprofv3 stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05h5; mkdir -p $O
for m in 0 1; do
  GSPLAT_MI355X_DIRECT_STEP=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p$m -o run -- python3 bench.py --config headline --steps 40 --warmup 10 --no-cpu-baseline --no-lane-occupancy --train-steps 0 > $O/b$m.json 2> $O/b$m.err || exit $?
  python3 tools/rocpd_stats.py $O/p$m/run_results.db $O/stats_$m.csv || exit $?
  rm -rf $O/p$m
done
