set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for cfg in c3 c2; do
  CFGS=$cfg timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/bk_$cfg -o run -- python3 tools/exp_bin_opts.py > gpurun_out/bk_$cfg.log 2>&1 || exit $?
  python3 tools/rocpd_stats.py gpurun_out/bk_$cfg/run_results.db gpurun_out/bk_stats_$cfg.csv || exit $?
  rm -rf gpurun_out/bk_$cfg
done
