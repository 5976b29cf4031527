# kernel-trace timelines of a few bench steps per config -> gpurun_out/timeline_<cfg>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for cfg in ${CFGS:-c3 headline}; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tl_$cfg -o run -- python3 bench.py --config $cfg --steps 6 --warmup 3 --no-cpu-baseline --no-lane-occupancy --train-steps 0 > gpurun_out/tl_bench_$cfg.log 2>&1 || exit $?
  python3 tools/step_timeline.py gpurun_out/tl_$cfg/run_results.db fused_fwd_kernel 5 > gpurun_out/timeline_$cfg.txt || exit $?
  rm -rf gpurun_out/tl_$cfg
done
