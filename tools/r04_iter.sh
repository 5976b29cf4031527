# Round-4 iteration on the GPU box: the named GPU test files, then same-process-setting A/B
# bench lines (env switches) on the named configs.  Output under gpurun_out/r04/.
#   TESTS="tests/test_gpu_speculative.py ..." CFGS="headline c3" AB="base:VAR=1 new:VAR=2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
L=gpurun_out/r04/iter.log; : > $L
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    -m gpu $TESTS >> $L 2>&1
  rc=$?; echo "[tests] rc=$rc" >> $L
  [ $rc -gt 1 ] && exit $rc
  [ $rc -ne 0 ] && [ -z "$BENCH_ANYWAY" ] && exit $rc
fi
for r in $(seq ${REPS:-1}); do
for c in ${CFGS:-}; do
  for ab in ${AB:-cur:X=0}; do
    name=${ab%%:*}; envs=${ab#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python3 bench.py --config $c --steps ${STEPS:-50} --warmup 10 \
      --no-cpu-baseline --no-lane-occupancy --train-steps ${TRAIN_STEPS:-10} > gpurun_out/r04/b_${c}_${name}_$r.json 2>> $L || exit $?
    python3 - "$c" "$name" "gpurun_out/r04/b_${c}_${name}_$r.json" >> $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
k = {n.replace("gsplat_", "")[:22]: round(v["ms_per_call"], 4) for n, v in d["kernels"].items()}
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], d.get("value_unchanged_caller"), d.get("train_iters_per_s"), k, flush=True)
PY
  done
done
done
if [ -n "$TIMELINE" ]; then
  for c in $TIMELINE; do
    timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tl_$c -o run -- python3 bench.py --config $c --steps 6 --warmup 3 --no-cpu-baseline --no-lane-occupancy --train-steps 0 > gpurun_out/r04/tl_bench_$c.log 2>&1 || exit $?
    python3 tools/step_timeline.py gpurun_out/tl_$c/run_results.db fused_fwd_kernel 5 > gpurun_out/r04/timeline_$c.txt || exit $?
    rm -rf gpurun_out/tl_$c
  done
fi
