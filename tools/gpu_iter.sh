# One iteration on the GPU box (the one parameterised driver for development runs; the
# round-end measurement is tools/round_profile.sh).  In order, each step optional:
#   TESTS="tests/test_gpu_x.py ..."   GPU tests (TEST_TIMEOUT, default 600 s; BENCH_ANYWAY=1
#                                      benches even after a test failure)
#   CFGS="headline c3" AB="base:VAR=1 new:VAR=2,VAR2=3" REPS=2
#                                      bench lines per config x env setting x repetition
#                                      (STEPS, TRAIN_STEPS), one summary line each in the log
#   GLOO2=1 (GLOO2_CFG)               bench.py at --gpus 2 over gloo, both ranks on the one GPU
#   TIMELINE="headline c3"            rocprofv3 kernel trace -> per-step launch timeline
# Output under gpurun_out/$ROUND/ (default "iter"): iter.log, b_<cfg>_<name>_<rep>.json,
# timeline_<cfg>.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-iter}
mkdir -p $O
L=$O/iter.log; : > $L
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
      --no-cpu-baseline --no-lane-occupancy --train-steps ${TRAIN_STEPS:-10} > $O/b_${c}_${name}_$r.json 2>> $L || exit $?
    python3 - "$c" "$name" "$O/b_${c}_${name}_$r.json" >> $L <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
k = {n.replace("gsplat_", "")[:22]: round(v["ms_per_call"], 4) for n, v in d["kernels"].items()}
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], d.get("value_unchanged_caller"), d.get("train_iters_per_s"), k, flush=True)
PY
  done
done
done
if [ -n "$GLOO2" ]; then
  # the N > 1 bench path rehearsed on one GPU: two ranks, gloo carrying the collectives
  BENCH_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
    --config ${GLOO2_CFG:-headline} --steps 10 --warmup 3 --no-cpu-baseline --no-lane-occupancy \
    --train-steps 2 > $O/gloo2_${GLOO2_CFG:-headline}.json 2>> $L || exit $?
  tail -n 1 $O/gloo2_${GLOO2_CFG:-headline}.json >> $L
fi
if [ -n "$TIMELINE" ]; then
  for c in $TIMELINE; do
    timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tl_$c -o run -- python3 bench.py --config $c --steps 6 --warmup 3 --no-cpu-baseline --no-lane-occupancy --train-steps 0 > $O/tl_bench_$c.log 2>&1 || exit $?
    python3 tools/step_timeline.py gpurun_out/tl_$c/run_results.db ${TL_MARK:-fused_fwd_proj_kernel} 5 > $O/timeline_$c.txt || exit $?
    rm -rf gpurun_out/tl_$c
  done
fi
