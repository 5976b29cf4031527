# dual-queue strip backward: parity, then same-box A/B of the raster variants (1,0,0 = dual
# queue at strip frames; 1,3,0 = one queue per strip)
set -o pipefail
L=gpurun_out/dq.log; : > $L
S=tools/gpu_step.sh
$S 900 $L python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_fullsize_fused.py tests/test_gpu_deterministic.py \
  -k "dual_queue or filled or fullsize or fused_render or deterministic or split" || exit 1
grep "\[parity\] dual" $L | head -5
for c in ${CFGS:-headline c4}; do
  for v in 1,0,0 1,3,0 1,0,0 1,3,0; do
    echo "== $c variant $v" >> $L
    GSPLAT_MI355X_RASTER_VARIANT=$v timeout -k 10 300 python3 bench.py --config $c --steps 50 \
      --warmup 10 --no-cpu-baseline --no-lane-occupancy --train-steps 5 > gpurun_out/dq1.log 2>&1 || exit 1
    python3 - >> $L <<'PY'
import json
d = json.loads(open("gpurun_out/dq1.log").read().strip().splitlines()[-1])
k = {n.replace("gsplat_", ""): round(v["ms_per_call"], 4) for n, v in d["kernels"].items()}
print(d["value"], d["ms_per_step"], d.get("value_unchanged_caller"), d.get("train_iters_per_s"), k)
PY
  done
done
