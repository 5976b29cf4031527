#!/bin/bash
# Same-box A/B of two builds of libgsplat_mi355x.so: bench.py (fused step, per-kernel ms)
# alternating LIBS (default ab/libA.so ab/libB.so) REPS times on CONFIG (default headline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-2}); do
  for L in ${LIBS:-ab/libA.so ab/libB.so}; do
    echo "== $L rep $r"
    GSPLAT_MI355X_LIB=$L timeout -k 10 300 python3 bench.py --config ${CONFIG:-headline} \
      --steps 50 --warmup 10 --no-cpu-baseline --train-steps ${TRAIN_STEPS:-5} > gpurun_out/ab.log 2>&1 || exit $?
    python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = {n.replace("gsplat_", ""): round(v["ms_per_call"], 4) for n, v in d["kernels"].items()}
print(d["value"], d["ms_per_step"], d.get("value_unchanged_caller"), d.get("train_iters_per_s"), k)
PY
  done
done
