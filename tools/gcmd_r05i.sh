# round 5: small-frame forward (S lanes per pixel): parity with it selected, then A/B
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
for L in 4 2; do
GSPLAT_MI355X_FWD_LANES=$L timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_fused_l1.py tests/test_gpu_caller_path.py tests/test_gpu_eval_render.py > $O/tests_$L.log 2>&1; rc=$?; echo "[tests lanes=$L] rc=$rc"; tail -3 $O/tests_$L.log
[ $rc -gt 1 ] && exit $rc
done
ROUND=r05i CFGS="c3 c2" AB="l0:GSPLAT_MI355X_FWD_LANES=0 l4:GSPLAT_MI355X_FWD_LANES=4 l2:GSPLAT_MI355X_FWD_LANES=2" REPS=2 STEPS=40 TRAIN_STEPS=5 bash tools/gpu_iter.sh; echo "[iter] rc=$?"
grep -v amdgpu.ids $O/iter.log | tail -14
