# round 5: the colour part after the depth sort (GSPLAT_MI355X_COLOURS_AFTER_SORT) -- parity
# with it on, then A/B at headline / c4 / c5
set -o pipefail
O=gpurun_out/r05zd; mkdir -p $O
GSPLAT_MI355X_COLOURS_AFTER_SORT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_preprocess_split.py tests/test_gpu_speculative.py tests/test_gpu_fullsize_fused.py tests/test_gpu_fused_l1.py > $O/tests.log 2>&1; rc=$?; echo "[tests] rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
ROUND=r05zd CFGS="headline c4 c5" AB="base:GSPLAT_MI355X_COLOURS_AFTER_SORT=0 late:GSPLAT_MI355X_COLOURS_AFTER_SORT=1" REPS=2 STEPS=40 TRAIN_STEPS=5 bash tools/gpu_iter.sh; rc=$?
grep -v amdgpu.ids gpurun_out/r05zd/iter.log | grep -E "^(headline|c4|c5) " | cut -c1-400
exit $rc
