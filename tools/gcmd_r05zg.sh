# round 5: the record backward pre-launched by the fused forward -- parity, then A/B
set -o pipefail
O=gpurun_out/r05zg; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused_l1.py tests/test_gpu_fused.py tests/test_gpu_speculative.py tests/test_gpu_fullsize_fused.py tests/test_gpu_optim.py tests/test_gpu_deterministic.py tests/test_gpu_multirank.py > $O/tests.log 2>&1; rc=$?; echo "[tests] rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
ROUND=r05zg CFGS="headline c3 c4" AB="base:GSPLAT_MI355X_PRELAUNCH_BWD=0 pre:GSPLAT_MI355X_PRELAUNCH_BWD=1" REPS=2 STEPS=40 TRAIN_STEPS=10 bash tools/gpu_iter.sh; rc=$?
grep -v amdgpu.ids gpurun_out/r05zg/iter.log | grep -E "^(headline|c3|c4) " | cut -c1-360
exit $rc
