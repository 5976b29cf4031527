# direct step with the L1 + SSIM train step: fused GPU tests, then train-rate A/B (autograd vs direct)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05h8
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_fused_l1.py tests/test_gpu_fused.py tests/test_gpu_multirank.py tests/test_gpu_fullsize_fused.py \
  > gpurun_out/r05h8/tests.log 2>&1 || exit $?
ROUND=r05h8 CFGS="c2 c3 headline" AB="auto:GSPLAT_MI355X_DIRECT_STEP=0 direct:GSPLAT_MI355X_DIRECT_STEP=1" REPS=2 TRAIN_STEPS=100 bash tools/gpu_iter.sh || exit $?
