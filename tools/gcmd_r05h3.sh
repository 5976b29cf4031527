# the direct fused step: parity tests, host timelines, bench A/B (autograd vs direct)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05h3
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_fused_l1.py tests/test_gpu_fused.py > gpurun_out/r05h3/tests.log 2>&1 || exit $?
for c in c3 c4 headline; do
  CFG=$c timeout -k 10 300 python3 tools/host_timeline.py > gpurun_out/r05h3/host_$c.txt 2>&1 || exit $?
done
ROUND=r05h3 CFGS="c3 c4 headline" AB="auto:GSPLAT_MI355X_DIRECT_STEP=0 direct:GSPLAT_MI355X_DIRECT_STEP=1" REPS=2 bash tools/gpu_iter.sh || exit $?
