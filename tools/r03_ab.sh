# parity suites on the current build, then same-box A/B of LIBS (default ab/libA.so ab/libB.so)
set -o pipefail
L=gpurun_out/ab_all.log; : > $L
S=tools/gpu_step.sh
$S 900 $L python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_fused.py tests/test_gpu_deterministic.py tests/test_gpu_pair_count.py} || exit 1
for c in ${CFGS:-headline c3 c4}; do
  echo "=== $c" >> $L
  CONFIG=$c REPS=${REPS:-2} timeout -k 10 900 bash tools/ab_libs.sh >> $L 2>&1 || exit 1
done
