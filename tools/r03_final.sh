# fused-path tests, then bench lines at headline and c3 (host-time check of the campos cache)
set -o pipefail
L=gpurun_out/final.log; : > $L
S=tools/gpu_step.sh
$S 600 $L python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_multirank.py tests/test_gpu_exchange.py tests/test_gpu_optim.py || exit 1
for c in headline c3 c3; do
  $S 300 $L python -u bench.py --config $c --no-cpu-baseline --no-lane-occupancy --train-steps 5 || exit 1
done
