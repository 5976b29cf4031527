set -o pipefail
L=gpurun_out/bench.log; : > $L
S=tools/gpu_step.sh
$S 300 $L python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_parity.py -k "binning or fused" -rf || exit 1
for c in ${CFGS:-c2 c3 headline}; do
  $S 300 $L python -u bench.py --config $c --no-cpu-baseline --no-lane-occupancy || exit 1
done
