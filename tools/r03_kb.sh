# keep-bits backward: parity subset, then same-box A/B bench lines (KB on / off / on)
set -o pipefail
L=gpurun_out/kb.log; : > $L
S=tools/gpu_step.sh
$S 600 $L python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_deterministic.py tests/test_gpu_fullsize_fused.py || exit 1
for c in ${CFGS:-headline c3 c4}; do
  for v in 1,0,0 1,0,1073741824 1,0,0; do
    echo "== $c variant $v" >> $L
    GSPLAT_MI355X_RASTER_VARIANT=$v $S 300 $L python -u bench.py --config $c --steps 30 \
      --no-cpu-baseline --no-lane-occupancy --train-steps 5 || exit 1
  done
done
