set -o pipefail
L=gpurun_out/split.log; : > $L
S=tools/gpu_step.sh
$S 400 $L python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deterministic.py tests/test_gpu_parity.py -k "split or bit_identical or raster_backward" -rf || exit 1
for c in headline c3 c4 c5; do CFG=$c $S 200 $L python -u tools/exp_chunk.py || exit 1; done
$S 500 $L python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_fullsize_fused.py tests/test_gpu_fullsize.py -rf
