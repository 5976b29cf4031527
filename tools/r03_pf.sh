set -o pipefail
L=gpurun_out/pf.log; : > $L
S=tools/gpu_step.sh
$S 400 $L python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_deterministic.py tests/test_gpu_fused.py -rf || exit 1
CHUNKS=0 FLAGS=0,0x10000000,0x20000000 CFGS="c3 c2" bash tools/r03_sweep.sh || exit 1
cat gpurun_out/sweep.log >> $L
$S 300 $L python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_fullsize_fused.py -k c3 -rf
