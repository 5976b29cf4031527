set -o pipefail
L=gpurun_out/bin.log; : > $L
S=tools/gpu_step.sh
$S 500 $L python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fused.py -k "binning or fused or headline" -rf || exit 1
$S 200 $L python -u tools/exp_bin_opts.py || exit 1
$S 200 $L python -u bench.py --config c2 --no-cpu-baseline --no-lane-occupancy
