# round 5: test-hooks library split (parity tests through it) + region binning at c4
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deterministic.py tests/test_gpu_caller_path.py tests/test_gpu_pair_count.py > $O/tests.log 2>&1; echo "[tests] rc=$?"; tail -3 $O/tests.log
timeout -k 10 400 python3 tools/exp_rb.py c4 512,4,0 1024,4,0 2048,4,0 1024,6,0 2048,8,0 512,2,0 512,4,10 512,4,20 512,4,40 > $O/c4.log 2>&1; echo "[c4] rc=$?"
grep -h "bin_spec\|Error" $O/c4.log
