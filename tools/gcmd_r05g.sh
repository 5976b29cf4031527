# round 5: pipelined placement ranking
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 300 python3 tools/exp_rb.py headline 512,2,0 512,4,0 512,2,10 512,2,40 512,2,0 > $O/h3.log 2>&1; echo "[h] rc=$?"
timeout -k 10 300 python3 tools/exp_rb.py c3 512,2,0 512,4,0 512,2,40 > $O/c3c.log 2>&1; echo "[c3] rc=$?"
timeout -k 10 300 python3 tools/exp_rb.py c5 512,4,0 > $O/c5c.log 2>&1; echo "[c5] rc=$?"
grep -h "bin_spec\|Error\|assert" $O/h3.log $O/c3c.log $O/c5c.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "binning or speculative" > $O/tests.log 2>&1; echo "[bin tests] rc=$?"; tail -2 $O/tests.log
