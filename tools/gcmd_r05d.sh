# round 5: region-binning sweep + the sparse / multi-view exchange tests
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "binning or speculative" > $O/tests.log 2>&1; echo "[bin tests] rc=$?"; tail -3 $O/tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_exchange.py tests/test_gpu_multirank.py > $O/xtests.log 2>&1; echo "[exchange tests] rc=$?"; tail -15 $O/xtests.log
timeout -k 10 300 python3 tools/exp_rb.py headline 512,4,0 512,4,9 256,4,0 1024,4,0 512,2,0 512,5,0 1024,5,0 > $O/h.log 2>&1 && timeout -k 10 300 python3 tools/exp_rb.py c5 512,4,0 512,4,9 1024,4,0 512,5,0 > $O/c5.log 2>&1 && timeout -k 10 300 python3 tools/exp_rb.py c3 512,4,0 256,4,0 512,2,0 > $O/c3.log 2>&1; cat $O/h.log $O/c5.log $O/c3.log | grep -v amdgpu.ids
for c in headline c4; do
  CFG=$c TIME_ONLY=1 timeout -k 10 240 python3 tools/bwd_attr.py 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a $O/attr.log
  CFG=$c GSPLAT_MI355X_LIB=ab/libattr.so timeout -k 10 240 python3 tools/bwd_attr.py 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a $O/attr.log
done
