# round 5: the generated first tile-sort pass, emission with a one-workgroup block scan from 1M Gaussians
set -o pipefail
O=gpurun_out/r05zf; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_speculative.py tests/test_gpu_bin_concurrency.py tests/test_c_abi.py > $O/tests.log 2>&1; rc=$?; echo "[tests] rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for C in c4 c5; do
timeout -k 10 240 python -u tools/exp_rb.py $C scheme=-1 scheme=-1 >> $O/rb.log 2>&1 || { echo "[rb $C] failed"; tail -5 $O/rb.log; exit 1; }
done
grep "median" $O/rb.log


