# round 5: vectorised tile table -- binning parity + timing, then the 2-rank gloo rehearsal of
# the bench's N > 1 path at c4 (both ranks on the one GPU)
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_speculative.py tests/test_gpu_sort.py tests/test_gpu_bin_concurrency.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1; rc=$?; echo "[tests] rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for C in headline c3 c4; do
timeout -k 10 240 python -u tools/exp_rb.py $C scheme=-1 scheme=-1 >> $O/rb.log 2>&1 || { echo "[rb $C] failed"; tail -5 $O/rb.log; exit 1; }
done
grep "median" $O/rb.log
ROUND=r05p GLOO2=1 GLOO2_CFG=c4 bash tools/gpu_iter.sh; rc=$?; echo "[gloo2] rc=$rc"; tail -3 gpurun_out/r05p/iter.log | cut -c1-1500
exit $rc
