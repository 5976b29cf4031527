# round 5: the sparse plan's scan without the in-place race -- exchange tests, then the record
# kinds over several steps at c4 (gloo, 2 ranks, 1 GPU)
set -o pipefail
O=gpurun_out/r05za; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_exchange.py tests/test_gpu_multirank.py > $O/tests.log 2>&1; rc=$?; echo "[tests] rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/exp_xchg_kinds.py c4 8 > $O/kinds.log 2>&1; rc=$?
grep -E "^rank|Error" $O/kinds.log | tail -16
exit $rc
