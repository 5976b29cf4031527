# round 5: record kinds of the fused exchange over several steps at c4 (gloo, 2 ranks, 1 GPU)
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/exp_xchg_kinds.py c4 6 > $O/kinds.log 2>&1; rc=$?
grep -E "rank|Error|error" $O/kinds.log | tail -20
exit $rc
