# round 5: exchange / multirank tests, queue backward parity + A/B
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_exchange.py tests/test_gpu_multirank.py > $O/xtests.log 2>&1; echo "[exchange tests] rc=$?"; tail -4 $O/xtests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fullsize_fused.py tests/test_gpu_fused_l1.py tests/test_gpu_fused.py > $O/ftests.log 2>&1; rc=$?; echo "[fused tests] rc=$rc"; tail -4 $O/ftests.log
[ $rc -gt 1 ] && exit $rc
ROUND=r05e CFGS="headline c4" AB="q:GSPLAT_MI355X_BWD_QUEUE=1 noq:GSPLAT_MI355X_BWD_QUEUE=0" REPS=2 STEPS=40 TRAIN_STEPS=5 bash tools/gpu_iter.sh; echo "[iter] rc=$?"
grep -v amdgpu.ids $O/iter.log | tail -12
timeout -k 10 200 python3 tools/exp_exchange.py > $O/exch.log 2>&1; echo "[exch timing] rc=$?"; grep -v amdgpu.ids $O/exch.log | tail -14
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_rb -o run -- python3 tools/exp_rb.py headline 512,2,0 > $O/prof_rb.log 2>&1; echo "[rocprof rb] rc=$?"
find $O/prof_rb -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/rb_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05e/rb_kernel_stats.csv")))
for r in rows[:25]:
    print(r["Name"][:90], r["Calls"], r["AverageNs"] if "AverageNs" in r else r.get("AverageUs"))
PY
rm -rf $O/prof_rb
