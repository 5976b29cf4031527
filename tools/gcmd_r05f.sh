# round 5: table kernel pipelining + parallel sparse plan; binning kernel profile
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_exchange.py tests/test_gpu_multirank.py > $O/xtests.log 2>&1; echo "[exchange tests] rc=$?"; tail -3 $O/xtests.log
timeout -k 10 200 python3 tools/exp_exchange.py > $O/exch.log 2>&1; echo "[exch timing] rc=$?"; grep -v amdgpu.ids $O/exch.log | tail -14
for c in headline c3; do
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof_rb_$c -o run -- python3 tools/exp_rb.py $c 512,2,0 > $O/prof_rb_$c.log 2>&1; echo "[rocprof rb $c] rc=$?"
db=$(find $O/prof_rb_$c -name "*.db" | head -1)
python3 tools/rocpd_stats.py $db $O/rb_stats_$c.csv && head -30 $O/rb_stats_$c.csv
rm -rf $O/prof_rb_$c
done
