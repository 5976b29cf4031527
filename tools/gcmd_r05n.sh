# round 5: stable-bucket placement ablations (timing only)
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
for C in headline c4; do
timeout -k 10 240 python -u tools/exp_rb.py $C scheme=3 sbabl=0 sbabl=1 sbabl=2 sbabl=4 sbabl=8 sbabl=9 sbabl=6 >> $O/rb.log 2>&1 || { echo "[rb $C] failed"; tail -5 $O/rb.log; exit 1; }
done
grep "median" $O/rb.log
