# round 5: per-kernel times of the stable-bucket binning (exp_rb under the kernel trace)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
for C in headline c4; do
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/pf_$C -o run -- python3 tools/exp_rb.py $C scheme=-1 > $O/pf_$C.log 2>&1 || exit $?
python3 tools/rocpd_stats.py gpurun_out/pf_$C/run_results.db $O/ks_$C.csv || exit $?
rm -rf gpurun_out/pf_$C
done
