# round 5: per-kernel times of the c5 binning (generated first pass on, then forced off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/pf_c5 -o run -- python3 tools/exp_rb.py c5 scheme=-1 > $O/pf_c5.log 2>&1 || exit $?
python3 tools/rocpd_stats.py gpurun_out/pf_c5/run_results.db $O/ks_c5_gen.csv || exit $?
rm -rf gpurun_out/pf_c5
