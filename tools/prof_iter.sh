# Kernel-trace stats of a short bench run per config (development; the round-end profile is
# tools/round_profile.sh).  CFGS="headline c5" ENVS="VAR=1 VAR2=2" ROUND=name
# -> gpurun_out/$ROUND/ks_<cfg>.csv (rocpd top-kernels summary) and pf_<cfg>.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-prof}
mkdir -p $O
for c in ${CFGS:-headline}; do
  env ${ENVS:-X=0} timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/pf_$c -o run -- \
    python3 bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
    --no-lane-occupancy --train-steps 0 > $O/pf_$c.log 2>&1 || exit $?
  python3 tools/rocpd_stats.py gpurun_out/pf_$c/run_results.db $O/ks_$c.csv || exit $?
  rm -rf gpurun_out/pf_$c
done
