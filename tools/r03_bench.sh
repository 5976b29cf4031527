set -o pipefail
L=gpurun_out/bench.log; : > $L
S=tools/gpu_step.sh
for c in ${CFGS:-headline c3}; do
  $S 300 $L python -u bench.py --config $c --no-cpu-baseline --no-lane-occupancy || exit 1
done
