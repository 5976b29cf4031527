set -o pipefail
L=gpurun_out/host.log; : > $L
S=tools/gpu_step.sh
$S 300 $L python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused.py -rf || exit 1
CFG=c3 $S 200 gpurun_out/cpuprof_c3_r3.log python -u tools/cpu_profile.py || exit 1
for c in c3 headline; do $S 300 $L python -u bench.py --config $c --no-cpu-baseline --no-lane-occupancy || exit 1; done
