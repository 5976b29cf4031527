# round 5: host-side cost of the c3 step (python wall vs GPU, torch.profiler CPU, cProfile)
set -o pipefail
O=gpurun_out/r05zc; mkdir -p $O
CFG=c3 timeout -k 10 300 python3 tools/cpu_profile.py > $O/cpu_c3.log 2>&1; rc=$?
head -20 $O/cpu_c3.log
exit $rc
