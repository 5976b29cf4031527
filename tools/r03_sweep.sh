set -o pipefail
L=gpurun_out/sweep.log; : > $L
S=tools/gpu_step.sh
for c in ${CFGS:-headline c3 c4 c5}; do CFG=$c CHUNKS=${CHUNKS:--1,0} FLAGS=${FLAGS:-0,0x10000000,0x20000000} $S 200 $L python -u tools/exp_chunk.py || exit 1; done
