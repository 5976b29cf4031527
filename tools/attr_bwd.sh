#!/bin/bash
# Attribution of the shipped strip backward's time: the same kernel with
# staging only (flag 64), without the record atomics (flag 1), and with the nine-value
# reduce-scatter replaced by a lane-local sum (a separate library built with
# -DGS_ABLATE_NO_REDUCE).  Interleaved timing by tools/exp_bwd.py on each CONFIGS entry.
# Build (here, CPU): tools/attr_bwd.sh build ; run (GPU box): tools/attr_bwd.sh run
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  mkdir -p ab/nored
  make -s -C gaussctrl_exp_amd/csrc BUILD=../../ab/nored OUT=../../ab/libNR.so \
    COMMON="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -DGS_ABLATE_NO_REDUCE" \
    ../../ab/libNR.so
  exit 0
fi
mkdir -p gpurun_out
for cfg in ${CONFIGS:-headline c4 c3}; do
  echo "== $cfg shipped library: flags 0 (shipped), 64 (staging only), 1 (no atomics)"
  CFG=$cfg FLAGS=0,64,1 timeout -k 10 240 python3 tools/exp_bwd.py
  echo "== $cfg no-reduce library: flags 0, 1 (no reduce, no atomics)"
  CFG=$cfg FLAGS=0,1 GSPLAT_MI355X_LIB=ab/libNR.so timeout -k 10 240 python3 tools/exp_bwd.py
done
