#!/bin/bash
# Attribution of the shipped strip backward's reduce + atomic tail: the record
# backward timed in the bench step (tools/gpu_iter.sh AB over GSPLAT_MI355X_LIB) with three
# ablation builds of the library beside the shipped one:
#   ablib/libNR.so  -DGS_ABLATE_NO_REDUCE  the nine-value reduce-scatter replaced by a lane-local sum
#   ablib/libNA.so  -DGS_ABLATE_NO_ATOMIC  the record atomics replaced by an empty consumer
#   ablib/libNN.so  both
# (results are wrong numerically in the ablations; only their time is read).  The libraries
# go to ablib/ (git-ignored, not gpurun-ignored: they travel to the box).
# Build (here, CPU): tools/attr_bwd.sh build ; run (GPU box): tools/attr_bwd.sh run
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  for v in "NR:-DGS_ABLATE_NO_REDUCE" "NA:-DGS_ABLATE_NO_ATOMIC" "NN:-DGS_ABLATE_NO_REDUCE -DGS_ABLATE_NO_ATOMIC"; do
    name=${v%%:*}; defs=${v#*:}
    mkdir -p ablib/$name
    make -s -C gaussctrl_exp_amd/csrc BUILD=../../ablib/$name OUT=../../ablib/lib$name.so \
      EXTRA="$defs" ../../ablib/lib$name.so
  done
  exit 0
fi
ROUND=${ROUND:-attr} CFGS="${CFGS:-headline c4}" REPS=${REPS:-2} \
  AB="ship:X=0 NR:GSPLAT_MI355X_LIB=ablib/libNR.so NA:GSPLAT_MI355X_LIB=ablib/libNA.so NN:GSPLAT_MI355X_LIB=ablib/libNN.so" \
  bash tools/gpu_iter.sh
