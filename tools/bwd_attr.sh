#!/bin/bash
# Where the record backward's time goes: an attribution build of the library
# (-DGS_BWD_ATTR: the strip backward sums s_memtime cycles of its blend rounds and their
# reduce9 + atomic tails into the wave log) run on the bench step by tools/bwd_attr.py.
# Build (here, CPU): tools/bwd_attr.sh build ; run (GPU box): CFGS="headline c4" tools/bwd_attr.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  mkdir -p ab/attr
  make -s -C gaussctrl_exp_amd/csrc BUILD=../../ab/attr OUT=../../ab/libattr.so \
    EXTRA="-DGS_BWD_ATTR -DGSPLAT_TEST_HOOKS" ../../ab/libattr.so
  exit 0
fi
mkdir -p gpurun_out
for cfg in ${CFGS:-headline}; do
  CFG=$cfg GSPLAT_MI355X_LIB=ab/libattr.so timeout -k 10 240 python3 tools/bwd_attr.py
done
