# round 5: the forward's longest-first tile order -- blend parity, then A/B on/off (hooks lib)
set -o pipefail
ROUND=r05o \
 CFGS="headline c4 c3" AB="on:GSPLAT_MI355X_RASTER_VARIANT=1/0/0 off:GSPLAT_MI355X_RASTER_VARIANT=1/0/524288" REPS=2 STEPS=40 TRAIN_STEPS=5 bash tools/gpu_iter.sh; rc=$?; echo "[iter] rc=$rc"
grep -v amdgpu.ids gpurun_out/r05o/iter.log | tail -16
exit $rc
