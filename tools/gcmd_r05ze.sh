# round 5: list-split part size sweep (GSPLAT_MI355X_CHUNK, hooks library) at headline and c4
set -o pipefail
ROUND=r05ze CFGS="headline c4" AB="base:GSPLAT_MI355X_CHUNK=0 c512:GSPLAT_MI355X_CHUNK=512 c704:GSPLAT_MI355X_CHUNK=704 c1408:GSPLAT_MI355X_CHUNK=1408" REPS=2 STEPS=40 TRAIN_STEPS=3 bash tools/gpu_iter.sh; rc=$?
grep -v amdgpu.ids gpurun_out/r05ze/iter.log | grep -E "^(headline|c4) " | cut -c1-330
exit $rc
