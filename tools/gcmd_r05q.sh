# round 5: per-step launch timeline of the headline and c3 steps (idle gaps between kernels)
set -o pipefail
ROUND=r05q TIMELINE="headline c3" bash tools/gpu_iter.sh; rc=$?; echo "[timeline] rc=$rc"
exit $rc
