# the N > 1 bench path with the direct step, rehearsed over gloo on the one GPU (headline, c4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ROUND=r05h6 GLOO2=1 GLOO2_CFG=headline bash tools/gpu_iter.sh || exit $?
ROUND=r05h6 GLOO2=1 GLOO2_CFG=c4 bash tools/gpu_iter.sh || exit $?
