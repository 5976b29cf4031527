# c3 per-step kernel timeline with the direct step (where the device still idles)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ROUND=r05h10 TIMELINE=c3 TL_MARK=fused_fwd_kernel bash tools/gpu_iter.sh || exit $?
