# c3 host-side cost: per-step kernel timeline (gaps) and the host profile of the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05h1
ROUND=r05h1 TIMELINE=c3 TL_MARK=fused_fwd_kernel bash tools/gpu_iter.sh || exit $?
CFG=c3 timeout -k 10 300 python3 tools/cpu_profile.py > gpurun_out/r05h1/cpu_c3.txt 2>&1 || exit $?
