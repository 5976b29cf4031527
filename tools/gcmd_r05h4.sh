# the direct step + raw stream handles: whole GPU suite, smoke, then c3 / c4 / headline A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gcmd_r05suite.sh || exit $?
ROUND=r05h4 CFGS="c3 c4 headline" AB="auto:GSPLAT_MI355X_DIRECT_STEP=0 direct:GSPLAT_MI355X_DIRECT_STEP=1" REPS=2 bash tools/gpu_iter.sh || exit $?
CFG=c3 timeout -k 10 300 python3 tools/host_timeline.py > gpurun_out/r05h4/host_c3.txt 2>&1 || exit $?
