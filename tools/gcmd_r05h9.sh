# final tree: whole GPU suite + smoke, then the c2 / c5 round profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gcmd_r05suite.sh || exit $?
bash tools/gcmd_r05y.sh || exit $?
