# the host path of a bench step at c3 and c4 (tools/host_timeline.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05h2
for c in c3 c4 headline; do
  CFG=$c timeout -k 10 300 python3 tools/host_timeline.py > gpurun_out/r05h2/host_$c.txt 2>&1 || exit $?
done
