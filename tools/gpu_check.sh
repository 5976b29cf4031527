#!/bin/bash
# GPU-box driver: parity tests -> smoke -> bench, each under its own time limit.
# Stops at the first step that crashes, aborts or times out (exit code other than 0/1),
# so nothing further touches a GPU that may be in a bad state.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
STEPS=${STEPS:-tests,smoke,bench}
rc=0
if [[ $STEPS == *tests* ]]; then
  step gpu_tests 900 python -m pytest tests -q -m gpu -p no:cacheprovider ${PYTEST_ARGS:-}; rc=$?
  ok $rc || exit $rc
fi
if [[ $STEPS == *smoke* ]]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
  ok $rc || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  step bench 900 python bench.py ${BENCH_ARGS:-}; rc=$?
  ok $rc || exit $rc
fi
exit 0
