# round 5: the whole GPU suite and smoke() on the current tree
set -o pipefail
O=gpurun_out/r05suite; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1; rc=$?
echo "[suite] rc=$rc"; tail -5 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
echo "[smoke] rc=$rc"; tail -3 $O/smoke.log
exit $rc
