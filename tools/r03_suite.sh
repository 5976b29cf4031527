set -o pipefail
L=gpurun_out/suite.log; : > $L
S=tools/gpu_step.sh
$S 900 $L python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests/ -rf || exit 1
$S 300 $L python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
