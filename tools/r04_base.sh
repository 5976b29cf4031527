set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-lane-occupancy --train-steps 20 > gpurun_out/r04/base_headline.json 2> gpurun_out/r04/base_headline.err || exit $?
timeout -k 10 300 python3 bench.py --config c3 --steps 50 --warmup 10 --no-cpu-baseline --no-lane-occupancy --train-steps 20 > gpurun_out/r04/base_c3.json 2> gpurun_out/r04/base_c3.err || exit $?
CFGS="headline c3" bash tools/r03_timeline.sh || exit $?
cp gpurun_out/timeline_headline.txt gpurun_out/r04/base_timeline_headline.txt
cp gpurun_out/timeline_c3.txt gpurun_out/r04/base_timeline_c3.txt
