# binning buffers allocated before the preprocess: GPU tests, then interleaved A/B against the
# committed tree (abprev/) at c3 / c4 / headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05h11; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_fused_l1.py tests/test_gpu_fused.py tests/test_gpu_speculative.py tests/test_gpu_fullsize_fused.py \
  > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  for c in c3 c4 headline; do
    for t in prev cur; do
      d=.; [ $t = prev ] && d=abprev
      (cd $d && timeout -k 10 300 python3 bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-lane-occupancy --train-steps 50 > $O/b_${c}_${t}_$r.json 2>> $O/err.log) || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels'].get('(outside the C-ABI calls)',{}).get('ms_per_call'); print(sys.argv[2], d['value'], d['ms_per_step'], k, d['train_iters_per_s'], flush=True)" $O/b_${c}_${t}_$r.json "$c $t $r" >> $O/ab.log || exit $?
    done
  done
done
