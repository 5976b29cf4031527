# train iters/s at c2 / c3: the tree before the direct step (abprev/) vs the current one, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05h7; mkdir -p $O
for r in 1 2; do
  for c in c2 c3; do
    for t in prev cur; do
      d=.; [ $t = prev ] && d=abprev
      (cd $d && timeout -k 10 300 python3 bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-lane-occupancy --train-steps 200 > $O/b_${c}_${t}_$r.json 2>> $O/err.log) || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['train_iters_per_s'], flush=True)" $O/b_${c}_${t}_$r.json "$c $t $r" >> $O/ab.log || exit $?
    done
  done
done
