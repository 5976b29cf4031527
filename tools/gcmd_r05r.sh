# round 5: same-box A/B of the round-3 (74cdd45), round-4 (e7a2031) and current trees, each
# with its own bench.py and libraries (tools/build_tree.sh), at c5 (train it/s) and c4 (the
# unchanged-caller path): VERDICT r4 weak #6
set -o pipefail
O=$PWD/gpurun_out/r05r; mkdir -p $O
for r in 1 2; do
for c in c5 c4; do
for t in ab/r03 ab/r04t .; do
  n=$(basename $t); [ "$t" = "." ] && n=r05
  (cd $t && timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-lane-occupancy --train-steps 10 > $O/b_${c}_${n}_$r.json 2> $O/b_${c}_${n}_$r.err) || { echo "[$t $c] failed"; tail -5 $O/b_${c}_${n}_$r.err; exit 1; }
  python3 - "$c" "$n" "$O/b_${c}_${n}_$r.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
k = {n.replace("gsplat_", "")[:26]: round(v["ms_per_call"], 4) for n, v in d["kernels"].items()}
print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], d.get("value_unchanged_caller"), d.get("train_iters_per_s"), k, flush=True)
PY
done
done
done
