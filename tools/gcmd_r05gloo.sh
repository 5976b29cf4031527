# round 5: the bench's N > 1 path rehearsed over gloo (2 ranks on the one GPU) at c4 and headline
set -o pipefail
ROUND=r05gloo GLOO2=1 GLOO2_CFG=c4 bash tools/gpu_iter.sh || exit $?
cp gpurun_out/r05gloo/gloo2_c4.json gpurun_out/r05gloo/keep_c4.json
ROUND=r05gloo GLOO2=1 GLOO2_CFG=headline bash tools/gpu_iter.sh || exit $?
for c in c4 headline; do f=gpurun_out/r05gloo/gloo2_$c.json; [ $c = c4 ] && f=gpurun_out/r05gloo/keep_c4.json
python3 - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"][:40], d["value"], "2views", d.get("value_2_views_per_gpu"), json.dumps(d["exchange"]))
print({k: v for k, v in d["kernels"].items() if "exchange" in k})
PY
done
