"""Per-kernel averages of rocprofv3 --pmc CSV passes (tools/pmc_bench.sh output).
Usage: pmc_summary.py gpurun_out [out.csv] [traffic.json [config]]

traffic.json (read by bench.py for roofline.traffic): per device kernel, the mean per-dispatch
FETCH_SIZE and WRITE_SIZE in KiB as rocprofv3 reports them (uncorrected), stored under the bench
config the counters were collected on (default headline); other configs' entries are kept."""
import json
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
cfg_arg = sys.argv[4] if len(sys.argv) > 4 else "headline"
files = glob.glob(os.path.join(root, "pmc", cfg_arg + "_*", "**", "*counter_collection.csv"),
                  recursive=True)
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if name.startswith("void gs::") or name.startswith("gs::"):
            name = re.sub(r"\(.*$", "", name)
        else:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, d in sorted(acc.items()):
    row = {"kernel": k}
    for c, v in sorted(d.items()):
        row[c] = sum(v) / len(v)
    rows.append(row)
cols = sorted({c for r in rows for c in r if c != "kernel"})
if len(sys.argv) > 3:
    tj = {r["kernel"]: {"fetch_kb": r.get("FETCH_SIZE"), "write_kb": r.get("WRITE_SIZE"),
                        "valu_quad_cycles": r.get("SQ_ACTIVE_INST_VALU"),
                        "insts_valu": r.get("SQ_INSTS_VALU"),
                        "insts_trans": r.get("SQ_INSTS_VALU_TRANS_F32"),
                        "wait_inst_any": r.get("SQ_WAIT_INST_ANY"),
                        "wave_cycles": r.get("SQ_WAVE_CYCLES")}
          for r in rows if "FETCH_SIZE" in r and "WRITE_SIZE" in r}
    cfg = cfg_arg
    try:
        with open(sys.argv[3]) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    doc.setdefault("source", "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_ACTIVE_INST_VALU "
                             "(quad-cycles), separate passes, tools/pmc_bench.sh")
    doc.setdefault("configs", {})[cfg] = {"kernels": tj}
    with open(sys.argv[3], "w") as f:
        json.dump(doc, f, indent=1)
out = sys.argv[2] if len(sys.argv) > 2 else None
w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
w.writerow(["kernel"] + cols)
for r in rows:
    w.writerow([r["kernel"]] + [f"{r.get(c, float('nan')):.4g}" for c in cols])
