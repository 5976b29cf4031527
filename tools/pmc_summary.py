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
import sys

from kname import short_name

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
# dispatches of each instantiation per pass (file): the bench picks the most-dispatched
# instantiation of an entry's kernel -- the one its timed step ran -- for per-step figures
ndisp = collections.defaultdict(lambda: collections.defaultdict(set))
cfg_arg = sys.argv[4] if len(sys.argv) > 4 else "headline"
files = glob.glob(os.path.join(root, "pmc", cfg_arg + "_*", "**", "*counter_collection.csv"),
                  recursive=True)
for f in files:
    for r in csv.DictReader(open(f)):
        name = short_name(r["Kernel_Name"])
        if not name.startswith(("void gs::", "gs::")):
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        ndisp[name][f].add(r.get("Dispatch_Id"))
# Per C-ABI entry of the binning, whose kernels (radix passes, scans) are shared between the
# depth sort (gsplat_bin_count_keyed) and the tile sort (gsplat_bin_emit): segment each pass's
# dispatch sequence -- a fused forward kernel starts a step's binning, the emission's first
# kernel (emit / tc_first / ep0_count, or the tile buckets' bk_count) starts bin_emit,
# bins_decode (the buckets: the long-list bk_sort) ends it -- and average the per-call sums of
# every counter over the calls seen.
# the emission's pre-launched head (gsplat_bin_emit_prelaunch), then the rest
# (gsplat_bin_emit_finish; all of it when the first tile pass is generated)
EMIT_HEAD = ("emit_kernel", "bk_count_kernel", "bk_scan_kernel", "bk_place_kernel")
EMIT_START = EMIT_HEAD + ("tc_first_kernel", "ep0_count_kernel")
EMIT_END = ("bins_decode_kernel", "ts_decode_kernel", "bk_sort_kernel<1024")
PRE, FIN = "gsplat_bin_emit_prelaunch", "gsplat_bin_emit_finish"
SPEC = "gsplat_bin_speculative"
entries = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in files:
    disp = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        if "Dispatch_Id" not in r:
            break
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    state, seg = None, 0
    count_part = []  # this segment's count-phase dispatches (re-labelled for the one-call binning)
    for d in sorted(disp):
        k = names[d]
        if "fused_fwd_kernel" in k or "fused_fwd_proj_kernel" in k or "project_fwd_kernel" in k:
            state, seg, count_part = "gsplat_bin_count_keyed_ex", seg + 1, []
            continue
        if state == "gsplat_bin_count_keyed_ex" and ("emit_scan_kernel" in k or
                                                      "ts_emit_kernel" in k):
            # gsplat_bin_speculative (rounds 4 and 5): count, emission and tile sort in one entry
            for dd in count_part:
                for c, v in disp[dd].items():
                    entries[state][(os.path.dirname(f), c)] -= v
                    entries[SPEC][(os.path.dirname(f), c)] += v
            state = SPEC
        elif state == "gsplat_bin_count_keyed_ex" and any(s in k for s in EMIT_START):
            state = PRE if any(s in k for s in EMIT_HEAD) else FIN
        elif state == PRE and not any(s in k for s in EMIT_HEAD):
            state = FIN
        if state is None:
            continue
        if not k.startswith("gs::") and not k.startswith("void gs::"):
            continue
        if "fused_fwd_sh_kernel" in k:  # (the preprocess's colour part, on its own stream)
            continue
        for c, v in disp[d].items():
            entries[state][(os.path.dirname(f), c)] += v
        calls[state].add((os.path.dirname(f), seg))
        if state == "gsplat_bin_count_keyed_ex":
            count_part.append(d)
        if state in (FIN, SPEC) and any(s in k for s in EMIT_END):
            state = None
entry_rows = {}
for e, d in entries.items():
    per = collections.defaultdict(list)
    ncall = collections.Counter(run for run, _ in calls[e])
    for (run, c), v in d.items():
        per[c].append(v / max(ncall[run], 1))
    entry_rows[e] = {c: sum(v) / len(v) for c, v in per.items()}
rows = []
for k, d in sorted(acc.items()):
    row = {"kernel": k, "dispatches": sum(len(v) for v in ndisp[k].values()) / max(len(ndisp[k]), 1)}
    for c, v in sorted(d.items()):
        row[c] = sum(v) / len(v)
    rows.append(row)
cols = sorted({c for r in rows for c in r if c not in ("kernel", "dispatches")})
if len(sys.argv) > 3:
    def pick(r):
        return {"fetch_kb": r.get("FETCH_SIZE"), "write_kb": r.get("WRITE_SIZE"),
                "valu_quad_cycles": r.get("SQ_ACTIVE_INST_VALU"),
                "insts_valu": r.get("SQ_INSTS_VALU"),
                "insts_trans": r.get("SQ_INSTS_VALU_TRANS_F32"),
                "wait_any": r.get("SQ_WAIT_ANY"),
                "wait_inst_any": r.get("SQ_WAIT_INST_ANY"),
                "wave_cycles": r.get("SQ_WAVE_CYCLES"),
                "dispatches": r.get("dispatches")}
    tj = {r["kernel"]: pick(r) for r in rows if "FETCH_SIZE" in r and "WRITE_SIZE" in r}
    ej = {e: pick(r) for e, r in entry_rows.items() if "FETCH_SIZE" in r and "WRITE_SIZE" in r}
    cfg = cfg_arg
    try:
        with open(sys.argv[3]) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    doc.setdefault("source", "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_ACTIVE_INST_VALU "
                             "(quad-cycles), separate passes, tools/pmc_bench.sh")
    doc.setdefault("configs", {})[cfg] = {"kernels": tj, "entries": ej}
    with open(sys.argv[3], "w") as f:
        json.dump(doc, f, indent=1)
out = sys.argv[2] if len(sys.argv) > 2 else None
w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
w.writerow(["kernel", "dispatches"] + cols)
for r in rows:
    w.writerow([r["kernel"], f"{r['dispatches']:.0f}"] + [f"{r.get(c, float('nan')):.4g}" for c in cols])
