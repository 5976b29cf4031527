"""Per-step GPU timeline from a rocprofv3 --kernel-trace database: the dispatches are cut into
steps at each launch of MARK (default: the fused forward kernel), and for the first STEPS
steps it prints the step span, the summed kernel time, the idle time, and the largest gaps
between consecutive kernels (with the kernels on either side) -- where the GPU waits for the
host.  Usage: step_timeline.py run_results.db [MARK] [STEPS]"""
import sqlite3
import sys

from kname import short_name

db = sqlite3.connect(sys.argv[1])
mark = sys.argv[2] if len(sys.argv) > 2 else "fused_fwd_kernel"
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 13
rows = db.execute("select name, start, end from kernels order by start").fetchall()


def short(n):
    return short_name(n)[:90]


cuts = [i for i, r in enumerate(rows) if mark in r[0]]
print(f"{len(rows)} dispatches, {len(cuts)} steps marked by {mark!r}")
gap_tot = {}
for s in range(min(nsteps, len(cuts) - 1)):
    a, b = cuts[s], cuts[s + 1]
    seg = rows[a:b]
    span = rows[b][1] - seg[0][1]
    busy = sum(e - st for _, st, e in seg)
    gaps = []
    for i in range(1, len(seg) + 1):
        nxt = rows[a + i]
        g = nxt[1] - seg[i - 1][2]
        if g > 0:
            gaps.append((g, short(seg[i - 1][0]), short(nxt[0])))
    gaps.sort(reverse=True)
    print(f"step {s}: {len(seg)} kernels, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"idle {(span - busy) / 1e3:.1f} us")
    for g, p, n in gaps[:6]:
        print(f"    gap {g / 1e3:7.1f} us  after {p}  before {n}")
    for g, p, n in gaps:
        gap_tot[(p, n)] = gap_tot.get((p, n), 0) + g
if gap_tot:
    print("largest gaps summed over the steps:")
    for (p, n), g in sorted(gap_tot.items(), key=lambda x: -x[1])[:8]:
        print(f"    {g / 1e3:8.1f} us  {p} -> {n}")
# one step's dispatch sequence (offset from the step start, duration), the last printed step
if len(cuts) > 1:
    s = min(nsteps, len(cuts) - 1) - 1
    a, b = cuts[s], cuts[s + 1]
    t0 = rows[a][1]
    print(f"step {s} sequence:")
    for n, st, e in rows[a:b]:
        print(f"    +{(st - t0) / 1e3:7.1f} us  {(e - st) / 1e3:7.1f} us  {short(n)}")
