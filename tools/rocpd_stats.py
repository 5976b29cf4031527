"""Summarise a rocprofv3 rocpd database (--kernel-trace) into the --stats CSV shape:
name, calls, total_us, average_us, percentage (rocpd top_kernels reports microseconds).  Usage: rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys

from kname import short_name

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, total_calls, total_duration, average, percentage "
                  "from top_kernels").fetchall()
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, tot, avg, pct in rows:
        short = short_name(name)[:200]  # full instantiation, argument list dropped
        w.writerow([short, calls, f"{tot:.0f}", f"{avg:.1f}", f"{pct:.2f}"])
print(f"{len(rows)} kernels -> {sys.argv[2]}")
