"""Summarise a rocprofv3 rocpd database (--kernel-trace) into the --stats CSV shape:
name, calls, total_us, average_us, percentage (rocpd top_kernels reports microseconds).  Usage: rocpd_stats.py run_results.db out.csv"""
import csv
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, total_calls, total_duration, average, percentage "
                  "from top_kernels").fetchall()
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, tot, avg, pct in rows:
        short = name.replace("(anonymous namespace)::", "")
        if short.startswith("void gs::") or short.startswith("gs::"):
            short = re.sub(r"\(.*$", "", short)  # drop the argument list of our kernels
        short = short[:160]
        w.writerow([short, calls, f"{tot:.0f}", f"{avg:.1f}", f"{pct:.2f}"])
print(f"{len(rows)} kernels -> {sys.argv[2]}")
