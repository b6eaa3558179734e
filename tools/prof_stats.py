#!/usr/bin/env python3
"""Per-kernel summary (rocprofv3 --kernel-trace --stats layout) from a
rocprofv3 results database: python tools/prof_stats.py run_results.db > out.csv"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                  "from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for name, n, s, a, lo, hi in rows:
    w.writerow([name, n, s, round(a, 1), round(100.0 * s / tot, 2), lo, hi])
