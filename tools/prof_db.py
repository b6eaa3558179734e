#!/usr/bin/env python3
"""Per-kernel stats from a rocprofv3 rocpd database (run_results.db):
python tools/prof_db.py DB [csv_out]  -> name, calls, total ms, avg ms, share."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
rows = db.execute(f"select {name}, count(*), sum(end-start), avg(end-start) from kernels group by {name} "
                  f"order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
lines = ["Name,Calls,TotalDurationNs,AverageNs,Percentage"]
for n, cnt, s, a in rows:
    lines.append(f'"{n}",{cnt},{s},{a:.1f},{100.0 * s / tot:.2f}')
    print(f"{s / 1e6:10.3f} ms {cnt:6d}x avg {a / 1e3:9.2f} us  {100.0 * s / tot:5.1f}%  {n[:80]}")
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write("\n".join(lines) + "\n")
