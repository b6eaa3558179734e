#!/usr/bin/env python3
"""Timeline of one C host bench-mode step (rank 0's process) from a rocprofv3
CSV run with --kernel-trace --memory-copy-trace:
python tools/timeline_chost.py DIR [pid-index]  -- steps start at k_chunk_summary."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
by_pid = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        by_pid[(f, r.get("Process_Id", "0"))].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                                      r.get("Queue_Id", "?"), r["Kernel_Name"].split("(")[0]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        by_pid[(f.replace("memory_copy", "kernel"), r.get("Process_Id", "0"))].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", "copy " + r.get("Direction", "")))
keys = sorted(by_pid, key=lambda k: -len(by_pid[k]))
ev = sorted(by_pid[keys[int(sys.argv[2]) if len(sys.argv) > 2 else 0]])
starts = [i for i, e in enumerate(ev) if e[3] == "k_chunk_summary"]
a, b = starts[-3], starts[-2]
t0 = ev[a][0]
for s, e, q, n in ev[a:b]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {q:6s} {n}")
print(f"step: {(ev[b][0] - t0) / 1e3:.1f} us")
