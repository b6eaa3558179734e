#!/usr/bin/env python3
"""One bench step as a timeline, from a rocprofv3 CSV run with
--kernel-trace --memory-copy-trace: python tools/timeline.py DIR [step]
DIR holds *_kernel_trace.csv (and *_memory_copy_trace.csv); a step starts at
a k_chunk_summary dispatch; step = index from the end (default 1 = the last
complete one).  Prints start offset (us), duration (us), queue/stream, name."""
import csv
import glob
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ev = []
for r in rows(os.path.join(d, "**", "*kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?") + "/" + r.get("Stream_Id", "?"),
               r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]))
for r in rows(os.path.join(d, "**", "*memory_copy_trace.csv")):
    n = int(r.get("Size", 0) or 0) if "Size" in r else 0
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy/" + r.get("Stream_Id", "?"),
               f"copy {r.get('Direction', '')} {n}B"))
ev.sort()
mark = os.environ.get("STEP_MARK", "k_chunk_summary")
starts = [i for i, e in enumerate(ev) if e[3] == mark]
if len(starts) < back + 1:
    sys.exit("not enough steps in the trace")
a, b = starts[-back - 1], starts[-back]
t0 = ev[a][0]
busy = 0
for s, e, q, n in ev[a:b]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {q:10s} {n}")
print(f"step: {(ev[b][0] - t0) / 1e3:.1f} us")
