#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter found under a rocprofv3 output
directory (one or more --pmc passes): python tools/pmc_kernels.py DIR [filter]
LAST=k in the environment: only each kernel's last k dispatches per pass (the
steady state of a run whose first call grows its tables)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"]
            if flt not in k:
                continue
            key = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            c = acc[k][r["Counter_Name"]]
            c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
last = int(os.environ.get("LAST", "0"))
for k, cs in sorted(acc.items()):
    print(k[:90])
    for c, v in sorted(cs.items()):
        if last:
            keep = {}
            for f in {key[0] for key in v}:
                ids = sorted((key for key in v if key[0] == f), key=lambda key: int(key[1]))[-last:]
                keep.update({key: v[key] for key in ids})
            v = keep
        print(f"   {c:28s} {sum(v.values()) / len(v):16.1f}   (n={len(v)})")
