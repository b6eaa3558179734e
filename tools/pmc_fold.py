#!/usr/bin/env python3
"""Per-kernel mean of every counter in the rocprofv3 --pmc CSV passes under a
directory (tools/pmc_hc.sh), the last dispatch of each kernel name excluded
when `--skip-first N` drops the first N dispatches (a table-growing first
run).  Prints JSON {kernel: {counter: mean}} for the kernels named on the
command line (all when none)."""
import collections
import csv
import glob
import json
import sys


def main():
    args = sys.argv[1:]
    skip = 0
    if args and args[0] == "--skip-first":
        skip = int(args[1])
        args = args[2:]
    d, names = args[0], set(args[1:])
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if names and k not in names:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: (sum(v[skip:]) / len(v[skip:]) if len(v) > skip else None) for c, v in sorted(cs.items())}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
