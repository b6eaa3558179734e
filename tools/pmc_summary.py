#!/usr/bin/env python3
"""Fold the rocprofv3 PMC passes of tools/pmc.sh into profiles/pmc_scan_main.json.

HBM bytes per K3 launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports
both in KiB, and on gfx950 FETCH_SIZE counts exactly half of a wide (16 B/lane)
coalesced streaming read (MI355X_MICROARCH.md, HBM section) -- K3 reads the CSV
that way.  The SQ pass is summarised as-is (per launch means)."""
import csv
import glob
import json
import os
import sys

KERNEL = "k_scan_main<0>"


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def per_launch(d, counter):
    vals = {}
    for r in rows(d):
        if KERNEL not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return (sum(vals.values()) / len(vals), len(vals)) if vals else (None, 0)


def bench_line(log):
    try:
        for line in open(log):
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    except OSError:
        pass
    return None


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    fetch, nf = per_launch(os.path.join(out, "fetch"), "FETCH_SIZE")
    write, nw = per_launch(os.path.join(out, "write"), "WRITE_SIZE")
    sq = {}
    for c in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS",
              "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_ANY"):
        v, _ = per_launch(os.path.join(out, "sq"), c)
        sq[c] = v
    b = bench_line(os.path.join(out, "fetch.log"))
    res = {
        "kernel": KERNEL,
        "input_bytes": b["config"]["bytes_per_gpu"] if b else None,
        "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"] if b else None,
        "fetch_size_kib_per_launch": fetch,
        "write_size_kib_per_launch": write,
        "launches_seen": {"fetch": nf, "write": nw},
        "hbm_bytes_per_launch": int((2 * fetch + write) * 1024) if fetch is not None and write is not None else None,
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halves 16B/lane streams)",
        "sq_per_launch": sq,
    }
    # written next to the passes (gpurun_out/ travels back); copy to profiles/
    with open(os.path.join(out, "pmc_scan_main.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
