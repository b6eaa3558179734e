#!/usr/bin/env python3
"""Fold the rocprofv3 PMC passes of tools/pmc.sh into OUT/pmc.json (copied to
profiles/pmc_scan_main.json).

Per kernel of the bench step, per launch (mean over dispatches):
  hbm_bytes   = (2 x FETCH_SIZE + WRITE_SIZE) x 1024.  rocprofv3 reports both in
                KiB; on gfx950 FETCH_SIZE counts exactly half of a wide (16 B/lane)
                coalesced streaming read (MI355X_MICROARCH.md, HBM section).  The
                correction is exact for k_scan_csv / k_chunk_summary (dwordx4 per
                lane streams); for gather-type kernels fetch_raw_bytes is given too.
  atomics     TCC_ATOMIC_sum (atomics reaching the L2), TCC_EA0_ATOMIC_sum
                (atomics leaving the L2 to memory), TA_*_ATOMIC_WAVEFRONTS_sum
                (atomic wave instructions issued), SQ_INSTS_LDS_ATOMIC
  sq          SQ_LDS_BANK_CONFLICT (cycles), SQ_INSTS_LDS, waits, ...
The file is stamped with the build id of the libmsa_hip.so in this tree
(msa_build_id(): hash of the kernel sources + flags, stable across rebuilds)
and with the bench line the passes ran (input bytes, K3 algorithmic bytes)."""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "music-analyst-ai_amd"))
KERNELS = ["k_scan_csv", "k_scan_struct", "k_scan_tokens", "k_miss_agg", "k_chunk_summary", "k_rec_spans", "k_rec_fast", "k_rec_fix", "k_col_gather", "k_col_lines",
           "k_artist_count", "k_tile_sort", "k_merge_pass",
           # the per-song counter (tools/pmc_wcs.sh, --wcs)
           "k_wcs_wrows", "k_wcs_rows", "k_wcs_map", "k_wcs_emit", "k_wcs_validate", "k_wcs_pairs",
           # the column splitter (tools/pmc_split.sh, --split): its two passes apart
           "k_csvcol<0>", "k_csvcol<1>"]
PASSES = ["fetch", "write", "sq", "atomic", "sq2"]


def build_id():
    import msa  # ctypes only: no GPU call

    return msa.build_id()


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    for k in KERNELS:
        if name.startswith(k + "(") or name.startswith(k + "<") or name == k:
            return k
    return None


def collect(out):
    acc = {}  # kernel -> counter -> {dispatch: value}
    for p in PASSES:
        for f in glob.glob(os.path.join(out, p, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = short(r.get("Kernel_Name", ""))
                    if not k:
                        continue
                    key = (p, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                    c = acc.setdefault(k, {}).setdefault(r["Counter_Name"], {})
                    c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def bench_line(log):
    try:
        for line in open(log):
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    except OSError:
        pass
    return None


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    wcs = "--wcs" in sys.argv  # passes over tools/bench_wcs.py: the roofline kernel is k_wcs_wrows
    split = "--split" in sys.argv  # passes over tools/bench_wcs.py --path split: its copy phase
    out = args[0] if args else "gpurun_out/pmc"
    per = collect(out)
    kernels = {}
    for k, c in per.items():
        e = {"counters": c}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            e["fetch_raw_bytes_per_launch"] = int(c["FETCH_SIZE"] * 1024)
            e["write_bytes_per_launch"] = int(c["WRITE_SIZE"] * 1024)
        kernels[k] = e
    b = bench_line(os.path.join(out, "fetch.log"))
    # the bench line names the roofline kernel ("k_scan_tokens (csv_tokens)", ...)
    if split and b and "k_col_gather" in kernels and "k_csvcol<1>" in kernels:
        # the splitter's copy phase per run: one k_col_gather per column + k_csvcol<1>
        nc = b["config"]["columns"]
        g, c1 = kernels["k_col_gather"], kernels["k_csvcol<1>"]
        kernels["copy_phase"] = {k: nc * g[k] + c1[k] for k in
                                 ("hbm_bytes_per_launch", "fetch_raw_bytes_per_launch", "write_bytes_per_launch")
                                 if k in g and k in c1}
        kernels["copy_phase"]["counters"] = {"note": f"{nc} x k_col_gather + k_csvcol<1>, per run"}
    rk = "k_wcs_wrows" if wcs else ("copy_phase" if split else
                                    ((b or {}).get("roofline", {}).get("kernel", "k_scan_csv").split(" ")[0]))
    res = {
        "build_id": build_id(),
        "input_bytes": b["config"]["bytes_per_gpu"] if b else None,
        "roofline_kernel": rk,
        "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"] if b else None,
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halves 16B/lane streams)",
        "command": ("tools/pmc_wcs.sh: rocprofv3 --pmc <group> -- python3 tools/bench_wcs.py --steps 1 --warmup 1 "
                    "--no-cpu-baseline" if wcs else
                    "tools/pmc_split.sh: rocprofv3 --pmc <group> -- python3 tools/bench_wcs.py --path split --steps 1 "
                    "--warmup 1 --no-cpu-baseline" if split else
                    "tools/pmc.sh: rocprofv3 --pmc <group> -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pcie"),
        "kernels": kernels,
    }
    k3 = kernels.get(rk, {})
    if res["alg_bytes_per_launch"] and k3.get("hbm_bytes_per_launch"):
        res["traffic_over_alg"] = round(k3["hbm_bytes_per_launch"] / res["alg_bytes_per_launch"], 3)
    with open(os.path.join(out, "pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    for k, e in sorted(kernels.items()):
        print(k, json.dumps({x: (round(y, 1) if isinstance(y, float) else y) for x, y in e["counters"].items()}))
        if "hbm_bytes_per_launch" in e:
            print("   hbm bytes/launch", e["hbm_bytes_per_launch"])
    print("traffic_over_alg", res.get("traffic_over_alg"))


if __name__ == "__main__":
    main()
