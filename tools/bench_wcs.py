"""Bench of the per-song word counter (DESIGN.md row f): msa_wcs_run over a
synthetic Zipfian lyric CSV resident in HBM (same generator and size as the
main bench: 5M songs, ~1.2 GB), one JSON line on stdout.

    python tools/bench_wcs.py [--songs N] [--steps K] [--warmup W] [--no-cpu-baseline]

The timed step is the whole msa_wcs_run (validation, row split, per-row
tokenise + count, ranking, by-song lines; results left in HBM) -- it syncs
with the host between phases, so wall-clock around it is the step time.
cpu_baseline: oracle/wcs_oracle.py (pure-Python restatement of the script,
kind "port", 1 core) on a bounded sample of the same corpus.

roofline: the dominant kernel k_wcs_wrows (wave per window of whole rows),
timed with HIP events on the library's stream (msa_wcs_kernel_ms); its
algorithmic bytes per launch = every input byte read once + 48 B per row
(row end 8 B read; distinct-word count 8 B and artist/song spans 32 B
written) + 8 B per (song, word) line written (n_pairs); `traffic` from the
PMC file of tools/pmc_rowf.sh when it is stamped with this build, else null.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "music-analyst-ai_amd"))
import msa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--songs", type=int, default=5_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", choices=["wcs", "split"], default="wcs",
                    help="wcs: msa_wcs_run (per-song counts); split: msa_csvcol_run (column files in HBM)")
    a = ap.parse_args()
    if a.path == "split":
        return bench_split(a)
    data = msa.gen_corpus(a.songs, mode="zipf", seed=1)
    n = len(data)
    lib = msa.load()
    import ctypes as C

    lib.msa_wcs_kernel_ms.argtypes = [C.c_void_p]
    lib.msa_wcs_kernel_ms.restype = C.c_double
    kms = []
    with msa.WordCountPerSong(0) as w:
        w.load_csv(data)
        for _ in range(a.warmup):
            w.count()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            w.count()
            kms.append(lib.msa_wcs_kernel_ms(w.h))
        dt = (time.perf_counter() - t0) / a.steps
        s = w.summary()
    k_ms = sum(kms) / len(kms)
    alg = n + 48 * s["total_rows"] + 8 * s["n_pairs"]
    achieved = alg / (k_ms * 1e-3) / 1e9
    roof = {"kernel": "k_wcs_wrows", "bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
            "frac": round(achieved / 8000.0, 4), "traffic": None, "avg_launch_ms": round(k_ms, 4),
            "alg_bytes_per_launch": alg}
    pmc = os.path.join(REPO, "profiles", "pmc_wcs_main.json")
    if os.path.exists(pmc):
        p = json.load(open(pmc))
        k = p.get("kernels", {}).get("k_wcs_wrows")
        if p.get("build_id") == msa.build_id() and p.get("input_bytes") == n and k:
            roof["traffic"] = k["hbm_bytes_per_launch"]
            roof["traffic_over_alg"] = round(k["hbm_bytes_per_launch"] / alg, 3)
        else:
            roof["counters"] = {"note": "PMC file not taken on this build / corpus"}
    out = {
        "metric": "CSV->per-song word counts GB/s (word_count_per_song.py path)",
        "value": round(n / dt / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u8",
        "data": "synthetic (csrc/msa_gen.c Zipfian lyric CSV, seed 1)",
        "config": {"workload": f"{a.songs} songs, {n} bytes, resident in HBM", "bytes_per_gpu": n, "summary": s},
        "roofline": roof,
    }
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import wcs_oracle  # checker restatement, timed as the CPU baseline only

        sample = msa.gen_corpus(20000, mode="zipf", seed=1)
        t0 = time.perf_counter()
        wcs_oracle.word_count_per_song(sample)
        ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(sample) / ct / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
                               "seconds": round(ct, 3),
                               "sample": f"20000 songs, {len(sample)} bytes, oracle/wcs_oracle.py (pure Python)"}
    print(json.dumps(out), flush=True)


def bench_split(a):
    """The column splitter (msa_csvcol_run).  roofline: its copy phase -- one
    k_col_gather per column (every value that is a raw copy of its input
    bytes, coalesced 16-byte stores) and k_csvcol<1> over the rows holding
    another value -- HIP events on the library's stream around the phase
    (msa_csvcol_kernel); algorithmic bytes per run = the column bytes read
    from the input and written (2 x column bytes) + 16 B per cell (its output
    offset and source); `traffic` = the phase's PMC bytes per run (the
    gathers' and k_csvcol<1>'s, tools/pmc_split.sh -> profiles/pmc_split_main.json
    "copy_phase") when that file is stamped with this build."""
    import ctypes as C

    data = msa.gen_corpus(a.songs, mode="zipf", seed=1)
    n = len(data)
    lib = msa.load()
    lib.msa_csvcol_kernel.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    kms, outb = [], 0
    with msa.WordCountPerSong(0) as w:
        w.load_csv(data)
        for _ in range(a.warmup):
            w.split_columns(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            nc, nr = w.split_columns(True)
            ms, ob = C.c_double(), C.c_uint64()
            lib.msa_csvcol_kernel(w.h, C.byref(ms), C.byref(ob))
            kms.append(ms.value)
            outb = ob.value
        dt = (time.perf_counter() - t0) / a.steps
    k_ms = sum(kms) / len(kms)
    alg = 2 * outb + 16 * nc * nr
    achieved = alg / (k_ms * 1e-3) / 1e9
    roof = {"kernel": "k_col_gather x columns + k_csvcol<1> (copy phase)", "bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
            "frac": round(achieved / 8000.0, 4), "traffic": None, "avg_launch_ms": round(k_ms, 4),
            "alg_bytes_per_launch": alg}
    pmc = os.path.join(REPO, "profiles", "pmc_split_main.json")
    if os.path.exists(pmc):
        p = json.load(open(pmc))
        k = p.get("kernels", {}).get("copy_phase")
        if p.get("build_id") == msa.build_id() and p.get("input_bytes") == n and k:
            roof["traffic"] = k["hbm_bytes_per_launch"]
            roof["traffic_over_alg"] = round(k["hbm_bytes_per_launch"] / alg, 3)
        else:
            roof["counters"] = {"note": "PMC file not taken on this build / corpus"}
    out = {"metric": "CSV->per-column files GB/s (split_csv_columns.py path)", "value": round(n / dt / 1e9, 3),
           "unit": "GB/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3),
           "higher_is_better": True, "dtype": "u8", "data": "synthetic (csrc/msa_gen.c Zipfian lyric CSV, seed 1)",
           "config": {"workload": f"{a.songs} songs, {n} bytes, resident in HBM", "bytes_per_gpu": n, "columns": nc,
                      "rows": nr, "column_bytes": outb},
           "roofline": roof}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import split_oracle  # checker restatement, timed as the CPU baseline only

        sample = msa.gen_corpus(20000, mode="zipf", seed=1)
        t0 = time.perf_counter()
        split_oracle.split_columns(sample, True)
        ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(sample) / ct / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
                               "seconds": round(ct, 3),
                               "sample": f"20000 songs, {len(sample)} bytes, oracle/split_oracle.py (pure Python)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
