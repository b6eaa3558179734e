#!/usr/bin/env python3
"""configs[4]: the adversarial high-cardinality corpus at scale -- stage times
(HIP events) of msa_run and the table sizes; with --oracle, byte parity of the
ranked outputs against oracle/msa_oracle as well.
Usage: python tools/highcard_bench.py [songs] [--oracle] [--steps K]"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "music-analyst-ai_amd"))
import msa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("songs", type=int, nargs="?", default=3_500_000)
ap.add_argument("--oracle", action="store_true")
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
t = time.time()
data = msa.gen_corpus(a.songs, mode="highcard", seed=4)
print(f"corpus {len(data)} bytes, {a.songs} songs, generated in {time.time() - t:.1f} s", flush=True)
with msa.Context(0) as c:
    c.load_csv(data)
    c.set_profiling(True)
    t = time.time()
    c.run(text_column=True)
    print(f"first run (tables grow) {time.time() - t:.2f} s", flush=True)
    c.profile(reset=True)
    t = time.time()
    for _ in range(a.steps):
        c.run(text_column=True)
    c.sync()
    dt = (time.time() - t) / a.steps
    p = c.profile(reset=True)
    s = c.summary()
    st = {k: round(v["ms"] / v["launches"], 3) for k, v in p.items()}
    print(f"ms/step {dt * 1e3:.2f}  GB/s {len(data) / dt / 1e9:.1f}  distinct words {s.n_words}  "
          f"artists {s.n_artists}  words {s.total_words}", flush=True)
    print("stages", st, flush=True)
    import ctypes
    c.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
    dbg = {}
    for nm in ("k3_misses", "mlog_full", "s_claimed", "m_claimed", "l_claimed", "split_attempts", "dense",
               "dense_veto"):
        v = ctypes.c_uint64(0)
        if c.lib.msa_debug_stat(c.h, nm.encode(), ctypes.byref(v)) == 0:
            dbg[nm] = v.value
    print("counters", dbg, flush=True)
    if a.oracle:
        d = tempfile.mkdtemp()
        p_ = os.path.join(d, "hc.csv")
        open(p_, "wb").write(data)
        t = time.time()
        r = subprocess.run([os.path.join(REPO, "oracle", "msa_oracle"), p_, "--output-dir", os.path.join(d, "o")],
                           capture_output=True, timeout=900)
        print(f"oracle rc {r.returncode} in {time.time() - t:.1f} s", flush=True)
        w = msa.table_csv_bytes(c.ranked(msa.MSA_TABLE_WORDS), "word")
        ar = msa.table_csv_bytes(c.ranked(msa.MSA_TABLE_ARTISTS), "artist")
        ew = open(os.path.join(d, "o", "word_counts.csv"), "rb").read()
        ea = open(os.path.join(d, "o", "top_artists.csv"), "rb").read()
        print(f"word_counts.csv identical: {w == ew} ({len(w)} bytes); top_artists.csv identical: {ea == ar}",
              flush=True)
