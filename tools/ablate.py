#!/usr/bin/env python3
"""Diagnostic: time K3 (k_scan_main<0>) under kernel ablations (MSA_ABLATE bits,
see msa_scan.hip).  Results of ablated runs are wrong by design; only the
stage times are read.  Usage: python tools/ablate.py [songs] [bits ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "music-analyst-ai_amd"))
import msa  # noqa: E402

songs = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
bits = [int(b) for b in sys.argv[2:]] or [0, 1, 2, 4, 8, 9]
data = msa.gen_corpus(songs, mode="zipf", seed=1)
print(f"corpus {len(data)} bytes", flush=True)
for b in bits:
    os.environ["MSA_ABLATE"] = str(b)
    with msa.Context(0) as c:
        c.load_csv(data)
        c.set_profiling(True)
        c.run()
        c.profile(reset=True)
        for _ in range(3):
            c.run()
        p = c.profile(reset=True)
        st = {k: round(v["ms"] / v["launches"], 3) for k, v in p.items()}
        print(f"ablate={b:2d} csv_scan={st.get('csv_scan')} ms  all={st}", flush=True)
