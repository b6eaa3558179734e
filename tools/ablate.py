#!/usr/bin/env python3
"""Diagnostic: time the split scan (k_scan_struct + k_scan_tokens) under
kernel ablations (MSA_ABLATE bits, see msa_k3.hip / msa_api.hip), with its
LDS-table miss count.  The product library reads no MSA_ABLATE: build a
diagnostic variant (`make -C music-analyst-ai_amd variant V=abl
FLAGS="-DMSA_DIAG=1 -DK3_ABLATE=1"`, then MSA_LIB=.../build/libmsa_hip_abl.so).  Results of ablated runs are wrong by design; only the
stage times are read.  Usage: python tools/ablate.py [songs] [bits ...]"""
import ctypes as C
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
        lib = msa.load()
        lib.msa_debug_stat.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint64)]
        mv, tw = C.c_uint64(), C.c_uint64()
        lib.msa_debug_stat(c.h, b"k3_misses", C.byref(mv))
        lib.msa_debug_stat(c.h, b"total_words", C.byref(tw))
        fx = C.c_uint64()
        lib.msa_debug_stat(c.h, b"span_fix", C.byref(fx))
        print(f"ablate={b:2d} csv_scan={st.get('csv_scan')} ms  misses={mv.value} of {tw.value} words  span_fix={fx.value}  all={st}",
              flush=True)
