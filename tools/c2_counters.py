"""configs[2] split counters (msa_debug_stat) after one run: how many records
k_rec_fast hands to k_rec_fix, the miss-log entries, the tables' claims.
Run ON the GPU box:  python3 tools/c2_counters.py [songs]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "music-analyst-ai_amd"))
import msa  # noqa: E402

songs = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
data = msa.gen_corpus(songs, seed=1)
c = msa.Context(0)
c.load_csv(data)
for _ in range(2):
    c.run(text_column=True)
c.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
out = {}
for nm in ("span_fix", "k3_misses", "mlog_full", "s_claimed", "m_claimed", "l_claimed", "total_words", "dense"):
    v = ctypes.c_uint64(0)
    if c.lib.msa_debug_stat(c.h, nm.encode(), ctypes.byref(v)) == 0:
        out[nm] = v.value
print(len(data), out, flush=True)
