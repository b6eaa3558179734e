"""Diagnostic: one forced-dense run of a highcard corpus, the dense counters printed."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "music-analyst-ai_amd"))
os.environ["MSA_DENSE_MIN"] = "0"
import msa  # noqa: E402

data = msa.gen_corpus(int(sys.argv[1]) if len(sys.argv) > 1 else 150_000, mode="highcard", seed=31)
with msa.Context(0) as c:
    c.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]

    def st(n):
        v = ctypes.c_uint64(0)
        r = c.lib.msa_debug_stat(c.h, n.encode(), ctypes.byref(v))
        return v.value if r == 0 else f"err{r}"
    for k in range(2):
        c.load_csv(data)
        c.run(text_column=True)
        print(k, {n: st(n) for n in ["dense", "dense_veto", "dense_n", "s_claimed", "m_claimed", "split_attempts",
                                     "k3_misses", "mlog_full", "overflow"]}, flush=True)
