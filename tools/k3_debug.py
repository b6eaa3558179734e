#!/usr/bin/env python3
"""Diagnostic: run the CSV scan with the current K3 and the round-1 kernel
(MSA_ABLATE=64) on torture corpora and print the first record whose
rec_start / nulrel / word counts differ."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "music-analyst-ai_amd"))
import msa  # noqa: E402


def arrays(data, ablate):
    os.environ["MSA_ABLATE"] = str(ablate)
    with msa.Context(0) as c:
        c.load_csv(data)
        c.split_columns(True)
        lib = c.lib
        n = C.c_uint64()
        lib.msa_debug_records.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        lib.msa_debug_records(c.h, None, None, 0, C.byref(n))
        rs = (C.c_uint64 * (n.value + 1))()
        nr = (C.c_uint32 * (n.value + 1))()
        lib.msa_debug_records(c.h, rs, nr, n.value + 1, C.byref(n))
        c.count()
        c.rank()
        w = c.ranked(msa.MSA_TABLE_WORDS)
        return list(rs), list(nr), w, c.summary()


for mode, seed, songs in [("torture", s, 1500) for s in range(1, 9)] + [("zipf", 3, 3000), ("highcard", 4, 3000)]:
    data = msa.gen_corpus(songs, mode=mode, seed=seed)
    a = arrays(data, 0)
    b = arrays(data, 64)
    bad = False
    n = min(len(a[0]), len(b[0]))
    for i in range(n - 1):
        if a[0][i] != b[0][i] or a[1][i] != b[1][i]:
            s = b[0][i]
            e = b[0][i + 1] if i + 1 < len(b[0]) else len(data)
            print(f"{mode}{seed}: record {i}: new rs={a[0][i]} nul={a[1][i]}  old rs={b[0][i]} nul={b[1][i]} "
                  f"bytes[{s}:{e}]={data[s:e][:160]!r} prev={data[max(0, s - 40):s]!r}")
            bad = True
            break
    if len(a[0]) != len(b[0]):
        print(f"{mode}{seed}: nrec differ {len(a[0])} vs {len(b[0])}")
        bad = True
    if a[2] != b[2]:
        da = dict(a[2]); db = dict(b[2])
        diffs = [(k, da.get(k), db.get(k)) for k in set(da) | set(db) if da.get(k) != db.get(k)]
        print(f"{mode}{seed}: words differ in {len(diffs)} keys, e.g. {diffs[:5]}; totals {a[3].total_words} vs {b[3].total_words}")
        bad = True
    print(f"{mode}{seed}: {'DIFF' if bad else 'same'}", flush=True)
