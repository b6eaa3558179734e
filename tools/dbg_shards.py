#!/usr/bin/env python3
"""Debug: per-rank LOCAL word tables of a sharded world (after split + count,
before the merge), for comparing kernel variants (MSA_K3SPLIT=0/1).
  python tools/dbg_shards.py OUTDIR WORLD MODE SONGS SEED   (spawns the ranks itself)"""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "music-analyst-ai_amd")

WORKER = r'''
import json, os, sys
sys.path.insert(0, os.environ["MSA_PKG"])
import torch, torch.distributed as dist
import msa
from msa import dist as mdist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
cuts = json.loads(os.environ["MSA_CUTS"])
data = open(os.environ["MSA_CSV"], "rb").read()[cuts[rank]:cuts[rank + 1]]
ctx = msa.Context(0)
ctx.load_csv(data)
comm = mdist.Comm()
ctx.set_shard(comm.rank == 0)
tail = mdist.resolve_piece(ctx, comm, msa.PIECE_CSV)
ctx.split_columns(False)
import ctypes
ctx.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
dbg = {}
for nm in ("k3_misses", "total_words", "overflow", "s_claimed", "m_claimed", "s_table_used", "m_table_used", "split_attempts"):
    v = ctypes.c_uint64(0)
    ctx.lib.msa_debug_stat(ctx.h, nm.encode(), ctypes.byref(v))
    dbg[nm] = v.value
need = comm.all_reduce_sum([int(ctx.artist_reader_needed())])[0]
ctx.set_artist_reader(bool(need))
if need:
    mdist.resolve_piece(ctx, comm, msa.PIECE_ARTISTS)
ctx.count()
for nm in ("s_claimed", "m_claimed", "l_claimed"):
    v = ctypes.c_uint64(0)
    ctx.lib.msa_debug_stat(ctx.h, nm.encode(), ctypes.byref(v))
    dbg["count_" + nm] = v.value
s = ctx.summary()
ctx.rank()
w = ctx.ranked(msa.MSA_TABLE_WORDS)
out = os.environ["MSA_OUT"] + f".r{rank}"
open(out + ".words", "wb").write(msa.table_csv_bytes(w, "word"))
json.dump({"songs": s.total_songs, "words": s.total_words, "tail": tail, "n_words": s.n_words, "dbg": dbg, "n": ctx.piece_size(msa.PIECE_CSV)}, open(out + ".json", "w"))
ctx.close()
dist.destroy_process_group()
'''


def main():
    out, world, mode, songs, seed = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import msa
    msa.load()
    from test_gpu_dist import cuts_for
    os.makedirs(out, exist_ok=True)
    data = msa.gen_corpus(songs, mode=mode, seed=seed, vocab=8000)
    csv = os.path.join(out, "in.csv")
    open(csv, "wb").write(data)
    cuts = cuts_for(data, world, "in_quotes")
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    script = os.path.join(out, "w.py")
    open(script, "w").write(WORKER)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   MSA_PKG=PKG, MSA_CSV=csv, MSA_CUTS=json.dumps(cuts), MSA_OUT=os.path.join(out, "res"))
        procs.append(subprocess.Popen([sys.executable, script], env=env))
    rc = [p.wait(timeout=200) for p in procs]
    print("rcs", rc, "cuts", cuts)


if __name__ == "__main__":
    main()
