#!/usr/bin/env python3
"""Diagnostic: the sharded pipeline of msa/dist.py (run_sharded +
gather_ranked) as a world of one (gloo, one process), for a kernel-trace
timeline of its exchange / import / re-rank overheads:
rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d D -o run -- python3 tools/prof_sharded.py [songs] [steps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "music-analyst-ai_amd"))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29511")
import torch.distributed as dist  # noqa: E402

import msa  # noqa: E402
from msa import dist as mdist  # noqa: E402

songs = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dist.init_process_group("gloo", rank=0, world_size=1)
comm = mdist.Comm()
data = msa.gen_corpus(songs, mode="zipf", seed=1)
with msa.Context(0) as ctx:
    ctx.load_csv(data)
    for _ in range(steps):
        mdist.run_sharded(ctx, comm, text_column=True)
        mdist.gather_ranked(ctx, comm, 0)
    ctx.sync()
dist.destroy_process_group()
print("done")
