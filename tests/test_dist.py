"""CPU: the multi-GPU routing and exchange logic of msa/dist.py with a gloo
world of 2-3 processes.  The GPU kernels are replaced by a small host stand-in
(FakeCtx) so that the boundary plan, the head exchange, the partitioned merge
and the final ranked gather (full and top-k) are exercised exactly as on RCCL; the GPU-backed
version of the same flow is tests/test_gpu_dist.py."""
import ctypes
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG  # noqa: F401  (puts the package on sys.path)
from msa import dist as mdist


# ------------------------------------------------------------- pure routing
def test_head_owners():
    assert mdist.head_owners([0, 5, 0, 3], [10, 10, 10, 10]) == [-1, 0, -1, 2]
    # rank 1 is entirely the middle of a record begun on rank 0
    assert mdist.head_owners([0, 10, 4], [10, 10, 10]) == [-1, 0, 0]
    assert mdist.head_owners([0, 10, 10, 0], [10, 10, 10, 10]) == [-1, 0, 0, -1]


def test_tail_plan():
    heads, sizes = [0, 10, 4], [10, 10, 10]
    assert mdist.tail_plan(0, heads, sizes) == ([0, 0, 0], [0, 10, 4])
    assert mdist.tail_plan(1, heads, sizes) == ([10, 0, 0], [0, 0, 0])
    assert mdist.tail_plan(2, heads, sizes) == ([4, 0, 0], [0, 0, 0])


# ------------------------------------------------------------ host stand-in
def record_starts(data: bytes):
    """Record starts of read_csv_record (parallel_spotify.c:549-633)."""
    starts, i, n = [0], 0, len(data)
    q = 0
    while i < n:
        c = data[i]
        i += 1
        if c == 0x22:
            if not q:
                q = 1
            elif i < n and data[i] == 0x22:
                i += 1
            else:
                q = 0
        elif not q and c in (0x0A, 0x0D):
            if c == 0x0D and i < n and data[i] == 0x0A:
                i += 1
            if i < n:
                starts.append(i)
    return starts


class FakeCtx:
    """Stands in for msa.Context: knows the whole logical file only to answer
    shard_head (the GPU computes it from the all-gathered shard functions)."""

    def __init__(self, full: bytes, lo: int, hi: int):
        self.full, self.lo, self.hi = full, lo, hi
        self.shard = full[lo:hi]
        self.skip, self.tail = 0, b""
        self.exported = b""
        self.counts, self.merged = {}, {}

    def piece_size(self, piece):
        return len(self.shard)

    def shard_function(self, piece):
        return hashlib.sha256(self.shard).digest()[:mdist.SHARD_FN_BYTES // 4] * 4

    def shard_head(self, piece, fns, sizes):
        nxt = [s for s in record_starts(self.full) if s >= self.lo]
        first = nxt[0] if nxt else len(self.full)
        return min(first, self.hi) - self.lo

    def segment_copy(self, piece, off, length, dst):
        ctypes.memmove(dst, self.shard[off:off + length], length)

    def segment_set(self, piece, skip, tail_ptr, tail_len):
        self.skip = skip
        self.tail = ctypes.string_at(tail_ptr, tail_len) if tail_len else b""

    def segment(self):
        return self.shard[self.skip:] + self.tail

    # merge: a "table" is a dict key -> count, exported as key-hash partitions
    def set_counts(self, table, counts):
        self.counts[table] = counts

    def export_partitions(self, table, nparts):
        parts = [[] for _ in range(nparts)]
        for k, c in self.counts[table].items():
            parts[int(hashlib.md5(k).hexdigest(), 16) % nparts].append(
                len(k).to_bytes(4, "little") + c.to_bytes(8, "little") + k)
        blobs = [b"".join(p) for p in parts]
        self.exported = b"".join(blobs)
        return [len(b) for b in blobs]

    def export_copy(self, dst):
        ctypes.memmove(dst, self.exported, len(self.exported))

    def export_ranked(self, table, limit):
        r = self.ranked(table, 0, limit or None)
        self.exported = b"".join(len(k).to_bytes(4, "little") + c.to_bytes(8, "little") + k for k, c in r)
        return len(self.exported)

    def import_partitions(self, table, src, offs):
        # like msa_import_partitions: the table becomes the union of the blocks
        raw = ctypes.string_at(src, offs[-1]) if offs[-1] else b""
        m = self.merged[table] = {}
        i = 0
        while i < len(raw):
            kl = int.from_bytes(raw[i:i + 4], "little")
            c = int.from_bytes(raw[i + 4:i + 12], "little")
            k = raw[i + 12:i + 12 + kl]
            m[k] = m.get(k, 0) + c
            i += 12 + kl

    def rank(self):
        pass

    def import_ranked(self, table, src, offs):
        # like msa_import_ranked: the table becomes the merge of the ranked blocks
        self.import_partitions(table, src, offs)

    def ranked(self, table, first=0, count=None):
        r = sorted(self.merged[table].items(), key=lambda kv: (-kv[1], kv[0]))
        return r[first:first + count] if count else r[first:]


def _count(keys):
    out = {}
    for k in keys:
        out[k] = out.get(k, 0) + 1
    return out


def _worker(rank, world, port, data, cuts, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = mdist.Comm()
        ctx = FakeCtx(data, cuts[rank], cuts[rank + 1])
        mdist.resolve_piece(ctx, comm, mdist.PIECE_CSV)
        seg = ctx.segment()
        # count "records" of this rank's segment and merge them by key
        recs = [seg[a:b] for a, b in zip(record_starts(seg), record_starts(seg)[1:] + [len(seg)])] if seg else []
        ctx.set_counts(0, _count(recs))
        ctx.set_counts(1, _count(r.split(b",")[0] for r in recs))  # a second table: first fields
        mdist.merge_tables(ctx, comm, (0, 1))  # both tables in one exchange
        top = {t: ctx.ranked(t, 0, 3) for t in (0, 1)}  # this rank's partitions
        root = mdist.gather_ranked(ctx, comm, tables=(0, 1))
        ranked = [ctx.ranked(t) for t in (0, 1)] if root else None
        tot = comm.all_reduce_sum([len(recs)])
        # top-k gather: each rank sends its top 3, the root ranks the union
        ctx.merged = {t: dict(top[t]) for t in (0, 1)}
        mdist.gather_ranked(ctx, comm, topk=3, tables=(0, 1))
        top3 = [ctx.ranked(t, 0, 3) for t in (0, 1)] if root else None
        q.put((rank, seg, ranked, tot, top3))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("cuts_kind", ["mid_quote", "boundary", "tiny"])
def test_gloo_world_resolves_and_merges(cuts_kind):
    rec = b'A,s,l,"one two\nthree"\r\nB,s,l,four\n"q,1",s,l,"x\r\ny"\nC,s,l,z\n'
    data = b"artist,song,link,text\n" + rec * 5
    n = len(data)
    if cuts_kind == "mid_quote":
        cuts = [0, data.index(b"two") + 1, data.rindex(b"x\r") + 2, n]
    elif cuts_kind == "boundary":
        cuts = [0, data.index(b"B,s"), n]
    else:
        cuts = [0, 3, 4, n]
    world = len(cuts) - 1
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_worker, args=(r, world, port, data, cuts, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, seg, ranked, tot, top3 = q.get(timeout=60)
        res[r] = (seg, ranked, tot, top3)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every record exactly once, in order, across the ranks' segments
    assert b"".join(res[r][0] for r in range(world)) == data
    whole = [data[a:b] for a, b in zip(record_starts(data), record_starts(data)[1:] + [n])]
    assert res[0][2] == [len(whole)]
    for t, keys in enumerate((whole, [r.split(b",")[0] for r in whole])):
        full = sorted(_count(keys).items(), key=lambda kv: (-kv[1], kv[0]))
        assert res[0][1][t] == full
        assert res[0][3][t] == full[:3]
    assert all(res[r][1] is None for r in range(1, world))
