"""Multi-GPU driver: one process per GPU, torch.distributed for the exchanges
(backend "nccl" = RCCL over xGMI with device tensors; "gloo" with host tensors
for CPU rehearsal and for several ranks sharing one GPU in tests).

It replaces the reference's MPI data flow (/root/reference/src/parallel_spotify.c):

* main 866-916 splits the column files at raw byte offsets and lets every rank
  re-synchronise with a fresh reader, so records at the cut points are lost or
  counted twice (tests/test_oracle.py::test_reference_is_np_dependent).  Here
  each rank computes the reader-state transfer function of its shard
  (msa_shard_function), the functions are all-gathered, and every rank knows
  the exact state at its first byte.  The bytes of a record that began on an
  earlier rank (its "head") move to the rank where the record begins, so every
  record is processed exactly once -- results are those of the single-process
  reference for any number of GPUs.  The same is done for the artist.csv
  pieces, whose reader can also carry quote state across pieces.
* main 1011-1025 + send/receive_hash_table (397-432) stream every key of every
  rank to rank 0 as three MPI messages each.  Here each rank exports its
  tables as key-hash partitions, one all-to-all moves partition p to rank p,
  and every rank merges and ranks its own key range; rank 0 then gathers the
  ranked partitions (or their top-k).

The routing logic (`head_owners`, `tail_plan`) is plain Python
so it is tested on CPU with a gloo world (tests/test_dist.py).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import MSA_TABLE_ARTISTS, MSA_TABLE_WORDS, PIECE_ARTISTS, PIECE_CSV, SHARD_FN_BYTES


# ------------------------------------------------------------------ routing
def head_owners(heads: Sequence[int], sizes: Sequence[int]) -> List[int]:
    """owner[r] = the rank where the record containing rank r's first byte
    begins: the nearest earlier rank that holds a record start (head < size).
    -1 for rank 0 and for ranks whose head is empty."""
    owners = []
    last_start = -1
    for r, (h, n) in enumerate(zip(heads, sizes)):
        owners.append(last_start if (r > 0 and h > 0) else -1)
        if r == 0 or h < n:
            last_start = r
    return owners


def tail_plan(rank: int, heads: Sequence[int], sizes: Sequence[int]) -> Tuple[List[int], List[int]]:
    """(send_counts, recv_counts) in bytes for the head exchange of `rank`."""
    world = len(sizes)
    owners = head_owners(heads, sizes)
    send = [0] * world
    recv = [0] * world
    if owners[rank] >= 0:
        send[owners[rank]] = heads[rank]
    for r in range(world):
        if owners[r] == rank:
            recv[r] = heads[r]
    return send, recv


# ----------------------------------------------------------------- exchange
class Comm:
    """Thin byte-exchange layer over torch.distributed."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else \
            torch.device("cpu")

    def all_gather_u64(self, values: Sequence[int]) -> List[List[int]]:
        t = torch.tensor(list(values), dtype=torch.int64, device=self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [o.tolist() for o in out]

    def all_gather_bytes(self, b: bytes) -> List[bytes]:
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [bytes(o.cpu().numpy().tobytes()) for o in out]

    def alltoallv(self, send: torch.Tensor, send_counts: List[int],
                  recv_counts: Optional[List[int]] = None) -> Tuple[torch.Tensor, List[int]]:
        """One all-to-all-v; recv_counts when every rank already knows them
        (else one all-gather of the send counts first)."""
        if recv_counts is None:
            recv_counts = [row[self.rank] for row in self.all_gather_u64(send_counts)]
        recv = torch.empty(max(1, sum(recv_counts)), dtype=torch.uint8, device=self.device)
        if self.world == 1:
            recv[: sum(recv_counts)].copy_(send[: sum(send_counts)])
        else:
            dist.all_to_all_single(recv[: sum(recv_counts)] if sum(recv_counts) else recv[:0],
                                   send[: sum(send_counts)] if sum(send_counts) else send[:0],
                                   output_split_sizes=recv_counts, input_split_sizes=send_counts, group=self.group)
        self.sync()
        return recv, recv_counts

    def sync(self):
        # the library reads received bytes on its own HIP stream
        if self.device.type == "cuda":
            torch.cuda.current_stream().synchronize()

    def all_reduce_sum(self, values: Sequence[int]) -> List[int]:
        t = torch.tensor(list(values), dtype=torch.int64, device=self.device)
        dist.all_reduce(t, group=self.group)
        return t.tolist()


# ------------------------------------------------------------------ driver
def resolve_piece(ctx, comm: Comm, piece: int) -> int:
    """Make this rank's piece start at a record boundary and end with the
    records that began here: returns the number of bytes appended."""
    size = ctx.piece_size(piece)
    # the functions and the sizes in one all-gather
    got = comm.all_gather_bytes(ctx.shard_function(piece) + size.to_bytes(8, "little"))
    fns = [g[:-8] for g in got]
    sizes = [int.from_bytes(g[-8:], "little") for g in got]
    head = ctx.shard_head(piece, fns[:comm.rank], sizes[:comm.rank]) if comm.rank > 0 else 0
    heads = [row[0] for row in comm.all_gather_u64([head])]
    send_counts, recv_plan = tail_plan(comm.rank, heads, sizes)
    send = torch.empty(max(1, head), dtype=torch.uint8, device=comm.device)
    if sum(send_counts):
        ctx.segment_copy(piece, 0, head, send.data_ptr())
    recv, recv_counts = comm.alltoallv(send, send_counts, recv_plan)
    tail = sum(recv_counts)
    ctx.segment_set(piece, head, recv.data_ptr() if tail else 0, tail)
    return tail


def _prefix(v: Sequence[int]) -> List[int]:
    out = [0]
    for x in v:
        out.append(out[-1] + x)
    return out


def _split_tables(comm: Comm, recv: torch.Tensor, mine: List[List[int]]) -> List[Tuple[torch.Tensor, List[int]]]:
    """recv holds, per source rank, its blocks of every table in table order
    (mine[src][t] bytes each): per table, the sources' blocks made contiguous
    and their offsets."""
    src_off = _prefix([sum(m) for m in mine])
    out = []
    for t in range(len(mine[0]) if mine else 0):
        segs, offs = [], [0]
        for src, m in enumerate(mine):
            start, n = src_off[src] + sum(m[:t]), m[t]
            if n:
                segs.append(recv[start:start + n])
            offs.append(offs[-1] + n)
        buf = torch.cat(segs) if len(segs) > 1 else (segs[0] if segs else recv[:1])
        out.append((buf, offs))
    comm.sync()  # the library reads these buffers on its own stream
    return out


def merge_tables(ctx, comm: Comm, tables: Sequence[int] = (MSA_TABLE_WORDS, MSA_TABLE_ARTISTS)):
    """The key-hash partitioned merge of several tables in ONE all-gather (the
    partition sizes) + ONE all-to-all (every table's partition p to rank p)."""
    W, me, T = comm.world, comm.rank, len(tables)
    bufs, parts = [], []
    for t in tables:
        pt = ctx.export_partitions(t, W)
        b = torch.empty(max(1, sum(pt)), dtype=torch.uint8, device=comm.device)
        ctx.export_copy(b.data_ptr())  # the export buffer is per context: copy before the next table's
        bufs.append(b)
        parts.append(pt)
    offs = [_prefix(pt) for pt in parts]
    pieces, send_counts = [], []
    for p in range(W):
        for ti in range(T):
            if parts[ti][p]:
                pieces.append(bufs[ti][offs[ti][p]:offs[ti][p + 1]])
        send_counts.append(sum(parts[ti][p] for ti in range(T)))
    send = torch.cat(pieces) if len(pieces) > 1 else (pieces[0] if pieces else bufs[0])
    sizes = comm.all_gather_u64([parts[ti][p] for ti in range(T) for p in range(W)])
    mine = [[sizes[src][ti * W + me] for ti in range(T)] for src in range(W)]
    recv, _ = comm.alltoallv(send, send_counts, [sum(m) for m in mine])
    for t, (buf, o) in zip(tables, _split_tables(comm, recv, mine)):
        ctx.import_partitions(t, buf.data_ptr(), o)


def merge_table(ctx, comm: Comm, table: int):
    merge_tables(ctx, comm, (table,))


def run_sharded(ctx, comm: Comm, text_column: bool = True) -> Tuple[int, int]:
    """The whole hot path for this rank's shard (already loaded with
    msa_load_csv).  Returns the global (total_songs, total_words); every rank
    ends holding the ranked tables of its own key partition."""
    ctx.set_shard(comm.rank == 0)
    resolve_piece(ctx, comm, PIECE_CSV)
    ctx.split_columns(text_column)
    # artist.csv lines are its records on every rank unless some rank's split
    # says otherwise; then every rank runs the exact reader on resolved pieces
    if comm.all_reduce_sum([int(ctx.artist_reader_needed())])[0]:
        ctx.set_artist_reader(True)
        resolve_piece(ctx, comm, PIECE_ARTISTS)
    else:
        ctx.set_artist_reader(False)
    ctx.count()
    s = ctx.summary()
    merge_tables(ctx, comm, (MSA_TABLE_WORDS, MSA_TABLE_ARTISTS))
    ctx.rank()
    songs, words = comm.all_reduce_sum([s.total_songs, s.total_words])
    return songs, words


def gather_ranked(ctx, comm: Comm, topk: Optional[int] = None,
                  tables: Sequence[int] = (MSA_TABLE_WORDS, MSA_TABLE_ARTISTS)) -> bool:
    """Device-side final gather: every rank serialises its ranked partition
    (or its top-k) with msa_export_ranked, one all-to-all moves the blocks to
    rank 0 (RCCL: GPU to GPU), and rank 0 merges them (msa_import_ranked: a
    k-way merge of the ranked blocks) -- the key partitions are disjoint, so
    that is the global ranking (its top-k when each rank sent its own top-k).  Returns True on rank 0, whose context
    then holds the global ranked tables (ctx.ranked / msa_write_table_csv).
    Replaces rank 0's receive + merge of every rank's table
    (parallel_spotify.c:1011-1025) and the final qsort (325-344)."""
    bufs, nbs = [], []
    for t in tables:  # every table's block in one all-gather (sizes) + one all-to-all
        nb = ctx.export_ranked(t, topk or 0)
        b = torch.empty(max(1, nb), dtype=torch.uint8, device=comm.device)
        ctx.export_copy(b.data_ptr())
        bufs.append(b[:nb])
        nbs.append(nb)
    pieces = [b for b in bufs if b.numel()]
    send = torch.cat(pieces) if len(pieces) > 1 else (pieces[0] if pieces else torch.empty(
        1, dtype=torch.uint8, device=comm.device))
    sizes = comm.all_gather_u64(nbs)
    counts = [0] * comm.world
    counts[0] = sum(nbs)
    mine = [list(row) for row in sizes] if comm.rank == 0 else [[0] * len(tables) for _ in range(comm.world)]
    recv, _ = comm.alltoallv(send, counts, [sum(m) for m in mine])
    if comm.rank != 0:
        return False
    for t, (buf, o) in zip(tables, _split_tables(comm, recv, mine)):
        ctx.import_ranked(t, buf.data_ptr(), o)
    return True
