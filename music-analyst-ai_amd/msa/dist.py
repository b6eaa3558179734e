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

    def alltoallv(self, send: torch.Tensor, send_counts: List[int]) -> Tuple[torch.Tensor, List[int]]:
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
    fns = comm.all_gather_bytes(ctx.shard_function(piece))
    sizes = [row[0] for row in comm.all_gather_u64([size])]
    head = ctx.shard_head(piece, fns[:comm.rank], sizes[:comm.rank]) if comm.rank > 0 else 0
    heads = [row[0] for row in comm.all_gather_u64([head])]
    send_counts, _ = tail_plan(comm.rank, heads, sizes)
    send = torch.empty(max(1, head), dtype=torch.uint8, device=comm.device)
    if sum(send_counts):
        ctx.segment_copy(piece, 0, head, send.data_ptr())
    recv, recv_counts = comm.alltoallv(send, send_counts)
    tail = sum(recv_counts)
    ctx.segment_set(piece, head, recv.data_ptr() if tail else 0, tail)
    return tail


def merge_table(ctx, comm: Comm, table: int):
    parts = ctx.export_partitions(table, comm.world)
    send = torch.empty(max(1, sum(parts)), dtype=torch.uint8, device=comm.device)
    ctx.export_copy(send.data_ptr())
    recv, recv_counts = comm.alltoallv(send, parts)
    offs = [0]
    for c in recv_counts:
        offs.append(offs[-1] + c)
    ctx.import_partitions(table, recv.data_ptr(), offs)


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
    merge_table(ctx, comm, MSA_TABLE_WORDS)
    merge_table(ctx, comm, MSA_TABLE_ARTISTS)
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
    got = []
    for t in tables:
        nbytes = ctx.export_ranked(t, topk or 0)
        send = torch.empty(max(1, nbytes), dtype=torch.uint8, device=comm.device)
        ctx.export_copy(send.data_ptr())
        counts = [0] * comm.world
        counts[0] = nbytes
        recv, recv_counts = comm.alltoallv(send, counts)
        got.append((t, recv, recv_counts))
    if comm.rank != 0:
        return False
    for t, recv, recv_counts in got:
        offs = [0]
        for c in recv_counts:
            offs.append(offs[-1] + c)
        ctx.import_ranked(t, recv.data_ptr(), offs)
    return True
