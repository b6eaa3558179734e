"""GPU: the multi-GPU path (msa/dist.py over libmsa_hip) with N processes on the
box's one GPU (gloo carries the exchanges through host memory; RCCL/xGMI on a
real multi-GPU node).  The logical CSV is cut at arbitrary byte offsets --
inside quoted multi-line lyrics, between '\\r' and '\\n', on record boundaries
-- and the merged, ranked result must be byte-identical to the single-process
reference semantics (the oracle at np=1)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import (PKG, REPO, files_equal, hash_file, read_outputs, run_oracle, run_with_heartbeat, say,
                      table_bytes, table_counts)

pytestmark = pytest.mark.gpu

WORKER = r'''
import json, os, sys
sys.path.insert(0, os.environ["MSA_PKG"])
import torch, torch.distributed as dist
import msa
from msa import dist as mdist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
cuts = json.loads(os.environ["MSA_CUTS"])
lo, hi = cuts[rank], cuts[rank + 1]
with open(os.environ["MSA_CSV"], "rb") as f:  # this rank's byte range only
    f.seek(lo)
    data = f.read(hi - lo)
ctx = msa.Context(0)
ctx.load_csv(data)
del data
comm = mdist.Comm()
songs, words = mdist.run_sharded(ctx, comm, text_column=False)
if os.environ.get("MSA_STAT_OUT"):  # which word path the split took (dense entries or tables)
    import ctypes
    ctx.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
    v = ctypes.c_uint64(0)
    ctx.lib.msa_debug_stat(ctx.h, b"dense", ctypes.byref(v))
    open(os.environ["MSA_STAT_OUT"] + f".{rank}", "w").write(str(v.value))
if mdist.gather_ranked(ctx, comm):
    w = ctx.ranked(msa.MSA_TABLE_WORDS)
    a = ctx.ranked(msa.MSA_TABLE_ARTISTS)
    out = os.environ["MSA_OUT"]
    open(out + ".words", "wb").write(msa.table_csv_bytes(w, "word"))
    open(out + ".artists", "wb").write(msa.table_csv_bytes(a, "artist"))
    json.dump({"total_songs": songs, "total_words": words}, open(out + ".json", "w"))
ctx.close()
dist.destroy_process_group()
'''


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_world(tmp_path, data, cuts, csv=None, timeout=240, env_extra=None):
    if csv is None:
        csv = tmp_path / "in.csv"
        csv.write_bytes(data)
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    out = str(tmp_path / "res")
    world = len(cuts) - 1
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   MSA_PKG=PKG, MSA_CSV=str(csv), MSA_CUTS=json.dumps(cuts), MSA_OUT=out, **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("distributed workers timed out")
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return (open(out + ".words", "rb").read(), open(out + ".artists", "rb").read(),
            json.load(open(out + ".json")))


def expected(tmp_path, data):
    p = tmp_path / "o.csv"
    p.write_bytes(data)
    r = run_oracle(str(p), str(tmp_path / "o"), ranks=1)
    assert r.returncode == 0
    return read_outputs(str(tmp_path / "o"))


def cuts_for(data, world, mode):
    n = len(data)
    if mode == "even":
        return [n * r // world for r in range(world)] + [n]
    if mode == "in_quotes":  # cut just after the opening quote of some lyric
        cs = [0]
        pos = 0
        for r in range(1, world):
            pos = data.index(b',"', n * r // world) + 2
            cs.append(pos)
        return cs + [n]
    if mode == "crlf":  # cut between '\r' and '\n'
        cs = [0]
        for r in range(1, world):
            cs.append(data.index(b"\r\n", n * r // world) + 1)
        return cs + [n]
    if mode == "record":  # exactly on record starts
        cs = [0]
        for r in range(1, world):
            cs.append(data.index(b'"\n', n * r // world) + 2)
        return cs + [n]
    raise ValueError(mode)


@pytest.mark.parametrize("world,mode,gen", [
    (2, "even", ("zipf", False)),
    (3, "in_quotes", ("zipf", False)),
    (2, "record", ("zipf", False)),
    (2, "crlf", ("zipf", True)),
    (4, "even", ("highcard", False)),
    (3, "even", ("torture", False)),
])
def test_sharded_equals_single_process(msa_mod, tmp_path, world, mode, gen):
    kind, crlf = gen
    data = msa_mod.gen_corpus(4000 if kind != "torture" else 3000, mode=kind, seed=17, crlf=crlf, vocab=8000)
    cuts = cuts_for(data, world, mode)
    words, artists, tot = run_world(tmp_path, data, cuts)
    exp = expected(tmp_path, data)
    assert tot == {k: exp["metrics"][k] for k in ("total_songs", "total_words")}
    assert words == exp["word_counts.csv"]
    assert artists == exp["top_artists.csv"]


@pytest.mark.parametrize("world,kind", [(5, "highcard"), (4, "torture")])
def test_sharded_gather_corank(msa_mod, tmp_path, world, kind):
    """msa_import_ranked's co-rank merge (k_mr_corank) with more blocks: many
    tiles per block, blocks of very different sizes, and (highcard) long keys
    sharing their first 16 bytes and a count across blocks (the tie path)."""
    data = msa_mod.gen_corpus(6000, mode=kind, seed=5, vocab=8000)
    cuts = cuts_for(data, world, "in_quotes")
    words, artists, tot = run_world(tmp_path, data, cuts)
    exp = expected(tmp_path, data)
    assert words == exp["word_counts.csv"]
    assert artists == exp["top_artists.csv"]


def test_sharded_tiny_shards(msa_mod, tmp_path):
    """More ranks than records in some shards: whole shards that are one
    record's middle, empty shards."""
    data = msa_mod.gen_corpus(40, mode="zipf", seed=3)
    n = len(data)
    cuts = [0, 10, 11, n // 2, n // 2 + 5, n]
    words, artists, tot = run_world(tmp_path, data, cuts)
    exp = expected(tmp_path, data)
    assert words == exp["word_counts.csv"]
    assert artists == exp["top_artists.csv"]
    assert tot["total_words"] == exp["metrics"]["total_words"]


@pytest.mark.timeout(300)
def test_sharded_highcard_every_table_overflows(msa_mod, tmp_path):
    """2 ranks on the corpus of test_gpu_scale.py whose cardinalities exceed
    every initial table: each rank's split/count and the merged partitions
    grow their tables and the result is still the single-process one.  The
    root's co-rank merge takes the whole union (no size limit, no re-rank:
    the round-3 count matrix fell back above 2^18 keys)."""
    data = msa_mod.gen_corpus(150_000, mode="highcard", seed=31)
    cuts = cuts_for(data, 2, "in_quotes")
    words, artists, tot = run_world(tmp_path, data, cuts)
    exp = expected(tmp_path, data)
    assert words.count(b"\n") > 4 * (1 << 18)
    assert tot == {k: exp["metrics"][k] for k in ("total_songs", "total_words")}
    assert words == exp["word_counts.csv"]
    assert artists == exp["top_artists.csv"]


# ---- BASELINE configs[3]'s shape: ONE logical multi-GB corpus (20M songs,
# ~4.7 GB, conftest.configs3_corpus) sharded over several ranks.  On this
# one-GPU box the ranks share the GPU; the exchanges go through host memory
# (gloo / the C host's shared-memory transport) instead of RCCL over xGMI --
# the data flow, boundaries and merge are the ones an 8-GPU node runs.
def file_cuts(path, world):
    """Cuts just after the opening quote of a lyric near every n*r/world."""
    n = os.path.getsize(path)
    cs = [0]
    with open(path, "rb") as f:
        for r in range(1, world):
            f.seek(n * r // world)
            w = f.read(1 << 16)
            cs.append(n * r // world + w.index(b',"') + 2)
    return cs + [n]


@pytest.mark.timeout(900)
def test_configs3_two_ranks_cut_in_quotes(msa_mod, configs3_corpus, tmp_path):
    """2 ranks (Python driver over torch.distributed) on the 4.7 GB corpus, the
    cut inside a quoted lyric: exact boundary exchange, key-hash all-to-all
    merge, device-side gather -- identical to the oracle at np = 1."""
    path, od = configs3_corpus
    words, artists, tot = run_world(tmp_path, None, file_cuts(path, 2), csv=path, timeout=600)
    exp = read_outputs_tables(od)
    assert tot == {k: exp["metrics"][k] for k in ("total_songs", "total_words")}
    assert words == exp["word_counts.csv"]
    assert artists == exp["top_artists.csv"]


def read_outputs_tables(od):
    with open(os.path.join(od, "performance_metrics.json")) as f:
        m = json.load(f)
    return {"word_counts.csv": open(os.path.join(od, "word_counts.csv"), "rb").read(),
            "top_artists.csv": open(os.path.join(od, "top_artists.csv"), "rb").read(),
            "metrics": {k: m[k] for k in ("total_songs", "total_words")}}


@pytest.mark.timeout(900)
def test_configs3_c_host_four_ranks_shm(configs3_corpus, tmp_path):
    """The drop-in C host with --processes 4 (MSA_TRANSPORT=shm: four ranks on
    the one GPU) on the 4.7 GB corpus: every output file identical to the
    oracle's at np = 1, performance_metrics.json reports 4 processes."""
    path, od = configs3_corpus
    cli = os.path.join(PKG, "bin", "parallel_spotify")
    out = tmp_path / "out"
    env = dict(os.environ, MSA_TRANSPORT="shm")
    p = run_with_heartbeat([cli, path, "--output-dir", str(out), "--processes", "4"], 800, "parallel_spotify -np 4",
                           env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    for f in ("word_counts.csv", "top_artists.csv"):
        assert files_equal(str(out / f), os.path.join(od, f)), f
    names = sorted(os.listdir(os.path.join(od, "split_columns")))
    assert sorted(os.listdir(out / "split_columns")) == names
    for n in names:
        assert files_equal(str(out / "split_columns" / n), os.path.join(od, "split_columns", n)), n
    with open(out / "performance_metrics.json") as f:
        m = json.load(f)
    e = read_outputs_tables(od)["metrics"]
    assert m["processes"] == 4 and (m["total_songs"], m["total_words"]) == (e["total_songs"], e["total_words"])


def test_rank_after_import_ranked_topk(msa_mod):
    """A table merged by msa_import_ranked (here one GPU's own top-k block) is
    ranked-only: a later msa_rank keeps the merged ranking (it must not rank
    the local count tables, which hold more keys than the merged arrays were
    sized for) and msa_export_partitions refuses it."""
    import ctypes
    msa = msa_mod
    data = msa.gen_corpus(3000, mode="zipf", seed=11)
    with msa.Context(0) as ctx:
        ctx.load_csv(data)
        ctx.run(text_column=False)
        full_w = ctx.ranked(msa.MSA_TABLE_WORDS)
        full_a = ctx.ranked(msa.MSA_TABLE_ARTISTS)
        k = 25
        assert len(full_w) > 10 * k
        for t, full in ((msa.MSA_TABLE_WORDS, full_w), (msa.MSA_TABLE_ARTISTS, full_a)):
            nb = ctx.export_ranked(t, k)
            buf = ctypes.create_string_buffer(nb)
            ctx.export_copy(ctypes.addressof(buf))
            ctx.import_ranked(t, ctypes.addressof(buf), [0, nb])
            assert ctx.ranked(t) == full[:k]
        ctx.rank()  # must leave both merged rankings as they are
        assert ctx.ranked(msa.MSA_TABLE_WORDS) == full_w[:k]
        assert ctx.ranked(msa.MSA_TABLE_ARTISTS) == full_a[:k]
        with pytest.raises(msa.MsaError):
            ctx.export_partitions(msa.MSA_TABLE_WORDS, 2)


# ---- BASELINE configs[3] at its stated size: the 100M-song corpus (~23.7 GB)
# through the C host as a 4-rank world on the one GPU (shm transport).  The
# generator's songs are independent draws, so the corpus is the concatenation
# of its song ranges and the np = 1 answer is the sum of the ranges' answers:
# the oracle runs on 5 ranges of 20M songs in parallel (each with the header
# line), their tables are summed and ranked by entry_compare_desc
# (parallel_spotify.c:176-188: count desc, then strcmp) and written as
# write_csv_entry does (307-319); the split files are the header line plus
# the ranges' bodies in order.  Everything lives in /dev/shm (host memory).
C3_FULL_SONGS = 100_000_000
C3_FULL_RANGES = 5


@pytest.mark.timeout(1500)
def test_configs3_full_size_c_host_four_ranks(msa_mod, tmp_path):
    """configs[3] at full size (100M songs, ~23.7 GB, one logical CSV):
    bin/parallel_spotify --processes 4 (four ranks on the one GPU, shm
    exchanges) -- word_counts.csv, top_artists.csv, both split files and the
    totals identical to the oracle's np = 1 answer."""
    import shutil
    import tempfile
    import xxhash

    base = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    d = tempfile.mkdtemp(dir=base, prefix="msa_c3full_")
    try:
        big = os.path.join(d, "c3full.csv")
        header = None
        procs = []
        with open(big, "wb") as f:
            for k in range(C3_FULL_RANGES):
                lo, hi = C3_FULL_SONGS * k // C3_FULL_RANGES, C3_FULL_SONGS * (k + 1) // C3_FULL_RANGES
                data = msa_mod.gen_corpus(C3_FULL_SONGS, mode="zipf", seed=1, vocab=50000, n_artists=5000,
                                          words_per_song=30, first_song=lo, count=hi - lo)
                f.write(data)
                if k == 0:
                    header = data[:data.index(b"\n") + 1]
                rp = os.path.join(d, f"r{k}.csv")
                with open(rp, "wb") as g:
                    if k:
                        g.write(header)
                    g.write(data)
                del data
                od = os.path.join(d, f"o{k}")
                procs.append((rp, od, subprocess.Popen([os.path.join(REPO, "oracle", "msa_oracle"), rp, "--output-dir", od],
                                                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)))
                say(f"  [configs3 full: range {k} generated, oracle started]")
        assert os.path.getsize(big) > 20 * (1 << 30)
        words, artists, songs, total_words = {}, {}, 0, 0
        hashes, hdrs, names = {}, {}, None
        for k, (rp, od, p) in enumerate(procs):
            while True:
                try:
                    _, err = p.communicate(timeout=30)
                    break
                except subprocess.TimeoutExpired:
                    say(f"  [configs3 full: oracle range {k} running]")
            assert p.returncode == 0, err[-2000:]
            for key, v in table_counts(os.path.join(od, "word_counts.csv")).items():
                words[key] = words.get(key, 0) + v
            for key, v in table_counts(os.path.join(od, "top_artists.csv")).items():
                artists[key] = artists.get(key, 0) + v
            with open(os.path.join(od, "performance_metrics.json")) as f:
                m = json.load(f)
            songs += m["total_songs"]
            total_words += m["total_words"]
            sd = os.path.join(od, "split_columns")
            names = sorted(os.listdir(sd))
            for n in names:
                if k == 0:
                    with open(os.path.join(sd, n), "rb") as f:
                        hdrs[n] = f.readline()
                    hashes[n] = xxhash.xxh3_128(hdrs[n])
                hash_file(os.path.join(sd, n), True, hashes[n])
            shutil.rmtree(od)
            os.remove(rp)
        out = os.path.join(d, "out")
        cli = os.path.join(PKG, "bin", "parallel_spotify")
        env = dict(os.environ, MSA_TRANSPORT="shm")
        p = run_with_heartbeat([cli, big, "--output-dir", out, "--processes", "4"], 900, "parallel_spotify -np 4 (23.7 GB)",
                               env=env)
        assert p.returncode == 0, p.stderr[-3000:]
        assert open(os.path.join(out, "word_counts.csv"), "rb").read() == table_bytes(b"word,count\n", words)
        assert open(os.path.join(out, "top_artists.csv"), "rb").read() == table_bytes(b"artist,count\n", artists)
        with open(os.path.join(out, "performance_metrics.json")) as f:
            m = json.load(f)
        assert (m["processes"], m["total_songs"], m["total_words"]) == (4, songs, total_words)
        sd = os.path.join(out, "split_columns")
        assert sorted(os.listdir(sd)) == names
        for n in names:
            h = xxhash.xxh3_128()
            hash_file(os.path.join(sd, n), False, h)
            assert h.digest() == hashes[n].digest(), n
    finally:
        shutil.rmtree(d, ignore_errors=True)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_dense_entries(msa_mod, tmp_path, world):
    """High cardinality on every shard with dense word entries forced
    (MSA_DENSE_MIN=0): each rank exports its dense entries' key partitions,
    imports its own partition into its tables and ranks it; rank 0's merged
    ranking is the oracle's (np=1) byte for byte.  The cuts fall inside quoted
    lyrics."""
    data = msa_mod.gen_corpus(60_000, mode="highcard", seed=23)
    cuts = cuts_for(data, world, "in_quotes")
    stat = str(tmp_path / "dense")
    w, a, m = run_world(tmp_path, data, cuts, env_extra={"MSA_DENSE_MIN": "0", "MSA_STAT_OUT": stat})
    exp = expected(tmp_path, data)
    assert m["total_songs"] == exp["metrics"]["total_songs"]
    assert m["total_words"] == exp["metrics"]["total_words"]
    assert w == exp["word_counts.csv"]
    assert a == exp["top_artists.csv"]
    assert [open(f"{stat}.{r}").read() for r in range(world)] == ["1"] * world
