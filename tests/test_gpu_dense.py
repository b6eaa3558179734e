"""GPU: dense word entries (k_mb_agg<true>, msa_k3.hip).  With high
cardinality the bucketed aggregation of the token pass's miss logs writes each
distinct 3..16-byte word's ranking entry itself -- no HBM word-table inserts,
slot lists, table clears or k_word_entries pass over them.  Forced here with
MSA_DENSE_MIN=0 (every split of a context dense); the outputs must equal the
oracle's byte for byte (process_lyrics + the hash table,
/root/reference/src/parallel_spotify.c:350-394, ranked by entry_compare_desc
161-188).  Also: the retries that leave the dense path (a multi-line text
label, overflowing logs), the automatic switch, and the shard guard."""
import ctypes

import pytest

from test_gpu_parity import EDGE, check_against_oracle

pytestmark = pytest.mark.gpu


def stat(c, name):
    c.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
    v = ctypes.c_uint64(0)
    assert c.lib.msa_debug_stat(c.h, name.encode(), ctypes.byref(v)) == 0
    return v.value


@pytest.fixture
def dense_ctx(msa_mod, monkeypatch):
    monkeypatch.setenv("MSA_DENSE_MIN", "0")
    c = msa_mod.Context(0)  # the library reads the settings when the context is made
    yield c
    c.close()


@pytest.mark.parametrize("case", ["highcard", "zipf", "torture", "highcard_medium"])
def test_dense_forced(msa_mod, dense_ctx, tmp_path, case):
    if case == "highcard":
        data = msa_mod.gen_corpus(150_000, mode="highcard", seed=31)
    elif case == "highcard_medium":
        data = msa_mod.gen_corpus(400_000, mode="highcard", seed=5)
    elif case == "zipf":
        data = msa_mod.gen_corpus(60_000, mode="zipf", seed=12)
    else:
        data = msa_mod.gen_corpus(1500, mode="torture", seed=3)
    check_against_oracle(msa_mod, dense_ctx, data, tmp_path, f"dn_{case}")
    assert stat(dense_ctx, "dense") == 1
    assert stat(dense_ctx, "dense_n") == stat(dense_ctx, "s_claimed") + stat(dense_ctx, "m_claimed")
    # again on the same context: the planes, logs and buckets are reused
    check_against_oracle(msa_mod, dense_ctx, data, tmp_path, f"dn_{case}_again")
    assert stat(dense_ctx, "dense") == 1


@pytest.mark.parametrize("name", sorted(EDGE))
def test_dense_edge_cases(msa_mod, dense_ctx, tmp_path, name):
    """Every edge case dense; a multi-line text label (its remainder's words
    would go into the tables) runs again through the tables."""
    check_against_oracle(msa_mod, dense_ctx, EDGE[name], tmp_path, f"dn_{name}")
    if name == "multiline_text_header":
        assert stat(dense_ctx, "dense") == 0
        assert stat(dense_ctx, "split_attempts") >= 2


def test_dense_then_tables_then_dense(msa_mod, dense_ctx, tmp_path):
    """Dense and table splits alternate on one context: a dense split leaves
    the word tables empty, a table split's claimed slots are cleared by the
    next split's prologue; a new input clears the previous input's veto."""
    a = msa_mod.gen_corpus(30_000, mode="highcard", seed=8)
    check_against_oracle(msa_mod, dense_ctx, a, tmp_path, "alt0")
    assert stat(dense_ctx, "dense") == 1
    check_against_oracle(msa_mod, dense_ctx, EDGE["multiline_text_header"], tmp_path, "alt1")  # vetoes dense
    assert stat(dense_ctx, "dense") == 0
    assert stat(dense_ctx, "s_table_used") == stat(dense_ctx, "s_claimed")
    check_against_oracle(msa_mod, dense_ctx, a, tmp_path, "alt2")
    assert stat(dense_ctx, "dense") == 1  # the veto held for the input that raised it


def test_dense_small_logs(msa_mod, tmp_path, monkeypatch):
    """Miss logs far too small: the dense split's overflowing partitions send
    it round again with grown logs (a flush that found its partition full
    went into the tables) -- same bytes, and the next run is dense at once."""
    monkeypatch.setenv("MSA_DENSE_MIN", "0")
    monkeypatch.setenv("MSA_MLOG_ENTRIES", "4096")
    c = msa_mod.Context(0)
    try:
        data = msa_mod.gen_corpus(20_000, mode="highcard", seed=31)
        check_against_oracle(msa_mod, c, data, tmp_path, "dn_mlog")
        first = stat(c, "split_attempts")
        assert first >= 2
        check_against_oracle(msa_mod, c, data, tmp_path, "dn_mlog2")
        assert stat(c, "split_attempts") == first + 1
        assert stat(c, "dense") == 1
    finally:
        c.close()


def test_dense_auto_switch(msa_mod, tmp_path, monkeypatch):
    """The automatic choice: a split whose previous run counted at least
    MSA_DENSE_MIN distinct S + M words is dense."""
    monkeypatch.setenv("MSA_DENSE_MIN", "1000")
    data = msa_mod.gen_corpus(40_000, mode="highcard", seed=9)
    with msa_mod.Context(0) as c:
        got = []
        for k in range(3):
            check_against_oracle(msa_mod, c, data, tmp_path, f"dn_auto{k}")
            got.append(stat(c, "dense"))
        # (the first run's first attempt counts through the tables; when its logs
        # overflow, the attempt after it already knows the cardinality)
        assert got[1:] == [1, 1]


def test_dense_off(msa_mod, tmp_path, monkeypatch):
    monkeypatch.setenv("MSA_DENSE_MIN", "0")
    monkeypatch.setenv("MSA_DENSE", "0")
    data = msa_mod.gen_corpus(20_000, mode="highcard", seed=2)
    with msa_mod.Context(0) as c:
        check_against_oracle(msa_mod, c, data, tmp_path, "dn_off")
        assert stat(c, "dense") == 0


def test_dense_shard_exports_partitions(msa_mod, dense_ctx, tmp_path):
    """A shard's dense word entries are exported as key-hash partitions from
    their planes (round 5 turned dense off for shards): a world of one --
    export, import, rank -- gives the oracle's bytes; after msa_rank the planes
    are reordered, so a dense export is refused there."""
    data = msa_mod.gen_corpus(20_000, mode="highcard", seed=4)
    dense_ctx.set_shard(True)
    p = tmp_path / "sh.csv"
    p.write_bytes(data)
    from conftest import read_outputs, run_oracle
    r = run_oracle(str(p), str(tmp_path / "o"), ranks=1)
    assert r.returncode == 0
    exp = read_outputs(str(tmp_path / "o"))
    dense_ctx.load_csv(data)
    dense_ctx.split_columns(text_column=False)
    dense_ctx.count()
    assert stat(dense_ctx, "dense") == 1
    for table in (msa_mod.MSA_TABLE_WORDS, msa_mod.MSA_TABLE_ARTISTS):
        sizes = dense_ctx.export_partitions(table, 1)
        buf = ctypes.create_string_buffer(max(1, sizes[0]))
        dense_ctx.export_copy(ctypes.addressof(buf))
        dense_ctx.import_partitions(table, ctypes.addressof(buf), [0, sizes[0]])
    dense_ctx.rank()
    assert msa_mod.table_csv_bytes(dense_ctx.ranked(msa_mod.MSA_TABLE_WORDS), "word") == exp["word_counts.csv"]
    assert msa_mod.table_csv_bytes(dense_ctx.ranked(msa_mod.MSA_TABLE_ARTISTS), "artist") == exp["top_artists.csv"]
    # a fresh dense split ranked without a merge: its planes are the ranking's now
    check_against_oracle(msa_mod, dense_ctx, data, tmp_path, "dn_shard2")
    assert stat(dense_ctx, "dense") == 1
    with pytest.raises(Exception):
        dense_ctx.export_partitions(msa_mod.MSA_TABLE_WORDS, 2)
