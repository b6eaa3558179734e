"""GPU: the configurations the bench claims, and table growth on every entry point.

* configs[2] at full size (5M Zipfian songs, ~1.19 GB resident in HBM, the
  corpus bench.py times) against the oracle, byte for byte;
* a high-cardinality corpus sized so that EVERY initial table overflows
  (> 512K distinct 3..8-byte words, > 131K 9..16-byte words, > 32K distinct
  long words and > 64K long-word occurrences, > 32K artists), through
  msa_run, through the separate msa_split_columns / msa_count / msa_rank entry
  points, and through the drop-in CLI.  The reference grows its tables
  (ht_resize, /root/reference/src/parallel_spotify.c:101-132) and never fails
  on cardinality; neither may libmsa_hip.
The 2-rank sharded world on the same corpus is in test_gpu_dist.py."""
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG, files_equal, read_outputs, run_oracle, run_with_heartbeat
from test_gpu_parity import check_against_oracle

pytestmark = pytest.mark.gpu
CLI = os.path.join(PKG, "bin", "parallel_spotify")

# cardinalities of this corpus (measured with the oracle): S 1.18M, M 683K,
# long 226K distinct words, 79K artists -- every initial capacity exceeded
HIGHCARD_SONGS = 150_000
HIGHCARD_SEED = 31


@pytest.fixture(scope="module")
def ctx(msa_mod):
    c = msa_mod.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def highcard(msa_mod, tmp_path_factory):
    data = msa_mod.gen_corpus(HIGHCARD_SONGS, mode="highcard", seed=HIGHCARD_SEED)
    d = tmp_path_factory.mktemp("hc")
    p = d / "hc.csv"
    p.write_bytes(data)
    r = run_oracle(str(p), str(d / "o"), ranks=1)
    assert r.returncode == 0, r.stderr
    return data, str(p), read_outputs(str(d / "o"))


def test_highcard_overflows_every_table_run(msa_mod, highcard):
    data, _, exp = highcard
    with msa_mod.Context(0) as c:  # fresh context: initial (small) capacities
        c.load_csv(data)
        c.run(text_column=True)
        s = c.summary()
        assert s.n_words > 2_000_000 and s.n_artists > 32_768
        assert msa_mod.table_csv_bytes(c.ranked(msa_mod.MSA_TABLE_WORDS), "word") == exp["word_counts.csv"]
        assert msa_mod.table_csv_bytes(c.ranked(msa_mod.MSA_TABLE_ARTISTS), "artist") == exp["top_artists.csv"]
        assert (s.total_songs, s.total_words) == (exp["metrics"]["total_songs"], exp["metrics"]["total_words"])


def test_highcard_overflows_every_table_stages(msa_mod, highcard):
    """msa_split_columns + msa_count + msa_rank (the CLI's and the sharded
    driver's call sequence) recover from overflow on their own."""
    data, _, exp = highcard
    with msa_mod.Context(0) as c:
        c.load_csv(data)
        c.split_columns(True)
        c.count()
        c.rank()
        s = c.summary()
        assert msa_mod.table_csv_bytes(c.ranked(msa_mod.MSA_TABLE_WORDS), "word") == exp["word_counts.csv"]
        assert msa_mod.table_csv_bytes(c.ranked(msa_mod.MSA_TABLE_ARTISTS), "artist") == exp["top_artists.csv"]
        assert s.total_words == exp["metrics"]["total_words"]
        for k, v in exp["split"].items():
            which = 0 if k == s.artist_file + ".csv" else 1
            assert c.split_column(which) == v, k


def test_highcard_cli(highcard, tmp_path):
    _, path, exp = highcard
    out = tmp_path / "out"
    p = subprocess.run([CLI, path, "--output-dir", str(out)], capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["word_counts.csv"] == exp["word_counts.csv"]
    assert got["top_artists.csv"] == exp["top_artists.csv"]
    assert got["split"] == exp["split"]
    assert got["metrics"]["total_words"] == exp["metrics"]["total_words"]


def test_tables_shrink_back_to_small_corpus(msa_mod, highcard, tmp_path):
    """A context whose tables grew keeps working on the next (small) input."""
    data, _, _ = highcard
    with msa_mod.Context(0) as c:
        c.load_csv(data)
        c.run(text_column=False)
        small = msa_mod.gen_corpus(2000, mode="torture", seed=9)
        check_against_oracle(msa_mod, c, small, tmp_path, "after_grow")


@pytest.mark.timeout(600)
def test_configs2_full_size(msa_mod, ctx, tmp_path):
    """BASELINE configs[2] exactly as bench.py builds it (5M songs, ~1.19 GB)."""
    data = msa_mod.gen_corpus(5_000_000, mode="zipf", seed=1, vocab=50000, n_artists=5000, words_per_song=30)
    assert len(data) > 1_000_000_000
    check_against_oracle(msa_mod, ctx, data, tmp_path, "configs2")


def check_files_against_oracle(msa_mod, c, od, tmp_path):
    """The context's ranked tables (written by msa_write_table_csv), split
    columns and totals against the oracle's output directory, byte for byte."""
    s = c.summary()
    words, artists = str(tmp_path / "w.csv"), str(tmp_path / "a.csv")
    c.write_table_csv(msa_mod.MSA_TABLE_WORDS, words, "word")
    c.write_table_csv(msa_mod.MSA_TABLE_ARTISTS, artists, "artist")
    assert files_equal(words, os.path.join(od, "word_counts.csv")), "word_counts.csv differs"
    assert files_equal(artists, os.path.join(od, "top_artists.csv")), "top_artists.csv differs"
    for which, name in ((0, s.artist_file), (1, s.text_file)):
        with open(os.path.join(od, "split_columns", name + ".csv"), "rb") as f:
            assert c.split_column(which) == f.read(), f"split column {name}.csv differs"
    m = read_metrics(od)
    assert (s.total_songs, s.total_words) == (m["total_songs"], m["total_words"])
    return s


def read_metrics(od):
    import json

    with open(os.path.join(od, "performance_metrics.json")) as f:
        return json.load(f)


@pytest.mark.timeout(900)
def test_corpus_over_4gib(msa_mod, configs3_corpus, tmp_path):
    """A 20M-song corpus (~4.7 GB > 2^32 bytes; configs[3]'s corpus family) on
    one GPU against the oracle: no 32-bit byte offset anywhere in the pipeline
    (at N = 2 the configs[3] shards are ~12 GB per GPU)."""
    path, od = configs3_corpus
    with open(path, "rb") as f:
        data = f.read()
    with msa_mod.Context(0) as c:
        c.load_csv(data)
        del data
        c.run(text_column=True)
        check_files_against_oracle(msa_mod, c, od, tmp_path)


# BASELINE configs[4]: the adversarial high-cardinality corpus at full scale.
# highcard seed 4 at 4.1M songs holds > 50M distinct words and > 1.7M artists
# (skewed); every table grows several times (the reference's ht_resize,
# parallel_spotify.c:101-132), the miss logs overflow into direct inserts, the
# ranking runs the radix sort with 16-byte-prefix tie refinement.
C4_SONGS = 4_100_000


@pytest.fixture(scope="module")
def configs4(msa_mod, tmp_path_factory):
    d = tmp_path_factory.mktemp("c4")
    path = str(d / "c4.csv")
    data = msa_mod.gen_corpus(C4_SONGS, mode="highcard", seed=4)
    with open(path, "wb") as f:
        f.write(data)
    od = str(d / "o")
    r = run_oracle(path, od, ranks=1, timeout=600)
    assert r.returncode == 0, r.stderr
    return data, path, od


@pytest.mark.timeout(900)
def test_configs4_run(msa_mod, configs4, tmp_path):
    data, _, od = configs4
    with msa_mod.Context(0) as c:  # fresh context: every table starts small
        c.load_csv(data)
        c.run(text_column=True)
        s = check_files_against_oracle(msa_mod, c, od, tmp_path)
        assert s.n_words >= 50_000_000 and s.n_artists > 1_000_000
        # the cold run (a one-shot CLI run): the first split of a large input
        # takes the dense entries, so no table grows round by round (round 5:
        # three split attempts, 6.6 s)
        import ctypes
        c.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
        v = ctypes.c_uint64(0)
        assert c.lib.msa_debug_stat(c.h, b"split_attempts", ctypes.byref(v)) == 0
        assert v.value <= 2, f"{v.value} split attempts on a cold configs[4] run"


@pytest.mark.timeout(900)
def test_configs4_cli(configs4, tmp_path):
    """The drop-in CLI on the same corpus: word_counts.csv, top_artists.csv and
    both split-column files identical to the oracle's."""
    _, path, od = configs4
    out = tmp_path / "out"
    p = run_with_heartbeat([CLI, path, "--output-dir", str(out)], 600, "parallel_spotify configs[4]")
    assert p.returncode == 0, p.stderr
    for f in ("word_counts.csv", "top_artists.csv"):
        assert files_equal(str(out / f), os.path.join(od, f)), f
    names = sorted(os.listdir(os.path.join(od, "split_columns")))
    assert sorted(os.listdir(out / "split_columns")) == names
    for n in names:
        assert files_equal(str(out / "split_columns" / n), os.path.join(od, "split_columns", n)), n
    m, e = read_metrics(str(out)), read_metrics(od)
    assert (m["total_songs"], m["total_words"]) == (e["total_songs"], e["total_words"])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("transport,procs", [("rccl", 1), ("shm", 2)])
def test_configs4_cli_ranks(configs4, tmp_path, transport, procs):
    """configs[4] through the rank layer: a world of one over the RCCL
    transport (MSA_RANK_PATH=1) -- its ~1.8 GB key-partition block for itself
    is a device copy, not an RCCL message (sent through ncclSend / ncclRecv to
    itself it had arrived corrupt) -- and two ranks sharing the GPU (shm): the
    merged word and artist rankings equal the oracle's."""
    _, path, od = configs4
    out = tmp_path / "out"
    env = dict(os.environ, MSA_TRANSPORT=transport)
    cmd = [CLI, path, "--output-dir", str(out)]
    if procs > 1:
        cmd += ["--processes", str(procs)]
    else:
        env["MSA_RANK_PATH"] = "1"
    p = run_with_heartbeat(cmd, 600, f"parallel_spotify configs[4] {transport} x{procs}", env=env)
    assert p.returncode == 0, p.stderr
    for f in ("word_counts.csv", "top_artists.csv"):
        assert files_equal(str(out / f), os.path.join(od, f)), f


@pytest.mark.parametrize("sort", ["radix", "merge"])
def test_sort_designs_agree(msa_mod, tmp_path, sort, monkeypatch):
    """Both ranking sorts, forced on every table size (MSA_SORT): the radix
    sort on the small torture tables (ties, empty and 16-byte-prefix-sharing
    keys) and the merge sort on the high-cardinality tables."""
    monkeypatch.setenv("MSA_SORT", sort)
    data = msa_mod.gen_corpus(1500, mode="torture", seed=5) if sort == "radix" else None
    with msa_mod.Context(0) as c:
        if sort == "radix":
            check_against_oracle(msa_mod, c, data, tmp_path, "sort_radix_torture")
            small = msa_mod.gen_corpus(3000, mode="highcard", seed=8, vocab=20000)
            check_against_oracle(msa_mod, c, small, tmp_path, "sort_radix_hc")
            for case in ("shared_prefix_ties", "long_words", "quotes_everywhere"):  # 16-byte-prefix tie runs
                raw = open(os.path.join(GOLDEN, case, "input.csv"), "rb").read()
                check_against_oracle(msa_mod, c, raw, tmp_path, f"sort_radix_{case}")
        else:
            big = msa_mod.gen_corpus(HIGHCARD_SONGS, mode="highcard", seed=HIGHCARD_SEED)
            check_against_oracle(msa_mod, c, big, tmp_path, "sort_merge_hc")
