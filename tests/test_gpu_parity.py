"""GPU parity: libmsa_hip (gfx950 kernels, called through the C ABI) against the
CPU oracle on the same inputs -- byte-identical word_counts.csv, top_artists.csv,
split column files and totals (reference semantics of `mpirun -np 1`,
/root/reference/src/parallel_spotify.c)."""
import os
import random

import pytest

from conftest import read_outputs, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(msa_mod):
    c = msa_mod.Context(0)
    yield c
    c.close()


def gpu_outputs(msa, ctx, data):
    ctx.load_csv(data)
    ctx.run(text_column=True)
    s = ctx.summary()
    out = {
        "word_counts.csv": msa.table_csv_bytes(ctx.ranked(msa.MSA_TABLE_WORDS), "word"),
        "top_artists.csv": msa.table_csv_bytes(ctx.ranked(msa.MSA_TABLE_ARTISTS), "artist"),
        "split": {s.artist_file + ".csv": ctx.split_column(0), s.text_file + ".csv": ctx.split_column(1)},
        "metrics": {"processes": 1, "total_songs": s.total_songs, "total_words": s.total_words},
    }
    return out


def check_against_oracle(msa, ctx, data, tmp_path, name):
    p = tmp_path / f"{name}.csv"
    p.write_bytes(data)
    od = tmp_path / f"orc_{name}"
    r = run_oracle(str(p), str(od), ranks=1)
    assert r.returncode == 0, r.stderr
    exp = read_outputs(str(od))
    got = gpu_outputs(msa, ctx, data)
    assert got["metrics"] == exp["metrics"]
    assert sorted(got["split"]) == sorted(exp["split"])
    for k in exp["split"]:
        assert got["split"][k] == exp["split"][k], f"split column {k} differs"
    for k in ("word_counts.csv", "top_artists.csv"):
        if got[k] != exp[k]:
            gl, el = got[k].split(b"\n"), exp[k].split(b"\n")
            first = next((i for i, (a, b) in enumerate(zip(gl, el)) if a != b), min(len(gl), len(el)))
            pytest.fail(f"{k} differs at line {first}: gpu={gl[first:first + 3]} oracle={el[first:first + 3]} "
                        f"(lines {len(gl)} vs {len(el)})")


@pytest.mark.parametrize("seed", list(range(1, 13)))
def test_torture(msa_mod, ctx, tmp_path, seed):
    data = msa_mod.gen_corpus(1500, mode="torture", seed=seed)
    check_against_oracle(msa_mod, ctx, data, tmp_path, f"torture{seed}")


@pytest.mark.parametrize("seed", [2, 5])
def test_torture_repeat_runs(msa_mod, ctx, tmp_path, seed):
    """Repeated runs on one loaded input (what bench.py times: later splits size
    their tables, logs and the dense choice from the earlier ones) give the
    oracle's bytes every time, on corpora whose records take the exact path."""
    msa = msa_mod
    data = msa.gen_corpus(1500, mode="torture", seed=seed)
    p = tmp_path / "t.csv"
    p.write_bytes(data)
    r = run_oracle(str(p), str(tmp_path / "orc"), ranks=1)
    assert r.returncode == 0, r.stderr
    exp = read_outputs(str(tmp_path / "orc"))
    ctx.load_csv(data)
    for _ in range(3):
        ctx.run(text_column=True)
        s = ctx.summary()
        assert msa.table_csv_bytes(ctx.ranked(msa.MSA_TABLE_WORDS), "word") == exp["word_counts.csv"]
        assert msa.table_csv_bytes(ctx.ranked(msa.MSA_TABLE_ARTISTS), "artist") == exp["top_artists.csv"]
        got = {s.artist_file + ".csv": ctx.split_column(0), s.text_file + ".csv": ctx.split_column(1)}
        assert got == exp["split"]


@pytest.mark.parametrize("mode,songs,crlf", [("zipf", 3000, False), ("zipf", 2000, True), ("highcard", 3000, False)])
def test_small_corpora(msa_mod, ctx, tmp_path, mode, songs, crlf):
    data = msa_mod.gen_corpus(songs, mode=mode, seed=7, vocab=20000, n_artists=500, crlf=crlf)
    check_against_oracle(msa_mod, ctx, data, tmp_path, f"{mode}{songs}{int(crlf)}")


@pytest.mark.parametrize("mode", ["zipf", "highcard"])
def test_medium_corpora(msa_mod, ctx, tmp_path, mode):
    """~40-60 MB: many chunks, many waves, real hash-table pressure."""
    data = msa_mod.gen_corpus(200_000, mode=mode, seed=21)
    check_against_oracle(msa_mod, ctx, data, tmp_path, f"{mode}_medium")


@pytest.mark.parametrize("mode", ["zipf", "highcard"])
def test_miss_logs_overflow_and_grow(msa_mod, tmp_path, monkeypatch, mode):
    """K3's miss logs sized far too small (MSA_MLOG_ENTRIES): the token pass
    drops what does not fit and flags OVF_MLOG, the split runs again with logs
    sized from what it counted -- same bytes as the oracle, and a second run on
    the same context needs no retry."""
    import ctypes
    monkeypatch.setenv("MSA_MLOG_ENTRIES", "4096")
    c = msa_mod.Context(0)
    try:
        data = msa_mod.gen_corpus(20_000, mode=mode, seed=31)
        c.lib.msa_debug_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]

        def stat(name):
            v = ctypes.c_uint64(0)
            assert c.lib.msa_debug_stat(c.h, name.encode(), ctypes.byref(v)) == 0
            return v.value

        check_against_oracle(msa_mod, c, data, tmp_path, f"mlog_{mode}")
        first = stat("split_attempts")
        assert first >= 2, "the tiny logs should have overflowed once"
        check_against_oracle(msa_mod, c, data, tmp_path, f"mlog2_{mode}")
        assert stat("split_attempts") == first + 1, "grown logs: one attempt"
    finally:
        c.close()


EDGE = {
    "header_only": b"artist,song,link,text\n",
    "header_no_newline": b"artist,song,link,text",
    "no_trailing_newline": b"artist,song,link,text\nA,s,l,\"hello world again\"",
    "cr_only": b"artist,song,link,text\rA,s,l,one two three\rB,s,l,\"four five\rsix\"\r",
    "short_records": b"a,b,c,d\nonly,two\n\n,,,\nX,y,z,alpha beta\n",
    "nul_bytes": b"a,b,c,d\nA\x00B,s,l,zero one\nC,s,l,two\x00three four\nD,s\x00,l,five six\n",
    "long_words": b"a,b,c,d\nA,s,l,\"" + b"x" * 17 + b" " + b"Y" * 300 + b" supercalifragilistic supercalifragilistic\"\n",
    "shared_prefix_ties": b"a,b,c,d\n" + b"".join(
        b"A,s,l,abcdefghijklmnop%s\n" % s for s in [b"zz", b"z", b"zzz", b"a", b"b", b"abc", b"z\x27"]),
    "multiline_text_header": b"a,b,c,\"multi\nline, header\"\nA,s,l,words here\n",
    "multiline_artist_header": b"\"art\nist, name\",b,c,d\nA,s,l,words here\nB,s,l,more\n",
    "quotes_everywhere": b"a,b,c,d\n\"A \"\"x\"\"\",s,l,\"say \"\"hi\"\" now\"\nB\"q,s,l,open quote\n\"z\n",
    "apostrophes": b"a,b,c,d\nA,s,l,''' '' 'tis rock'n'roll don't O'NEIL\n",
    "whitespace_fields": b"a,b,c,d\n  A  ,s,l,   \t  \n\t,s,l, x y z \n",
    "utf8": "a,b,c,d\nBeyoncé,s,l,café naïve über straße\n".encode(),
}


@pytest.mark.parametrize("name", sorted(EDGE))
def test_edge_cases(msa_mod, ctx, tmp_path, name):
    check_against_oracle(msa_mod, ctx, EDGE[name], tmp_path, name)


def fuzz_fields(seed, n=4000):
    """Records whose artist / lyric fields stress the column-span paths: quoted
    names with "" pairs, padding spaces and tabs inside and outside the quotes,
    names past 32 and 48 bytes, unquoted and space-padded lyrics, lyrics that
    end right after a quote, records with fewer than four fields."""
    rng = random.Random(seed)
    bits = ["a", "Bo", "x y", '"', '""', " ", "  ", "\t", "Zed", "q", "0", "'", "é"]
    out = ["artist,song,link,text\n"]
    for i in range(n):
        name = "".join(rng.choice(bits) for _ in range(rng.choice([0, 1, 2, 4, 8, 14, 22])))
        r = rng.random()
        if r < 0.6:
            art = " " * rng.randint(0, 2) + '"' + name.replace('"', '""') + '"' + " " * rng.randint(0, 2)
        elif r < 0.95:
            art = name.replace('"', "").replace(",", "")
        else:
            art = name  # unquoted with quotes: the exact artist reader
        words = " ".join(rng.choice(["love", "You", "don't", "la", "xx", "a", "Go!", "quoted\"s"])
                         for _ in range(rng.randint(0, 9)))
        t = rng.random()
        if t < 0.5:
            text = '"' + words.replace('"', '""') + '"'
        elif t < 0.7:
            text = " " * rng.randint(1, 3) + '"' + words.replace('"', '""') + '"' + " " * rng.randint(1, 3)
        elif t < 0.85:
            text = words.replace('"', "").replace(",", " ")
        elif t < 0.95:
            text = '"' + words.replace('"', '""') + '\n' + words.replace('"', "") + '"'
        else:
            text = '""'
        if rng.random() < 0.03:
            out.append(f"{art},s{i}\n")  # too few fields
        else:
            out.append(f"{art},s{i},/l/{i},{text}" + rng.choice(["\n", "\r\n", "\n"]))
    return "".join(out).encode()


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fuzz_fields(msa_mod, ctx, tmp_path, seed):
    check_against_oracle(msa_mod, ctx, fuzz_fields(seed), tmp_path, f"fuzz{seed}")


def test_fuzz_fields_quote_free_artists(msa_mod, ctx, tmp_path):
    """The same without unquoted quote-bearing names: the artist lines shortcut
    stays on, so the in-register quoted-key path decides the artist table."""
    data = b"\n".join(l for l in fuzz_fields(9).split(b"\n") if not (l[:1] != b'"' and b'"' in l.split(b",")[0]))
    check_against_oracle(msa_mod, ctx, data, tmp_path, "fuzz_qf")


def test_text_column_stage_orders(msa_mod, ctx, tmp_path):
    """text.csv is written on a side stream (launched with the artist pass or
    the ranking, or by the entry point that first needs it): every order of
    the stage calls -- and a new input before the old pass finished -- still
    gives the oracle's columns and tables."""
    a = msa_mod.gen_corpus(3000, mode="zipf", seed=41)
    b = msa_mod.gen_corpus(2500, mode="torture", seed=42)
    exp = {}
    for name, data in (("a", a), ("b", b)):
        path = tmp_path / f"{name}.csv"
        path.write_bytes(data)
        r = run_oracle(str(path), str(tmp_path / f"o_{name}"), ranks=1)
        assert r.returncode == 0, r.stderr
        exp[name] = read_outputs(str(tmp_path / f"o_{name}"))

    def check_split(name):
        s = ctx.summary()
        assert ctx.split_column(0) == exp[name]["split"][s.artist_file + ".csv"]
        assert ctx.split_column(1) == exp[name]["split"][s.text_file + ".csv"]

    def check_tables(name):
        assert msa_mod.table_csv_bytes(ctx.ranked(msa_mod.MSA_TABLE_WORDS), "word") == exp[name]["word_counts.csv"]
        assert msa_mod.table_csv_bytes(ctx.ranked(msa_mod.MSA_TABLE_ARTISTS), "artist") == exp[name]["top_artists.csv"]

    ctx.load_csv(a)
    ctx.split_columns(text_column=True)
    check_split("a")                        # split only: the entry point launches it
    ctx.load_csv(b)
    ctx.split_columns(text_column=True)
    ctx.count()                             # launched beside the artist pass
    check_split("b")
    ctx.rank()
    check_tables("b")
    ctx.count()                             # a second count changes nothing
    ctx.rank()
    check_tables("b")
    ctx.load_csv(a)
    ctx.run(text_column=True)               # joined at the end of the run
    ctx.load_csv(b)                         # a new input right after
    ctx.run(text_column=True)
    check_split("b")
    check_tables("b")


def test_empty_file_fails_loudly(msa_mod, ctx):
    ctx.load_csv(b"")
    with pytest.raises(msa_mod.MsaError) as e:
        ctx.run()
    assert e.value.code == -3  # MSA_ERR_NOHEADER


def test_bad_header_fails_loudly(msa_mod, ctx):
    ctx.load_csv(b"a,b\nA,s,l,x\n")
    with pytest.raises(msa_mod.MsaError) as e:
        ctx.run()
    assert e.value.code == -4  # MSA_ERR_BADHEADER


def test_failed_split_leaves_no_stale_slots(msa_mod, ctx, tmp_path):
    """A split that fails after its scan (bad header: the artist count and the
    word tables ran) must not leave claimed table slots behind for the next run."""
    ctx.load_csv(b"a,b\nSame,s,l,\"repeated words repeated words\"\nOther,s,l,\"more words here\"\n")
    with pytest.raises(msa_mod.MsaError):
        ctx.run()
    data = b"artist,song,link,text\nSame,s,l,\"repeated words again\"\nNew,s,l,\"fresh words\"\n"
    check_against_oracle(msa_mod, ctx, data, tmp_path, "after_failed_split")


# ---------------------------------------------------------------- golden vectors
from test_oracle import CASES as GOLDEN_CASES, golden  # noqa: E402


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_golden_reference_np1(msa_mod, ctx, case):
    """Byte-identical to the REAL reference (`mpirun -np 1`) on its own outputs."""
    from conftest import GOLDEN

    res, files = golden(case, 1)
    data = open(os.path.join(GOLDEN, case, "input.csv"), "rb").read()
    if res["returncode"] != 0:
        ctx.load_csv(data)
        with pytest.raises(msa_mod.MsaError) as e:
            ctx.run()
        assert e.value.code in (-3, -4)
        return
    got = gpu_outputs(msa_mod, ctx, data)
    assert got["metrics"] == {k: res[k] for k in ("processes", "total_songs", "total_words")}
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert got["split"] == files["split"]
