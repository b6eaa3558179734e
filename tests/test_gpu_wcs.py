"""GPU parity of the per-song word counter (msa_wcs_*, csrc/msa_wcs.hip).

* golden: byte-identical word_counts_by_song.csv / word_counts_global.csv and
  row count against outputs of the REAL reference script
  (tests/golden/wcs/, made by tests/golden/make_wcs_golden.py); inputs the
  script fails on must be refused.
* oracle: oracle/wcs_oracle.py (checker only) on fresh seeded torture corpora
  and Zipfian corpora, incl. a forced tiny word table (growth path).
* full-size properties on a 200k-song corpus: the by-song counts of every
  word sum to its global count, global counts sum to the token total,
  ranking order (count desc) holds.
"""
import os
import random
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, "golden"))
import wcs_oracle  # noqa: E402
from conftest import golden_delimiter  # noqa: E402
from test_wcs_oracle import CASES, GOLD, case_encoding, load_case  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wcs(msa_mod):
    w = msa_mod.WordCountPerSong(0)
    yield w
    w.close()


@pytest.mark.parametrize("name", CASES)
def test_wcs_golden(msa_mod, wcs, name):
    data, exp = load_case(name)
    wcs.set_delimiter(golden_delimiter(os.path.join(GOLD, name)))
    wcs.set_encoding(case_encoding(name))
    try:
        if exp is None:
            with pytest.raises(msa_mod.MsaError):
                wcs.run(data)
            return
        assert wcs.run(data) == exp
    finally:
        wcs.set_delimiter(",")
        wcs.set_encoding("utf-8-sig")


def _torture(seed, n):
    from make_wcs_golden import torture

    return torture(seed, n).encode("utf-8")


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6, 7, 8])
def test_wcs_torture_vs_oracle(wcs, seed):
    data = _torture(1000 + seed, 400)
    assert wcs.run(data) == wcs_oracle.word_count_per_song(data)


@pytest.mark.parametrize("seed,crlf", [(11, False), (12, True)])
def test_wcs_zipf_vs_oracle(msa_mod, wcs, seed, crlf):
    data = msa_mod.gen_corpus(1500, mode="zipf", seed=seed, crlf=crlf, vocab=3000)
    assert wcs.run(data) == wcs_oracle.word_count_per_song(data)


def _fuzz_text(seed, n=600):
    """Lyrics mixing ASCII, the two-byte Latin-1 letters (upper / lower case, ß,
    the excluded × and ÷), other UTF-8 (é in NFD, ’, emoji), apostrophes and
    escaped quotes at every offset of the 16-byte blocks the tokenizer walks."""
    import random
    rng = random.Random(seed)
    bits = ["a", "Zz", "'", "don't", "ÀÉÎ", "àéî", "ß", "Þþ", "×", "÷", "e\u0301", "’", "😀", "ÿ", "1", "Ü",
            " ", "  ", ",", ".", '"', "x" * 15, "ÉÉÉÉÉÉÉÉ", "ö'", "\t"]
    rows = ["artist,song,link,text"]
    for i in range(n):
        text = "".join(rng.choice(bits) for _ in range(rng.randint(0, 40)))
        rows.append(f'A{i % 7},S{i},/l/{i},"' + text.replace('"', '""') + '"')
    return ("\n".join(rows) + "\n").encode("utf-8")


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_wcs_fuzz_tokens_vs_oracle(wcs, seed):
    data = _fuzz_text(seed)
    assert wcs.run(data) == wcs_oracle.word_count_per_song(data)


def test_wcs_table_growth(msa_mod):
    """A 2^4-slot word table overflows; the run grows it and repeats."""
    data = msa_mod.gen_corpus(800, mode="highcard", seed=21, vocab=20000)
    exp = wcs_oracle.word_count_per_song(data)
    with msa_mod.WordCountPerSong(0) as w:
        w.set_table_bits(4)
        assert w.run(data) == exp


def test_wcs_edge_inputs(msa_mod, wcs):
    hdr = b"artist,song,link,text\n"
    cases = [
        hdr + b'A,S,/l,"' + b"x" * 5000 + b'"\n',                     # one long token
        hdr + b'A,S,/l,"ab""cd""ef ghi"\n',                             # escaped quotes split tokens
        hdr + b'A,S,/l,"abc"def ghi\n',                                  # token across a closing quote
        hdr + b"A,S,/l,\xc3\x80\xc3\x81\xc3\x82 \xc3\x97\xc3\x97\xc3\x97\n",  # latin-1 letters, x sign
        b"\xef\xbb\xbf" + hdr + b"A,S,/l,words here\r\n\r\nB,T,/l,more words\r",  # BOM, CR, blank line
        hdr + b'A,S,/l,"unterminated words\nsecond line',               # EOF inside quotes
        hdr + (b"A,S,/l,alpha beta gamma\n" * 3000),                    # many rows, one word set
    ]
    for d in cases:
        assert wcs.run(d) == wcs_oracle.word_count_per_song(d), d[:80]
    for bad in (hdr + b"A,S,/l,ab\xffcd\n", hdr + b"A,S,/l,ab\x00cd\n", hdr + b"A,S\n",
                hdr + b'A,S,/l,"' + b"y" * 131073 + b'"\n', b"", b"x,y\n1,2\n"):
        with pytest.raises(msa_mod.MsaError):
            wcs.run(bad)


def test_wcs_full_size_properties(msa_mod, wcs):
    data = msa_mod.gen_corpus(200000, mode="zipf", seed=31, vocab=50000)
    rows, by_song, glob = wcs.run(data)
    s = wcs.summary()
    assert rows == 200000 == s["total_rows"]
    g = {}
    prev = None
    for line in glob.split(b"\r\n")[1:-1]:
        w, c = line.rsplit(b",", 1)
        c = int(c)
        assert prev is None or c <= prev
        prev = c
        g[w] = c
    assert len(g) == s["n_words"]
    assert sum(g.values()) == s["total_tokens"]
    acc = {}
    nlines = 0
    for line in by_song.split(b"\r\n")[1:-1]:
        w, c = line.rsplit(b",", 2)[1:]
        acc[w] = acc.get(w, 0) + int(c)
        nlines += 1
    assert nlines == s["n_pairs"]
    assert acc == g
    # a random sample of songs against the oracle, row by row
    lines = data.split(b"\n")
    rnd = random.Random(5)
    hdr = lines[0] + b"\n"
    for _ in range(3):
        k = rnd.randrange(1, len(lines) - 400)
        sample = hdr + b"\n".join(lines[k:k + 300]) + b"\n"  # may start/end inside a quoted lyric
        try:
            exp = wcs_oracle.word_count_per_song(sample)
        except wcs_oracle.WcsError:  # a cut lyric leaves a short row: both refuse
            with pytest.raises(msa_mod.MsaError):
                wcs.run(sample)
            continue
        assert wcs.run(sample) == exp


@pytest.mark.parametrize("name", [c for c in CASES if c in ("basic", "crlf_cr_blank", "zipf_300", "err_missing_col",
                                                          "err_short_row", "torture_2") or c.startswith("sniff_")
                                  or c.startswith("utf8")])
def test_wcs_cli_golden(msa_mod, name, tmp_path):
    """bin/word_count_per_song writes the script's two files and prints its row
    count -- invoked like the golden run: with its --delimiter, or without one
    (the CLI's own csv.Sniffer restatement then picks it, as the script did),
    and its --encoding (utf-8 keeps a BOM in the first header name)."""
    cli = os.path.join(msa_mod.PKG_DIR, "bin", "word_count_per_song")
    data, exp = load_case(name)
    args = open(os.path.join(GOLD, name, "args.txt")).read().split()
    inp = tmp_path / "in.csv"
    inp.write_bytes(data)
    out = tmp_path / "out"
    r = subprocess.run([cli, str(inp), "--output-dir", str(out)] + args, capture_output=True, timeout=120)
    if exp is None:
        assert r.returncode != 0
        return
    assert r.returncode == 0, r.stderr
    assert f"Processadas {exp[0]} linhas".encode() in r.stdout
    assert (out / "word_counts_by_song.csv").read_bytes() == exp[1]
    assert (out / "word_counts_global.csv").read_bytes() == exp[2]


@pytest.mark.parametrize("outdir", ["out/", "./out", "out//sub/", "./out/./sub", "."])
def test_wcs_cli_prints_paths_like_pathlib(msa_mod, outdir, tmp_path):
    """The script prints os.fspath(Path(output_dir)) (word_count_per_song.py:148-155)."""
    from pathlib import Path

    cli = os.path.join(msa_mod.PKG_DIR, "bin", "word_count_per_song")
    data, exp = load_case("basic")
    inp = tmp_path / "in.csv"
    inp.write_bytes(data)
    r = subprocess.run([cli, str(inp), "--output-dir", outdir, "--delimiter", ","], capture_output=True, timeout=120,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    od = Path(outdir)
    want = (f"Concluído. Processadas {exp[0]} linhas. Arquivos gerados em {os.fspath(od)}\n"
            f" - {os.fspath(od / 'word_counts_global.csv')}\n - {os.fspath(od / 'word_counts_by_song.csv')}\n")
    assert r.stdout.decode() == want


# ---- k_wcs_wrows (wave per window of whole rows) at its boundaries: every
# input runs twice, once with the default path and once with every row on the
# thread-per-row walk (MSA_WCS_ABLATE=8); both must equal the oracle, and the
# summary says how many rows the window walk left to the per-row walk.
def _window_edges(seed):
    """Rows sized around the window's 1 KiB span (row ends at offsets 1008..1040
    of a 16-byte aligned start, rows over 1 KiB), windows of 32 tiny rows,
    windows with more than 192 token runs, the text as the FIRST column, and a
    last row with no newline ending in an empty text field."""
    rng = random.Random(seed)
    text_first = seed % 2 == 1
    rows = ["text,artist,song,link" if text_first else "artist,song,link,text"]

    def row(i, text):
        t = '"' + text.replace('"', '""') + '"' if rng.random() < 0.5 or "\n" in text or "," in text else text
        return f"{t},A{i % 5},S{i},/l/{i}" if text_first else f"A{i % 5},S{i},/l/{i},{t}"

    i = 0
    for _ in range(60):
        kind = rng.randrange(5)
        if kind == 0:      # one row whose end sweeps the window's last bytes
            n = rng.randrange(1000, 1045)
            words = []
            while sum(len(w) + 1 for w in words) < n:
                words.append(rng.choice(["alpha", "be", "gamma", "don't", "x", "zeta", "ÀÉÎ", "night"]))
            rows.append(row(i, " ".join(words)[:n]))
        elif kind == 1:    # a run of tiny rows (windows of WR_M = 32 rows)
            for _ in range(rng.randrange(30, 70)):
                rows.append(row(i, rng.choice(["ok", "yes yes", "", "la la la", "hey"])))
                i += 1
        elif kind == 2:    # > 192 token runs in one window
            rows.append(row(i, " ".join(rng.choice("abcdefgh") for _ in range(rng.randrange(300, 700)))))
        elif kind == 3:    # a row over 1 KiB
            rows.append(row(i, ("long words keep going " * rng.randrange(50, 120)).strip()))
        else:              # padding rows of random length shift the alignment
            rows.append(row(i, "pad " * rng.randrange(1, 40) + "end"))
        i += 1
    body = "\n".join(rows) + "\n"
    # the last row: no newline, its text field empty (ends with the delimiter)
    body += "Z,S9,/l/9," if not text_first else ",Z,S9,/l/9"
    return body.encode("utf-8")


def _run_both(msa_mod, wcs, data, monkeypatch):
    monkeypatch.delenv("MSA_WCS_ABLATE", raising=False)
    got = wcs.run(data)
    fb = wcs.summary()["fallback_rows"]
    monkeypatch.setenv("MSA_WCS_ABLATE", "8")
    try:
        walked = wcs.run(data)
        assert wcs.summary()["fallback_rows"] > 0  # every row on the per-row walk
    finally:
        monkeypatch.delenv("MSA_WCS_ABLATE", raising=False)
    return got, walked, fb


@pytest.mark.parametrize("seed", range(1, 9))
def test_wcs_window_edges_both_paths(msa_mod, wcs, seed, monkeypatch):
    data = _window_edges(seed)
    exp = wcs_oracle.word_count_per_song(data)
    got, walked, fb = _run_both(msa_mod, wcs, data, monkeypatch)
    assert walked == exp
    assert got == exp
    assert fb > 0  # rows over 1 KiB / windows over WR_TCAP token runs took the per-row walk


def test_wcs_window_walk_takes_every_plain_row(msa_mod, wcs, monkeypatch):
    """Plain Zipf input: the window walk settles every row itself."""
    data = msa_mod.gen_corpus(3000, mode="zipf", seed=77, vocab=4000)
    got, walked, fb = _run_both(msa_mod, wcs, data, monkeypatch)
    assert got == walked == wcs_oracle.word_count_per_song(data)
    assert fb == 0


@pytest.mark.parametrize("shift", range(0, 48, 3))
def test_wcs_row_end_sweeps_window_end(msa_mod, wcs, shift, monkeypatch):
    """A first row of 1000 + shift bytes ends at every offset around byte 1023
    of its window; the short rows after it follow at every alignment."""
    hdr = "artist,song,link,text\n"
    first = "A,S0,/l/0," + ("word " * 400)[: 1000 + shift - len("A,S0,/l/0,") - 1] + "\n"
    rest = "".join(f"A,S{i},/l/{i},tiny row {i} words\n" for i in range(1, 40))
    data = (hdr + first + rest).encode()
    got, walked, _ = _run_both(msa_mod, wcs, data, monkeypatch)
    assert got == walked == wcs_oracle.word_count_per_song(data)
