"""CPU: the C restatement of csv.Sniffer (music-analyst-ai_amd/host/msa_sniff.c,
used by bin/word_count_per_song when --delimiter is omitted) against the
stdlib's csv.Sniffer -- the very code the reference scripts call
(word_count_per_song.py:42-49, split_csv_columns.py:48-66) -- on the same
65536-character samples: CSV-like data with every preferred delimiter and
others, quoted / unquoted / multi-line fields, ", " spacing, non-ASCII text
and delimiters, junk, and samples where sniffing fails."""
import csv
import os
import random
import subprocess

import pytest

from conftest import PKG

BIN = os.path.join(PKG, "bin", "msa_sniff_test")


@pytest.fixture(scope="module")
def sniff_bin():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", PKG, "bin/msa_sniff_test"], check=True, capture_output=True, timeout=120)
    return BIN


def py_sniff(path):
    """What the scripts compute: fh.read(65536) under utf-8-sig, csv.Sniffer().sniff."""
    with open(path, encoding="utf-8-sig", newline="") as fh:
        try:
            sample = fh.read(65536)
        except UnicodeDecodeError:
            return "decode-error"
    try:
        d = csv.Sniffer().sniff(sample)
    except csv.Error:
        return "0 0 0"
    return f"1 {ord(d.delimiter)} {int(bool(d.skipinitialspace))}"


WORDS = ["the", "love", "Hello", "naïve", "Ærø", "x", "1999", "don't", "a b", "q\"q", "中文", "αβγ", "", "  "]


def rand_field(rnd, delim):
    w = " ".join(rnd.choice(WORDS) for _ in range(rnd.randint(0, 4)))
    style = rnd.random()
    if style < 0.35:
        return '"' + w.replace('"', '""') + ("\n" + w if rnd.random() < 0.2 else "") + '"'
    if style < 0.45:
        return "'" + w.replace("'", "") + "'"
    return w.replace(delim, " ").replace("\n", " ").replace('"', "")


def rand_csv(rnd, n_rows):
    delim = rnd.choice([",", ",", ";", "\t", "|", " ", ":", "#", "×", "-"])
    sp = " " if rnd.random() < 0.2 else ""
    ncol = rnd.randint(1, 6)
    eol = rnd.choice(["\n", "\r\n", "\n", "\r"])
    rows = []
    for _ in range(n_rows):
        k = ncol if rnd.random() < 0.9 else rnd.randint(1, ncol + 2)
        rows.append((delim + sp).join(rand_field(rnd, delim) for _ in range(k)))
    return eol.join(rows) + (eol if rnd.random() < 0.7 else "")


def junk(rnd, n):
    alpha = ["a", "b", " ", ",", ";", "\t", '"', "'", "\n", "\r", "é", "中", "_", "-", ".", ":", "|", "0"]
    return "".join(rnd.choice(alpha) for _ in range(n))


def cases():
    rnd = random.Random(20261016)
    out = []
    for i in range(160):
        out.append(rand_csv(rnd, rnd.choice([1, 2, 3, 5, 12, 40, 200])))
    for i in range(60):
        out.append(junk(rnd, rnd.choice([0, 1, 5, 30, 300, 3000])))
    out += ["", "\n\n", "a", '"x"', "'y'\n'z'", "a,b\n", "a;b;c\nd;e;f\n", "a, b, c\nd, e, f\n", '"a","b"\n"c","d"',
            "x\ty\n1\t2\n", "one two three\nfour five six\n", ",,,\n,,,\n", '"only, one"\n', "a:b\nc:d\ne:f:g\n"]
    # > 65536 characters: only the first 65536 are the sample
    big = rand_csv(random.Random(5), 4000)
    out.append(big)
    out.append("﻿" + "artist,song,link,text\n" + big)
    return out


def test_sniffer_matches_stdlib(sniff_bin, tmp_path):
    paths, want = [], []
    for i, text in enumerate(cases()):
        p = tmp_path / f"s{i}.csv"
        p.write_bytes(text.encode("utf-8"))
        paths.append(str(p))
        want.append(py_sniff(str(p)))
    bad = tmp_path / "bad.csv"
    bad.write_bytes(b"a,b\n\xff\xfe,c\n")
    paths.append(str(bad))
    want.append(py_sniff(str(bad)))
    got = subprocess.run([sniff_bin] + paths, capture_output=True, text=True, timeout=120).stdout.split("\n")
    mism = [(os.path.basename(p), w, g) for p, w, g in zip(paths, want, got) if w != g]
    assert not mism, mism[:10]
    # the generator must exercise both sniffing paths and the failure
    kinds = {w.split()[0] for w in want}
    assert {"0", "1"} <= kinds
    assert len({w for w in want if w.startswith("1")}) >= 6


def test_sniffer_on_the_corpora(sniff_bin, tmp_path, msa_mod=None):
    """The synthetic lyric corpora sniff as ',' (the reference's own data shape)."""
    import sys
    sys.path.insert(0, PKG)
    import msa

    for mode in ("zipf", "highcard", "torture"):
        data = msa.gen_corpus(400, mode=mode, seed=3)
        p = tmp_path / f"{mode}.csv"
        p.write_bytes(data)
        got = subprocess.run([sniff_bin, str(p)], capture_output=True, text=True, timeout=60).stdout.strip()
        assert got == py_sniff(str(p)), mode
