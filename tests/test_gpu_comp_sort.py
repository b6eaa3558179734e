"""GPU: the words' composite radix-sort key (msa_sort.hip, msa_radix_sort_comp).

The large-table ranking sorts ONE 64-bit word per entry: the dense rank of the
entry's count among the table's distinct counts in its top 0, 1 or 2 bytes
(one distinct count, <= 256, more) and the key's first 8, 7 or 6 bytes below
it; entries equal in that word are ordered by the tie refinement from the
first uncovered key byte on.  The reference orders by count descending, then
by strcmp (entry_compare_desc, /root/reference/src/parallel_spotify.c:178-188).

Each case builds a table where one width occurs and long runs of keys share
both the covered prefix and a count -- short, 9..16-byte and long (> 16 byte)
keys mixed -- so the refinement orders every run.  MSA_SORT=radix forces the
radix path at these sizes (it starts at 2^18 keys otherwise); MSA_COMP_SORT=0
runs the K2/K1 sort the composite key replaced, on the same inputs."""
import random

import pytest

from test_gpu_parity import check_against_oracle

pytestmark = pytest.mark.gpu


def letters(i, n):
    """i as n base-26 letters (tokens are letters only: digits would split them)."""
    s = []
    for _ in range(n):
        s.append(chr(ord("a") + i % 26))
        i //= 26
    return "".join(reversed(s))


def corpus(words, seed):
    """(word, count) pairs -> a CSV whose lyrics hold each word `count` times."""
    toks = []
    for w, c in words:
        toks += [w] * c
    random.Random(seed).shuffle(toks)
    rows = ["artist,song,link,text\n"]
    for k, i in enumerate(range(0, len(toks), 40)):
        rows.append(f'band{k % 13},song{k},/a/{k}.html,"{" ".join(toks[i:i + 40])}"\n')
    return "".join(rows).encode()


def case_words(case):
    if case == "one_count":  # every count 1: gid bytes 0, all 8 key bytes in the word
        ws = [("prefixab" + letters(i, 3), 1) for i in range(3000)]  # one run of 3000 tied on 8 bytes
        ws += [("prefixabcdefghij" + letters(i, 3), 1) for i in range(1500)]  # long keys tied on 16 bytes
        ws += [(letters(i, 4), 1) for i in range(2000)]
        return ws
    if case == "byte_gid":  # 3 distinct counts: one gid byte, 7 key bytes
        ws = [("sharedq" + letters(i, 3), 1 + i % 3) for i in range(3000)]
        ws += [("sharedqrstuvwxyzab" + letters(i, 2), 1 + i % 3) for i in range(600)]
        ws += [(letters(i, 5), 1 + i % 3) for i in range(1500)]
        return ws
    # 300 distinct counts: two gid bytes, 6 key bytes
    ws = [("shared" + letters(i, 3), 1 + i % 300) for i in range(3000)]
    ws += [("sharedabcdefghijkl" + letters(i, 2), 1 + i % 300) for i in range(676)]
    ws += [("sh" + letters(i, 2), 1 + i % 7) for i in range(600)]
    return ws


@pytest.mark.parametrize("comp", ["1", "0"])
@pytest.mark.parametrize("case", ["one_count", "byte_gid", "two_byte_gid"])
def test_comp_sort_widths(msa_mod, tmp_path, monkeypatch, case, comp):
    monkeypatch.setenv("MSA_SORT", "radix")
    monkeypatch.setenv("MSA_COMP_SORT", comp)
    data = corpus(case_words(case), seed=len(case))
    with msa_mod.Context(0) as c:  # the library reads both settings when the context is made
        check_against_oracle(msa_mod, c, data, tmp_path, f"comp_{case}_{comp}")


def test_comp_sort_zipf(msa_mod, tmp_path, monkeypatch):
    """A Zipfian table (hundreds of distinct counts, the bench's shape) forced
    through the composite sort."""
    monkeypatch.setenv("MSA_SORT", "radix")
    data = msa_mod.gen_corpus(20000, mode="zipf", seed=11)
    with msa_mod.Context(0) as c:
        check_against_oracle(msa_mod, c, data, tmp_path, "comp_zipf")


def case_runs(case):
    """Tie runs of bounded length: groups sharing their first 8 key bytes and a
    count (k_tie_seg orders runs of <= 64 entries; one longer run sends the
    round through the radix sort)."""
    ws = []
    if case == "short_runs":  # runs of 2..64; long keys tie again on bytes 8..23 (a second round)
        for g in range(160):
            size, cnt = 2 + g % 63, 1 + g % 3
            ws += [("q" + letters(g, 7) + letters(i, 2), cnt) for i in range(size)]
        for g in range(40):
            ws += [("zz" + letters(g, 6) + "abcdefghijklmnop" + letters(i, 2), 2) for i in range(1 + g % 20)]
        return ws
    sizes = [64] * 40 if case == "runs_64" else [64] * 20 + [65] + [3] * 50
    for g, size in enumerate(sizes):
        ws += [("r" + letters(g, 7) + letters(i, 3), 1) for i in range(size)]
    return ws


@pytest.mark.parametrize("seg", ["1", "0"])
@pytest.mark.parametrize("case", ["short_runs", "runs_64", "runs_65"])
def test_tie_rounds_short_runs(msa_mod, tmp_path, monkeypatch, case, seg):
    """k_tie_seg (MSA_TIE_SEG=1, the default) against the radix-sorted tie
    rounds (MSA_TIE_SEG=0) and the oracle: runs of up to 64 entries, exactly
    64, and one of 65 (the round falls back to the radix sort)."""
    monkeypatch.setenv("MSA_SORT", "radix")
    monkeypatch.setenv("MSA_TIE_SEG", seg)
    data = corpus(case_runs(case), seed=7 + len(case))
    with msa_mod.Context(0) as c:
        check_against_oracle(msa_mod, c, data, tmp_path, f"tieseg_{case}_{seg}")


def test_blob_regrow(msa_mod, tmp_path, monkeypatch):
    """The key blob of radix-sorted tables (k_blob_len, the offsets' scan,
    k_blob_write) against the oracle, three inputs on one context: the second
    holds 70-byte words, longer than the blob estimate allows for (48 bytes
    per long word) -- its blob is written past the capacity, grown and written
    again; the third is a high-cardinality table of > 1 M keys."""
    monkeypatch.setenv("MSA_SORT", "radix")
    with msa_mod.Context(0) as c:
        check_against_oracle(msa_mod, c, corpus(case_words("byte_gid"), seed=3), tmp_path, "blob_small")
        ws = [(letters(i, 6) + "x" * 63 + letters(i, 1), 1 + i % 2) for i in range(4000)]
        ws += [(letters(i, 5), 1) for i in range(3000)]
        check_against_oracle(msa_mod, c, corpus(ws, seed=5), tmp_path, "blob_long")
        big = msa_mod.gen_corpus(100000, mode="highcard", seed=9)
        check_against_oracle(msa_mod, c, big, tmp_path, "blob_hc")
