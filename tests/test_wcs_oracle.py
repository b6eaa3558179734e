"""Per-song word counter oracle (oracle/wcs_oracle.py) pinned against outputs
of the real reference script (tests/golden/wcs/, make_wcs_golden.py)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import wcs_oracle  # noqa: E402
from conftest import golden_delimiter, golden_dialect  # noqa: E402,F401

GOLD = os.path.join(HERE, "golden", "wcs")
CASES = sorted(os.listdir(GOLD))


def load_case(name):
    d = os.path.join(GOLD, name)
    rd = lambda f: open(os.path.join(d, f), "rb").read()  # noqa: E731
    exp = None
    if not os.path.exists(os.path.join(d, "error.txt")):
        exp = (int(rd("rows.txt")), rd("word_counts_by_song.csv"), rd("word_counts_global.csv"))
    return rd("input.csv"), exp


def case_encoding(name):
    from conftest import golden_encoding

    return golden_encoding(open(os.path.join(GOLD, name, "args.txt")).read().split())


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    data, exp = load_case(name)
    d = golden_delimiter(os.path.join(GOLD, name))
    enc = case_encoding(name)
    if exp is None:
        with pytest.raises(wcs_oracle.WcsError):
            wcs_oracle.word_count_per_song(data, d, enc)
        return
    assert wcs_oracle.word_count_per_song(data, d, enc) == exp


def test_oracle_refuses_bad_bytes():
    with pytest.raises(wcs_oracle.WcsError):
        wcs_oracle.word_count_per_song(b"artist,song,text\nA,S,ab\xffcd\n")
    with pytest.raises(wcs_oracle.WcsError):
        wcs_oracle.word_count_per_song(b"artist,song,text\nA,S,ab\x00cd\n")
    with pytest.raises(wcs_oracle.WcsError):
        wcs_oracle.word_count_per_song(b"artist,song,text\nA,S,\"" + b"x" * 131073 + b"\"\n")
