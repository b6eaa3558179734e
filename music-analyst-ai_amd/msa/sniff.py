"""Delimiter detection of the row (f) scripts, for the Python hosts.

word_count_per_song.py detect_delimiter (42-49) and split_csv_columns.py
detect_csv_params (48-66) read the first 65536 characters of the file (opened
with the script's encoding, newline="") and ask the stdlib's csv.Sniffer --
these functions do exactly that (the same stdlib class; the C host has a
restatement, host/msa_sniff.c, checked against it by tests/test_sniff.py)."""
from __future__ import annotations

import csv
from typing import Tuple


def read_sample(path: str, encoding: str = "utf-8-sig", size: int = 65536) -> str:
    with open(path, "r", encoding=encoding, newline="") as fh:
        return fh.read(size)


def detect_delimiter(sample: str) -> str:
    """word_count_per_song.py:42-49 -- the sniffed delimiter, ',' when sniff fails."""
    try:
        return csv.Sniffer().sniff(sample).delimiter
    except csv.Error:
        return ","


def detect_csv_params(sample: str) -> Tuple[str, bool]:
    """split_csv_columns.py:48-66 -- (delimiter, skipinitialspace); (',', False) on failure."""
    try:
        d = csv.Sniffer().sniff(sample)
        return d.delimiter, bool(d.skipinitialspace)
    except Exception:
        return ",", False


def gpu_supported(delimiter: str, quotechar: str = '"') -> bool:
    """What the GPU reader implements: one ASCII byte other than the quotechar, CR, LF, NUL."""
    return len(delimiter) == 1 and 0 < ord(delimiter) < 128 and delimiter not in quotechar + "\r\n"
