"""CPU oracle for the column splitter -- TEST INFRASTRUCTURE ONLY.

Only tests/ may use this module, and only as the checker; the product path
(libmsa_hip's msa_csvcol_* entry points, driven by msa/split_columns.py)
never calls it.

Restates the data part of /root/reference/scripts/split_csv_columns.py
main (124-199) for the dialect of detect_csv_params (48-66): the script's
--delimiter or its csv.Sniffer guess (default ','), the --quotechar (default
'"'), the sniffed skipinitialspace (False with --delimiter), and the
--encoding's BOM handling ("utf-8-sig" drops a leading BOM, "utf-8" keeps it
as the first field's first character; a single-byte codec such as latin-1
reads every byte as one character and writes it back unchanged):
* rows: CPython 3.10 csv.reader (wcs_oracle.csv_rows -- the same _csv state
  machine; blank lines are rows with no fields, csv.reader yields them);
* columns: len(first row); each later row contributes row[i] or "" (175-178);
* each value is written by csv.writer(lineterminator="\\n", QUOTE_MINIMAL)
  as a one-field row: quoted (quotechars doubled) when it holds the
  delimiter, the quotechar or '\\n' ('\\r' is NOT quoted with this
  lineterminator), and a lone empty value is written quoted.

Parity: pinned against outputs of the real script in tests/golden/split/
(tests/golden/make_split_golden.py).
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wcs_oracle import WcsError, _utf8_check, csv_rows  # noqa: E402,F401


def write_value(v: bytes, delim: bytes = b",", quote: bytes = b'"') -> bytes:
    """csv.writer(...).writerow([v]) with lineterminator '\\n', QUOTE_MINIMAL."""
    if v == b"" or any(c in v for c in delim + quote + b"\n"):
        return quote + v.replace(quote, quote + quote) + quote + b"\n"
    return v + b"\n"


def split_columns(data: bytes, has_header: bool = True, delimiter: str = ",", quotechar: str = '"',
                  skipinitialspace: bool = False, strip_bom: bool = True, utf8: bool = True):
    """-> (first-row fields, [body bytes of column i]) ; raises WcsError / ValueError("CSV vazio.").
    utf8 False: a single-byte codec (every byte one character; decode + encode
    the identity), so the same byte-level split with no UTF-8 check."""
    if utf8:
        _utf8_check(data)
    elif 0 in data:
        raise WcsError("line contains NUL")
    d, q = delimiter.encode(), quotechar.encode()
    rows = csv_rows(data, ord(delimiter), ord(quotechar), skipinitialspace, strip_bom)
    first = next(rows, None)
    if first is None:
        raise ValueError("CSV vazio.")
    nc = len(first)
    bodies = [[] for _ in range(nc)]
    if not has_header:
        for i in range(nc):
            bodies[i].append(write_value(first[i], d, q))
    for row in rows:
        for i in range(nc):
            bodies[i].append(write_value(row[i] if i < len(row) else b"", d, q))
    return first, [b"".join(b) for b in bodies]
