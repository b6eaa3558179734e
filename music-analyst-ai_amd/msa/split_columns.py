"""split_csv_columns on the GPU: host mirror of
/root/reference/scripts/split_csv_columns.py (same arguments, file naming,
output bytes and messages) whose data path -- CSV record/field splitting and
the per-column csv.writer bytes -- runs in libmsa_hip (msa_csvcol_*,
csrc/msa_wcs.hip).  File naming and the final writes stay on the host, as in
the script (sanitize_filename 24-28, the name loop 159-174).

    python -m msa.split_columns data.csv [--output-dir D] [--delimiter ,]
           [--quotechar '"'] [--encoding utf-8-sig] [--no-header] [--force]

Without --delimiter the dialect is detect_csv_params' (46-66): the stdlib's
csv.Sniffer on the first 65536 characters (msa/sniff.py), ',' when it fails,
with its skipinitialspace; --quotechar is the reader's and the writer's quote
character either way.  --encoding utf-8-sig (default) drops a leading BOM and
writes one at the start of every output file; utf-8 keeps it as the first
header name's first character and writes none.  A single-byte ASCII-compatible
codec (latin-1, cp1252, ...; msa.single_byte_codec) reads every byte as one
character and writes it back unchanged, so the GPU's byte-level split is the
script's; the header names are decoded and written in that codec, and input
holding a byte the codec leaves undefined raises the script's
UnicodeDecodeError.  Known divergence, on that error path only: the error
comes from decoding the whole file at once, so its message gives the byte's
position in the file, where the script's TextIOWrapper reports it within the
chunk it was decoding; and when the byte lies past the script's 64 KiB sniff
sample the script has already written the column files' first rows when it
fails, while this path fails before writing any column file
(tests/test_split_oracle.py::test_split_undefined_byte_late).  The GPU reader takes one-byte ASCII delimiters and
quotechars other than CR, LF, NUL (and each other); multi-byte codecs other
than UTF-8 (UTF-16, Shift-JIS, ...) and other characters are refused.
"""
from __future__ import annotations

import argparse
import re
from pathlib import Path
from typing import List, Optional

from . import WordCountPerSong, single_byte_codec
from .sniff import detect_csv_params, gpu_supported, read_sample


def sanitize_filename(name: str, max_len: int = 80) -> str:
    """split_csv_columns.py:24-28: newlines to spaces, strip, runs of
    characters outside [\\w\\-. ] to '_', whitespace runs to '_', cut to 80."""
    s = (name or "").replace("\n", " ").replace("\r", " ").strip()
    s = re.sub(r"[^\w\-. ]+", "_", s, flags=re.UNICODE)
    s = re.sub(r"\s+", "_", s)
    return (s or "col")[:max_len]


def _header_line(h: str, delimiter: str = ",", quotechar: str = '"') -> str:
    """csv.writer(QUOTE_MINIMAL, lineterminator "\n", the dialect's quotechar).writerow([h])"""
    if h == "" or any(c in h for c in (delimiter, quotechar, "\n")):
        return quotechar + h.replace(quotechar, quotechar * 2) + quotechar + "\n"
    return h + "\n"


def split_csv_columns(csv_path: str, output_dir: Optional[str] = None, delimiter: Optional[str] = None,
                      quotechar: str = '"', encoding: str = "utf-8-sig", no_header: bool = False,
                      force: bool = False, device: int = 0) -> List[Path]:
    in_path = Path(csv_path)
    if not in_path.exists():
        raise SystemExit(f"Erro: arquivo não encontrado: {in_path}")
    enc = encoding.lower().replace("_", "-")
    utf8 = enc in ("utf-8-sig", "utf-8", "utf8")
    undefined = None if utf8 else single_byte_codec(encoding)
    if not utf8 and undefined is None:
        raise SystemExit(f"only UTF-8 and single-byte ASCII-compatible encodings are implemented on the GPU path, "
                         f"not {encoding!r}")
    text_enc = "utf-8" if utf8 else encoding  # header names: decoded and written in the file's encoding
    skipinitialspace = False
    if not delimiter:  # detect_csv_params: csv.Sniffer on the script's sample
        delimiter, skipinitialspace = detect_csv_params(read_sample(str(in_path), encoding))
    quotechar = quotechar or '"'  # detect_csv_params: (quotechar or '"')
    if not (gpu_supported(delimiter, quotechar) and gpu_supported(quotechar, delimiter)):
        raise SystemExit(f"dialect delimiter={delimiter!r} quotechar={quotechar!r} "
                         f"is not implemented on the GPU path")
    base_out = Path(output_dir) if output_dir else in_path.with_suffix("").parent / f"{in_path.stem}_columns"
    base_out.mkdir(parents=True, exist_ok=True)
    data = in_path.read_bytes()
    if undefined:  # bytes the codec leaves undefined: the script's reader raises UnicodeDecodeError
        import numpy as np

        if np.isin(np.frombuffer(data, np.uint8), np.array(sorted(undefined), np.uint8)).any():
            data.decode(encoding)
    with WordCountPerSong(device) as w:
        w.set_dialect(delimiter, quotechar, skipinitialspace)
        w.set_encoding(encoding)
        w.load_csv(data)
        try:
            ncols, _ = w.split_columns(has_header=not no_header)
        except Exception as e:  # MSA_ERR_NOHEADER carries the script's message
            if "CSV vazio" in str(e):
                raise SystemExit("CSV vazio.")
            raise
        if no_header:
            headers = [f"col{i + 1}" for i in range(ncols)]
        else:
            raw = [w.column_header(i).decode(text_enc) for i in range(ncols)]
            headers = [h if h.strip() else f"col{i + 1}" for i, h in enumerate(raw)]
        seen, names = set(), []
        for i, h in enumerate(headers, start=1):
            name = sanitize_filename(str(h)) or f"col{i}"
            cand, k = f"{name}.csv", 2
            while cand.lower() in seen or ((base_out / cand).exists() and not force):
                cand = f"{name}_{k}.csv"
                k += 1
            seen.add(cand.lower())
            names.append(cand)
        bom = "\ufeff".encode("utf-8") if enc == "utf-8-sig" else b""
        for i in range(ncols):
            with open(base_out / names[i], "wb") as fh:
                fh.write(bom)
                if not no_header:
                    fh.write(_header_line(headers[i], delimiter, quotechar).encode(text_enc))
                fh.write(w.column_body(i))
    print(f"Concluído. {ncols} arquivo(s) gerado(s) em: {base_out}")
    for name in names:
        print(f" - {base_out / name}")
    return [base_out / n for n in names]


def main(argv=None):
    ap = argparse.ArgumentParser(description="Split a CSV into one file per column (GPU data path).")
    ap.add_argument("csv_path")
    ap.add_argument("--output-dir", dest="output_dir", default=None)
    ap.add_argument("--delimiter", dest="delimiter", default=None)
    ap.add_argument("--quotechar", dest="quotechar", default='"')
    ap.add_argument("--encoding", dest="encoding", default="utf-8-sig")
    ap.add_argument("--no-header", dest="no_header", action="store_true")
    ap.add_argument("--force", dest="force", action="store_true")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    split_csv_columns(a.csv_path, a.output_dir, a.delimiter, a.quotechar, a.encoding, a.no_header, a.force, a.device)


if __name__ == "__main__":
    main()
