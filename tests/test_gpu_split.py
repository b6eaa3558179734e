"""GPU parity of the column splitter (msa_csvcol_*, driven by
msa/split_columns.py, the host mirror of split_csv_columns.py): output files
byte-identical to the real script's (tests/golden/split/) and to the oracle
on fresh torture / Zipf corpora."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, "golden"))
import split_oracle  # noqa: E402
from test_split_oracle import CASES, GOLD, case_dialect, load_case  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", CASES)
def test_split_golden(msa_mod, name, tmp_path):
    from msa.split_columns import split_csv_columns

    data, args, exp = load_case(name)
    inp = tmp_path / "in.csv"
    inp.write_bytes(data)
    od = tmp_path / "cols"
    # the script's own invocation: --delimiter as recorded, else the host
    # sniffs (delimiter + skipinitialspace); --quotechar and --encoding as recorded
    delim = args[args.index("--delimiter") + 1] if "--delimiter" in args else None
    _, quote, _, enc = case_dialect(name, args)
    kw = dict(quotechar=quote, encoding=enc, no_header="--no-header" in args)
    if exp is None:  # UnicodeDecodeError: a byte the single-byte codec leaves undefined, as the script raises
        with pytest.raises((SystemExit, msa_mod.MsaError, UnicodeDecodeError)):
            split_csv_columns(str(inp), str(od), delim, **kw)
        return
    split_csv_columns(str(inp), str(od), delim, **kw)
    got = {p.name: p.read_bytes() for p in od.iterdir()}
    assert got == exp


def test_split_existing_files_get_suffixes(msa_mod, tmp_path):
    """Without --force, names of files already present are skipped (_2, _3, ...)."""
    from msa.split_columns import split_csv_columns

    inp = tmp_path / "in.csv"
    inp.write_bytes(b"a,b\n1,2\n")
    od = tmp_path / "cols"
    first = split_csv_columns(str(inp), str(od), ",")
    second = split_csv_columns(str(inp), str(od), ",")
    assert [p.name for p in first] == ["a.csv", "b.csv"]
    assert [p.name for p in second] == ["a_2.csv", "b_2.csv"]
    assert split_csv_columns(str(inp), str(od), ",", force=True)[0].name == "a.csv"


@pytest.mark.parametrize("seed,has_header", [(1, True), (2, False), (3, True)])
def test_split_torture_vs_oracle(msa_mod, seed, has_header):
    from make_wcs_golden import torture

    data = torture(2000 + seed, 500).encode("utf-8")
    first, bodies = split_oracle.split_columns(data, has_header)
    with msa_mod.WordCountPerSong(0) as w:
        w.load_csv(data)
        nc, _ = w.split_columns(has_header)
        assert nc == len(first)
        assert [w.column_header(i) for i in range(nc)] == first
        assert [w.column_body(i) for i in range(nc)] == bodies


def test_split_zipf_vs_oracle(msa_mod):
    data = msa_mod.gen_corpus(3000, mode="zipf", seed=17, crlf=True)
    first, bodies = split_oracle.split_columns(data, True)
    with msa_mod.WordCountPerSong(0) as w:
        w.load_csv(data)
        nc, nr = w.split_columns(True)
        assert nr == 3000
        assert [w.column_body(i) for i in range(nc)] == bodies
        # the same context then runs the per-song counter (shared buffer pool)
        w.count()
        assert w.summary()["total_rows"] == 3000


def test_split_cli(msa_mod, tmp_path):
    """`python -m msa.split_columns` (the script's command line) writes the
    script's files and prints its summary line."""
    import subprocess

    data, args, exp = load_case("basic")
    inp = tmp_path / "in.csv"
    inp.write_bytes(data)
    od = tmp_path / "cols"
    r = subprocess.run([sys.executable, "-m", "msa.split_columns", str(inp), "--output-dir", str(od)] + args,
                       capture_output=True, timeout=120, cwd=msa_mod.PKG_DIR)
    assert r.returncode == 0, r.stderr
    assert "Concluído. 4 arquivo(s) gerado(s) em:".encode() in r.stdout
    assert {p.name: p.read_bytes() for p in od.iterdir()} == exp


def dialect_corpus(seed: int, rows: int, delim: str, quote: str, space_after: bool) -> bytes:
    """Random rows of a dialect: fields holding the delimiter, the quotechar,
    '"', CR/LF, spaces and UTF-8 letters, quoted (quotechar doubled) when they
    need it or at random; with space_after, ' ' after delimiters (sometimes
    before a quoted field) -- skipinitialspace input."""
    import random

    rnd = random.Random(seed)
    alpha = ["a", "b", "Zé", " ", delim, quote, '"', "\n", "\r\n", "x y", "ü"]
    out = []
    for _ in range(rows):
        fields = []
        for _ in range(rnd.randint(1, 5)):
            v = "".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 6)))
            if any(c in v for c in (delim, quote, "\n", "\r")) or rnd.random() < 0.3:
                v = quote + v.replace(quote, quote * 2) + quote
            elif v.startswith(" ") and space_after:
                v = v.lstrip(" ")  # would be skipped: not an interesting difference
            fields.append(v)
        sep = delim + (" " * rnd.randint(0, 2) if space_after else "")
        out.append(sep.join(fields))
    return ("\n".join(out) + "\n").encode("utf-8")


@pytest.mark.parametrize("delim,quote,skip", [(",", "'", False), (";", "|", False), (",", '"', True), (",", "'", True),
                                              ("\t", "'", True), (" ", '"', True), (";", ",", False)])
def test_split_dialects_vs_oracle(msa_mod, delim, quote, skip):
    """--quotechar and skipinitialspace dialects (split_csv_columns.py:58,
    90-95): the GPU reader and writer against the oracle on random rows."""
    for seed in range(3):
        data = dialect_corpus(300 + seed, 400, delim, quote, skip)
        first, bodies = split_oracle.split_columns(data, True, delim, quote, skip)
        with msa_mod.WordCountPerSong(0) as w:
            w.set_dialect(delim, quote, skip)
            w.load_csv(data)
            nc, _ = w.split_columns(True)
            assert [w.column_header(i) for i in range(nc)] == first
            assert [w.column_body(i) for i in range(nc)] == bodies


def test_split_quotechar_equal_to_default_delimiter(msa_mod, tmp_path):
    """--quotechar ',' with a ';' delimiter (Python's csv accepts it): the host
    mirror sets the pair in one call, so the old ',' delimiter does not make
    the new quotechar look invalid."""
    from msa.split_columns import split_csv_columns

    data = dialect_corpus(7, 200, ";", ",", False)
    first, bodies = split_oracle.split_columns(data, True, ";", ",", False)
    inp = tmp_path / "in.csv"
    inp.write_bytes(data)
    files = split_csv_columns(str(inp), str(tmp_path / "cols"), delimiter=";", quotechar=",", encoding="utf-8")
    assert len(files) == len(bodies)
    for f, b in zip(files, bodies):
        assert f.read_bytes().endswith(b)


def test_per_song_counter_refuses_other_quoting(msa_mod):
    """csv.DictReader(fh, delimiter=...) (word_count_per_song.py:115) reads the
    default dialect: msa_wcs_run refuses a quotechar / skipinitialspace."""
    with msa_mod.WordCountPerSong(0) as w:
        w.set_quoting("'", False)
        with pytest.raises(msa_mod.MsaError):
            w.run(b"artist,song,text\nA,S,hello world\n")


def test_encodings_outside_the_byte_path(msa_mod, tmp_path):
    """Multi-byte codecs other than UTF-8 are refused by the splitter; a
    single-byte codec is the splitter's only (the per-song counter's tokens are
    Unicode words of UTF-8 text)."""
    from msa import WordCountPerSong
    from msa.split_columns import split_csv_columns

    inp = tmp_path / "in.csv"
    inp.write_bytes(b"a,b\n1,2\n")
    for enc in ("shift_jis", "utf-16", "gbk"):
        with pytest.raises(SystemExit):
            split_csv_columns(str(inp), str(tmp_path / enc), ",", encoding=enc)
    with WordCountPerSong(0) as w:
        w.set_encoding("latin-1")
        w.load_csv(b"artist,song,text\na,b,c\n")
        with pytest.raises(msa_mod.MsaError):
            w.count()
