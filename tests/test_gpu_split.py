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
from conftest import golden_dialect  # noqa: E402
from test_split_oracle import CASES, GOLD, load_case  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", CASES)
def test_split_golden(msa_mod, name, tmp_path):
    from msa.split_columns import split_csv_columns

    data, args, exp = load_case(name)
    inp = tmp_path / "in.csv"
    inp.write_bytes(data)
    od = tmp_path / "cols"
    # the script's own invocation: --delimiter as recorded, else the host sniffs
    delim = args[args.index("--delimiter") + 1] if "--delimiter" in args else None
    _, skip = golden_dialect(os.path.join(GOLD, name))
    if exp is None or skip:  # skipinitialspace dialects are refused (not implemented on the GPU path)
        with pytest.raises((SystemExit, msa_mod.MsaError)):
            split_csv_columns(str(inp), str(od), delim, no_header="--no-header" in args)
        return
    split_csv_columns(str(inp), str(od), delim, no_header="--no-header" in args)
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
