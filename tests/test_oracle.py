"""CPU: pin the oracle (oracle/msa_oracle.c) against the golden vectors that the
REAL reference produced (tests/golden/make_golden.py), at np=1 and np=4, and --
when the reference binary is built here -- against the reference itself on
fresh seeded corpora."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, MPIRUN, ORACLE, REF_BIN, PKG, read_outputs, run_oracle

# parallel_spotify cases hold np1/ and np4/ (tests/golden/wcs/ holds the per-song counter's vectors)
CASES = sorted(d for d in os.listdir(GOLDEN) if os.path.isdir(os.path.join(GOLDEN, d, "np1")))


def golden(case, np_):
    d = os.path.join(GOLDEN, case, f"np{np_}")
    with open(os.path.join(d, "result.json")) as f:
        res = json.load(f)
    files = {}
    if res["returncode"] == 0:
        for n in ("word_counts.csv", "top_artists.csv"):
            with open(os.path.join(d, n), "rb") as f:
                files[n] = f.read()
        sd = os.path.join(d, "split_columns")
        files["split"] = {n: open(os.path.join(sd, n), "rb").read() for n in sorted(os.listdir(sd))}
    return res, files


def test_golden_present():
    assert len(CASES) >= 20


@pytest.mark.parametrize("np_", [1, 4])
@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_golden(case, np_, tmp_path):
    res, files = golden(case, np_)
    out = tmp_path / "o"
    p = run_oracle(os.path.join(GOLDEN, case, "input.csv"), str(out), ranks=np_)
    if res["returncode"] != 0:
        assert p.returncode != 0
        assert res["stderr_first_line"].encode() in p.stderr
        return
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["metrics"] == {k: res[k] for k in ("processes", "total_songs", "total_words")}
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert got["split"] == files["split"]
    assert p.stdout.decode("latin-1") == res["stdout"]


def _have_ref():
    return os.path.exists(REF_BIN) and os.path.exists(MPIRUN)


@pytest.mark.skipif(not _have_ref(), reason="reference binary not built here (make -C oracle ref)")
@pytest.mark.parametrize("mode,seed,np_", [("torture", 101, 1), ("torture", 102, 3), ("torture", 103, 4),
                                           ("zipf", 104, 2), ("highcard", 105, 4)])
def test_oracle_matches_live_reference(mode, seed, np_, tmp_path):
    """Fresh seeds, not in the golden set: oracle == `mpirun -np P` reference."""
    gen = os.path.join(PKG, "bin", "msa_gen")
    csv = tmp_path / "in.csv"
    subprocess.run([gen, str(csv), "--songs", "800", "--mode", mode, "--seed", str(seed), "--vocab", "4000"],
                   check=True, capture_output=True)
    env = dict(os.environ, PATH="/opt/conda/bin:" + os.environ.get("PATH", ""))
    r = subprocess.run([MPIRUN, "-np", str(np_), REF_BIN, str(csv), "--output-dir", str(tmp_path / "r")],
                       capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    p = run_oracle(str(csv), str(tmp_path / "o"), ranks=np_)
    assert p.returncode == 0
    a, b = read_outputs(str(tmp_path / "r")), read_outputs(str(tmp_path / "o"))
    assert a == b
    assert r.stdout == p.stdout


def test_reference_is_np_dependent():
    """Documented reference behaviour: its even byte split of the
    column files (parallel_spotify.c:866-916) re-synchronises rank r>0 with a
    fresh quote state, so results depend on the process count.  libmsa_hip
    implements the np=1 semantics for any number of GPUs."""
    diffs = 0
    for case in CASES:
        r1, f1 = golden(case, 1)
        r4, f4 = golden(case, 4)
        if r1["returncode"] == 0 and (f1["word_counts.csv"] != f4["word_counts.csv"] or
                                      r1["total_songs"] != r4["total_songs"]):
            diffs += 1
    assert diffs >= 1


def test_song_ranges_sum_to_the_whole(msa_mod, tmp_path):
    """The checker of test_gpu_dist.py's full-size configs[3] test: the oracle
    over a corpus's song ranges (each with the header line), tables summed and
    ranked again (conftest.table_counts / table_bytes), split bodies
    concatenated -- byte-identical to the oracle over the whole corpus."""
    import xxhash

    from conftest import hash_file, table_bytes, table_counts

    total, parts = 20000, 4
    whole = b""
    header = None
    words, artists, songs, twords, hashes = {}, {}, 0, 0, {}
    for k in range(parts):
        lo, hi = total * k // parts, total * (k + 1) // parts
        data = msa_mod.gen_corpus(total, mode="zipf", seed=1, vocab=50000, n_artists=5000, words_per_song=30,
                                  first_song=lo, count=hi - lo)
        whole += data
        if k == 0:
            header = data[:data.index(b"\n") + 1]
        rp = tmp_path / f"r{k}.csv"
        rp.write_bytes((header if k else b"") + data)
        od = tmp_path / f"o{k}"
        assert run_oracle(str(rp), str(od)).returncode == 0
        for key, v in table_counts(str(od / "word_counts.csv")).items():
            words[key] = words.get(key, 0) + v
        for key, v in table_counts(str(od / "top_artists.csv")).items():
            artists[key] = artists.get(key, 0) + v
        m = json.loads((od / "performance_metrics.json").read_text())
        songs += m["total_songs"]
        twords += m["total_words"]
        for n in sorted(os.listdir(od / "split_columns")):
            p = str(od / "split_columns" / n)
            if k == 0:
                hashes[n] = xxhash.xxh3_128(open(p, "rb").readline())
            hash_file(p, True, hashes[n])
    wp = tmp_path / "whole.csv"
    wp.write_bytes(whole)
    assert run_oracle(str(wp), str(tmp_path / "ow")).returncode == 0
    exp = read_outputs(str(tmp_path / "ow"))
    assert table_bytes(b"word,count\n", words) == exp["word_counts.csv"]
    assert table_bytes(b"artist,count\n", artists) == exp["top_artists.csv"]
    m = json.loads((tmp_path / "ow" / "performance_metrics.json").read_text())
    assert (songs, twords) == (m["total_songs"], m["total_words"])
    for n, h in hashes.items():
        assert h.digest() == xxhash.xxh3_128(exp["split"][n]).digest(), n
