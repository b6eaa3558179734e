"""Shared test helpers.

CPU tests (`-m "not gpu"`) check the oracle against the golden vectors made by
the REAL reference (tests/golden/), the host logic and the C ABI surface.
GPU tests (`-m gpu`) run libmsa_hip on an MI355X and compare it byte-for-byte
with the oracle / golden vectors.  The oracle (oracle/msa_oracle) is only ever
used here as the checker.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "music-analyst-ai_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE = os.path.join(REPO, "oracle", "msa_oracle")
REF_BIN = os.path.join(REPO, "oracle", "_ref", "parallel_spotify")
MPIRUN = "/opt/conda/bin/mpirun"

if PKG not in sys.path:
    sys.path.insert(0, PKG)


_CONFIG = None


def pytest_configure(config):
    global _CONFIG
    _CONFIG = config
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libmsa_hip kernels)")


def say(msg):
    """A line on the terminal now, past pytest's output capture: long fixture
    work (multi-GB corpora, their oracle runs) shows progress instead of
    looking hung."""
    capman = _CONFIG.pluginmanager.getplugin("capturemanager") if _CONFIG else None
    if capman is None:
        print(msg, flush=True)
        return
    with capman.global_and_fixture_disabled():
        print(msg, flush=True)


def run_with_heartbeat(cmd, timeout, what, every=30, env=None):
    """subprocess.run(cmd) that prints a progress line every `every` seconds."""
    import time

    t0 = time.time()
    with subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env) as p:
        while True:
            try:
                out, err = p.communicate(timeout=every)
                break
            except subprocess.TimeoutExpired:
                if time.time() - t0 > timeout:
                    p.kill()
                    p.communicate()
                    raise
                say(f"  [{what}: {time.time() - t0:.0f} s]")
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def read_outputs(outdir):
    """The files a parallel_spotify run leaves in its --output-dir."""
    out = {
        "word_counts.csv": _read(os.path.join(outdir, "word_counts.csv")),
        "top_artists.csv": _read(os.path.join(outdir, "top_artists.csv")),
        "split": {},
    }
    sd = os.path.join(outdir, "split_columns")
    if os.path.isdir(sd):
        for n in sorted(os.listdir(sd)):
            out["split"][n] = _read(os.path.join(sd, n))
    with open(os.path.join(outdir, "performance_metrics.json")) as f:
        m = json.load(f)
    out["metrics"] = {k: m[k] for k in ("processes", "total_songs", "total_words")}
    return out


def files_equal(a, b, chunk=1 << 24):
    """Byte-for-byte comparison of two (possibly multi-GB) files."""
    if os.path.getsize(a) != os.path.getsize(b):
        return False
    with open(a, "rb") as fa, open(b, "rb") as fb:
        while True:
            x, y = fa.read(chunk), fb.read(chunk)
            if x != y:
                return False
            if not x:
                return True


def table_counts(path):
    """{key: count} of a word_counts.csv / top_artists.csv (write_csv_entry lines,
    parallel_spotify.c:307-319)."""
    out = {}
    with open(path, "rb") as f:
        f.readline()
        for line in f:
            j = line.rindex(b'",')
            out[line[1:j].replace(b'""', b'"')] = int(line[j + 2:])
    return out


def table_bytes(header, counts):
    """The table as write_table_csv writes it: entry_compare_desc order (count
    desc, then strcmp; parallel_spotify.c:176-188), write_csv_entry lines."""
    rows = sorted(counts.items(), key=lambda kv: (-kv[1], kv[0]))
    return header + b"".join(b'"' + k.replace(b'"', b'""') + b'",' + str(v).encode() + b"\n" for k, v in rows)


def hash_file(path, skip_first_line, h):
    with open(path, "rb") as f:
        if skip_first_line:
            f.readline()
        while True:
            b = f.read(1 << 24)
            if not b:
                return
            h.update(b)


def run_oracle(csv_path, outdir, ranks=1, word_limit=0, artist_limit=0, timeout=300):
    """The CPU oracle (C restatement of parallel_spotify.c, virtual np)."""
    if not os.path.exists(ORACLE):
        # a missing checker must never turn parity tests into skips
        pytest.fail("oracle/msa_oracle not built (make -C oracle): parity cannot be checked")
    cmd = [ORACLE, csv_path, "--output-dir", outdir, "--ranks", str(ranks)]
    if word_limit:
        cmd += ["--word-limit", str(word_limit)]
    if artist_limit:
        cmd += ["--artist-limit", str(artist_limit)]
    return run_with_heartbeat(cmd, timeout, "oracle " + os.path.basename(csv_path))


@pytest.fixture(scope="session")
def msa_mod():
    import msa

    msa.load()
    return msa


def golden_delimiter(case_dir):
    """The delimiter the reference script ran a golden case with: its
    --delimiter, else what its csv.Sniffer picked on the 65536-character
    sample (the stdlib class the script calls, via msa/sniff.py)."""
    args = open(os.path.join(case_dir, "args.txt")).read().split()
    if "--delimiter" in args:
        return args[args.index("--delimiter") + 1]
    from msa.sniff import detect_delimiter, read_sample

    try:
        return detect_delimiter(read_sample(os.path.join(case_dir, "input.csv"), golden_encoding(args)))
    except UnicodeDecodeError:
        return ","


def golden_encoding(args):
    """The --encoding a golden case ran with (the scripts' default utf-8-sig)."""
    return args[args.index("--encoding") + 1] if "--encoding" in args else "utf-8-sig"


def golden_dialect(case_dir):
    """(delimiter, skipinitialspace) of split_csv_columns.py's detect_csv_params."""
    args = open(os.path.join(case_dir, "args.txt")).read().split()
    if "--delimiter" in args:
        return args[args.index("--delimiter") + 1], False
    from msa.sniff import detect_csv_params, read_sample

    try:
        return detect_csv_params(read_sample(os.path.join(case_dir, "input.csv"), golden_encoding(args)))
    except UnicodeDecodeError:
        return ",", False


# BASELINE configs[3]'s corpus family at a size one GPU box holds twice over:
# 20M songs of the bench generator (~4.7 GB > 2^32 bytes).  Written once per
# session with its oracle outputs (np = 1); test_gpu_scale.py runs it on one
# context, test_gpu_dist.py as sharded worlds (Python driver and C host).
C3_SONGS = 20_000_000


@pytest.fixture(scope="session")
def configs3_corpus(msa_mod, tmp_path_factory):
    d = tmp_path_factory.mktemp("c3")
    path = str(d / "c3.csv")
    data = msa_mod.gen_corpus(C3_SONGS, mode="zipf", seed=1, vocab=50000, n_artists=5000, words_per_song=30)
    assert len(data) > (1 << 32)
    with open(path, "wb") as f:
        f.write(data)
    del data
    od = str(d / "o")
    r = run_oracle(path, od, ranks=1, timeout=600)
    assert r.returncode == 0, r.stderr
    return path, od
