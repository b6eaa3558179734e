"""GPU: the drop-in CLI (music-analyst-ai_amd/bin/parallel_spotify, the C host
over libmsa_hip) against the reference's own outputs -- same files, same bytes,
same stdout (parallel_spotify.c:1027-1053)."""
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG, read_outputs
from test_oracle import CASES, golden

pytestmark = pytest.mark.gpu
CLI = os.path.join(PKG, "bin", "parallel_spotify")


@pytest.mark.parametrize("writer", ["host", "device"])
@pytest.mark.parametrize("case", [c for c in CASES if c.startswith(("zipf", "torture", "multiline", "nul", "long"))])
def test_cli_matches_reference(case, writer, tmp_path):
    """writer: word_counts.csv / top_artists.csv formatted by the host loop
    (tables up to MSA_CSV_HOST_MAX lines, the default for these sizes) or on
    the device (k_csv_len, scan, k_csv_put: MSA_CSV_HOST_MAX=0)."""
    res, files = golden(case, 1)
    out = tmp_path / "out"
    env = dict(os.environ, MSA_CSV_HOST_MAX="0" if writer == "device" else str(1 << 20))
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(out)],
                       capture_output=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["metrics"] == {k: res[k] for k in ("processes", "total_songs", "total_words")}
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert got["split"] == files["split"]
    assert p.stdout.decode("latin-1") == res["stdout"]
    m = json.load(open(out / "performance_metrics.json"))
    assert set(m) == {"processes", "total_songs", "total_words", "compute_time", "total_time"}


@pytest.mark.parametrize("writer", ["host", "device"])
def test_cli_limits(writer, tmp_path):
    case = "zipf_small"
    res, files = golden(case, 1)
    out = tmp_path / "out"
    env = dict(os.environ, MSA_CSV_HOST_MAX="0" if writer == "device" else str(1 << 20))
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(out),
                        "--word-limit", "7", "--artist-limit", "3"], capture_output=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    w = open(out / "word_counts.csv", "rb").read()
    a = open(out / "top_artists.csv", "rb").read()
    assert w == b"\n".join(files["word_counts.csv"].split(b"\n")[:8]) + b"\n"
    assert a == b"\n".join(files["top_artists.csv"].split(b"\n")[:4]) + b"\n"


@pytest.mark.parametrize("case,msg", [("empty_file", b"Dataset does not contain a header row"),
                                      ("bad_header", b"Unable to parse dataset header")])
def test_cli_errors(case, msg, tmp_path):
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(tmp_path / "o")],
                       capture_output=True, timeout=120)
    assert p.returncode != 0
    assert msg in p.stderr


# ------------------------------------------------------------------ ranks
# --processes N: N rank processes (host shared-memory transport when they
# share the box's one GPU; RCCL with one GPU per rank).  Results must equal
# the single-process reference for every N -- the reference's own depend on
# -np (tests/test_oracle.py::test_reference_is_np_dependent).
@pytest.mark.parametrize("case,procs", [("zipf_small", 2), ("zipf_small", 3), ("torture_3", 2), ("torture_17", 4),
                                        ("zipf_crlf", 3), ("nul_bytes", 2), ("long_words", 2),
                                        ("multiline_artist_header", 2), ("quotes_everywhere", 3), ("header_only", 2),
                                        ("highcard_small", 4), ("cr_only", 2)])
def test_cli_processes_match_single(case, procs, tmp_path):
    if case not in CASES:
        pytest.skip(f"no golden case {case}")
    res, files = golden(case, 1)
    out = tmp_path / "out"
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(out),
                        "--processes", str(procs)], capture_output=True, timeout=180)
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["metrics"] == {"processes": procs, "total_songs": res["total_songs"], "total_words": res["total_words"]}
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert got["split"] == files["split"]
    assert p.stdout.decode("latin-1") == res["stdout"]


def test_cli_rank_path_rccl_world_of_one(tmp_path):
    """The RCCL transport end to end on the box's one GPU (a world of one:
    communicator init, all-gathers, send/recv to self)."""
    case = "zipf_small"
    res, files = golden(case, 1)
    out = tmp_path / "out"
    env = dict(os.environ, MSA_RANK_PATH="1", MSA_TRANSPORT="rccl")
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(out)],
                       capture_output=True, timeout=180, env=env)
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert got["split"] == files["split"]
    assert p.stdout.decode("latin-1") == res["stdout"]


def test_cli_processes_limits(tmp_path):
    case = "zipf_small"
    res, files = golden(case, 1)
    out = tmp_path / "out"
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(out), "--processes", "3",
                        "--word-limit", "7", "--artist-limit", "3"], capture_output=True, timeout=180)
    assert p.returncode == 0, p.stderr
    assert open(out / "word_counts.csv", "rb").read() == b"\n".join(files["word_counts.csv"].split(b"\n")[:8]) + b"\n"
    assert open(out / "top_artists.csv", "rb").read() == b"\n".join(files["top_artists.csv"].split(b"\n")[:4]) + b"\n"
    assert p.stdout.decode("latin-1") == res["stdout"]


@pytest.mark.parametrize("case,msg", [("empty_file", b"Dataset does not contain a header row"),
                                      ("bad_header", b"Unable to parse dataset header")])
def test_cli_processes_errors(case, msg, tmp_path):
    """A failing rank ends the whole job (the others may wait in a collective)."""
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(tmp_path / "o"),
                        "--processes", "2"], capture_output=True, timeout=120)
    assert p.returncode != 0
    assert msg in p.stderr


@pytest.mark.parametrize("procs,transport", [(1, None), (2, "shm"), (4, "shm"), (1, "rccl")])
def test_cli_bench_mode(msa_mod, procs, transport, tmp_path):
    """bench.py --driver chost: the C host's bench mode (each rank generates its
    song range of the synthetic corpus, times the whole pipeline) reports the
    corpus bytes of all ranks and rank 0's stage profile."""
    env = dict(os.environ)
    if transport:
        env["MSA_TRANSPORT"] = transport
    songs = 20000
    p = subprocess.run([CLI, "-", "--synthetic-songs", str(songs), "--processes", str(procs), "--bench-steps", "2",
                        "--bench-warmup", "1", "--output-dir", str(tmp_path / "o")],
                       capture_output=True, timeout=180, env=env)
    assert p.returncode == 0, p.stderr
    res = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert res["driver"] == "chost" and res["ranks"] == procs and res["steps"] == 2
    assert res["bytes_total"] == len(msa_mod.gen_corpus(songs, mode="zipf", seed=1))
    assert res["stages"]["csv_scan"][1] == 2 and res["seconds"] > 0


# ------------------------------------------------------------- under mpirun
# The reference is launched as `mpirun -np N ./bin/parallel_spotify <csv>`
# (scripts/run_performance.sh:23).  The drop-in run the same way joins the N
# processes as one job (host/msa_ranks.c msa_launcher_run): the np=1 results,
# written once, with "processes": N.
MPIRUN = "/opt/conda/bin/mpirun"


def _no_launcher_env():
    return {k: v for k, v in os.environ.items()
            if not k.startswith(("PMI_", "OMPI_", "PMIX_", "MPI_LOCAL", "HYDRA"))}


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun in this image")
@pytest.mark.parametrize("case,np_", [("zipf_small", 2), ("zipf_small", 4), ("torture_17", 4), ("torture_3", 2),
                                      ("multiline_artist_header", 2), ("highcard_small", 4), ("nul_bytes", 2),
                                      ("header_only", 2)])
def test_cli_under_mpirun_matches_single(case, np_, tmp_path):
    if case not in CASES:
        pytest.skip(f"no golden case {case}")
    res, files = golden(case, 1)
    out = tmp_path / "out"
    p = subprocess.run([MPIRUN, "-np", str(np_), CLI, os.path.join(GOLDEN, case, "input.csv"),
                        "--output-dir", str(out)], capture_output=True, timeout=180, env=_no_launcher_env())
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["metrics"] == {"processes": np_, "total_songs": res["total_songs"], "total_words": res["total_words"]}
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert got["split"] == files["split"]
    assert p.stdout.decode("latin-1") == res["stdout"]


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun in this image")
@pytest.mark.parametrize("case,msg", [("empty_file", b"Dataset does not contain a header row"),
                                      ("bad_header", b"Unable to parse dataset header")])
def test_cli_under_mpirun_errors(case, msg, tmp_path):
    """A rank that fails ends the job (mpirun itself leaves the others running)."""
    p = subprocess.run([MPIRUN, "-np", "2", CLI, os.path.join(GOLDEN, case, "input.csv"),
                        "--output-dir", str(tmp_path / "o")], capture_output=True, timeout=120,
                       env=_no_launcher_env())
    assert p.returncode != 0
    assert msg in p.stderr


@pytest.mark.parametrize("case,procs", [("highcard_small", 2), ("highcard_small", 4), ("zipf_small", 3),
                                        ("torture_17", 2)])
def test_cli_processes_dense_entries(case, procs, tmp_path):
    """--processes N with dense word entries forced on every rank
    (MSA_DENSE_MIN=0): the ranks' merge exports their dense entries' key
    partitions -- the same files as the reference at np=1."""
    if case not in CASES:
        pytest.skip(f"no golden case {case}")
    res, files = golden(case, 1)
    out = tmp_path / "out"
    p = subprocess.run([CLI, os.path.join(GOLDEN, case, "input.csv"), "--output-dir", str(out),
                        "--processes", str(procs)], capture_output=True, timeout=180,
                       env=dict(os.environ, MSA_DENSE_MIN="0"))
    assert p.returncode == 0, p.stderr
    got = read_outputs(str(out))
    assert got["metrics"] == {"processes": procs, "total_songs": res["total_songs"], "total_words": res["total_words"]}
    assert got["word_counts.csv"] == files["word_counts.csv"]
    assert got["top_artists.csv"] == files["top_artists.csv"]
    assert p.stdout.decode("latin-1") == res["stdout"]
