"""CPU: the rank layer of the C host (music-analyst-ai_amd/host/msa_ranks.c,
used by `bin/parallel_spotify --processes N` in place of MPI): the shard
routing (the C twin of msa/dist.py head_owners / tail_plan), the launcher, and
the shared-memory transport's all-gather / all-to-all-v with N forked ranks
-- the gloo-world analogue for the C path; the RCCL transport and the GPU
pipeline over it are exercised by tests/test_gpu_cli.py."""
import os
import subprocess

import pytest

from conftest import PKG

BIN = os.path.join(PKG, "bin", "msa_ranks_test")


@pytest.fixture(scope="module")
def ranks_bin():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", PKG, "bin/msa_ranks_test"], check=True, capture_output=True, timeout=120)
    return BIN


def test_routing(ranks_bin):
    p = subprocess.run([ranks_bin, "routing"], capture_output=True, timeout=30)
    assert p.returncode == 0, p.stderr


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shm_exchange(ranks_bin, world):
    p = subprocess.run([ranks_bin, "exchange", str(world)], capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr


@pytest.mark.parametrize("world", [2, 4])
def test_failed_rank_ends_the_job(ranks_bin, world):
    """A rank that fails before a collective must not leave the others (and
    the launcher) waiting forever: the launcher returns its exit code."""
    p = subprocess.run([ranks_bin, "fail", str(world)], capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr


MPIRUN = "/opt/conda/bin/mpirun"
needs_mpirun = pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no MPICH Hydra mpirun in this image")


def _no_launcher_env():
    return {k: v for k, v in os.environ.items()
            if not k.startswith(("PMI_", "OMPI_", "PMIX_", "MPI_LOCAL", "HYDRA"))}


def _shm_leftovers():
    """msa_* blocks in /dev/shm, except those of a job still running (msa_<pid>_...
    with that process alive: another xdist worker's job, created after a
    test's `before` snapshot)."""
    out = []
    for f in os.listdir("/dev/shm"):
        if not f.startswith("msa_"):
            continue
        pid = f.split("_")[1]
        if pid.isdigit() and os.path.exists(f"/proc/{pid}"):
            continue
        out.append(f)
    return sorted(out)


@needs_mpirun
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_mpirun_ranks_join_one_job(ranks_bin, world, tmp_path):
    """`mpirun -np N` (Hydra, the reference's launcher: run_performance.sh:23)
    starts N unrelated processes; they join as one job over PMI-1 and a
    /dev/shm block and run the same all-gather / all-to-all-v checks as the
    forked ranks."""
    before = _shm_leftovers()
    p = subprocess.run([MPIRUN, "-np", str(world), ranks_bin, "launched"], capture_output=True, timeout=120,
                       cwd=tmp_path, env=_no_launcher_env())
    assert p.returncode == 0, p.stderr
    assert set(_shm_leftovers()) <= set(before)  # (other xdist workers' jobs may end meanwhile)


@needs_mpirun
def test_mpirun_failed_rank_ends_the_job(ranks_bin, tmp_path):
    """mpirun does not end the other processes when one exits with an error:
    the failing rank flags the job and the others leave their barriers."""
    before = _shm_leftovers()
    p = subprocess.run([MPIRUN, "-np", "3", ranks_bin, "launched", "fail"], capture_output=True, timeout=120,
                       cwd=tmp_path, env=_no_launcher_env())
    assert p.returncode != 0
    assert set(_shm_leftovers()) <= set(before)


@pytest.mark.parametrize("world", [2, 4])
def test_openmpi_environment_ranks_join(ranks_bin, world, tmp_path):
    """Open MPI's variables (OMPI_COMM_WORLD_RANK/SIZE, PMIX_NAMESPACE) and no
    PMI descriptor: the ranks poll for the block rank 0 publishes.  Rank 0 is
    started last, so the others really wait for it."""
    env = _no_launcher_env()
    ns = f"msa-test-{os.getpid()}-{world}"
    procs = []
    for r in list(range(1, world)) + [0]:
        e = dict(env, OMPI_COMM_WORLD_RANK=str(r), OMPI_COMM_WORLD_SIZE=str(world),
                 OMPI_COMM_WORLD_LOCAL_SIZE=str(world), PMIX_NAMESPACE=ns)
        procs.append(subprocess.Popen([ranks_bin, "launched"], env=e, cwd=tmp_path,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    for p in procs:
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err
    assert not any(ns.replace("-", "_") in f or ns in f for f in _shm_leftovers())


def test_launcher_spanning_nodes_is_refused(ranks_bin, tmp_path):
    """The shared block is node-local: a job whose ranks are not all on this
    node is refused, not silently split into per-node jobs."""
    e = dict(_no_launcher_env(), OMPI_COMM_WORLD_RANK="0", OMPI_COMM_WORLD_SIZE="4",
             OMPI_COMM_WORLD_LOCAL_SIZE="2", PMIX_NAMESPACE=f"msa-span-{os.getpid()}")
    p = subprocess.run([ranks_bin, "launched"], env=e, capture_output=True, timeout=60, cwd=tmp_path)
    assert p.returncode != 0 and b"more than one node" in p.stderr


@needs_mpirun
def test_mpirun_cli_without_gpu_fails_cleanly(tmp_path):
    """bin/parallel_spotify under mpirun on a host without a GPU: every rank
    fails (no device) and the job ends with an error instead of hanging or
    writing partial outputs; --processes next to the launcher's ranks is
    refused."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: the CLI runs (tests/test_gpu_cli.py)")
    cli = os.path.join(PKG, "bin", "parallel_spotify")
    if not os.path.exists(cli):
        pytest.skip("CLI not built")
    csv = tmp_path / "in.csv"
    csv.write_bytes(b"artist,song,link,text\nA,s,l,\"hello world\"\n")
    env = _no_launcher_env()
    p = subprocess.run([MPIRUN, "-np", "2", cli, str(csv), "--output-dir", str(tmp_path / "o")],
                       capture_output=True, timeout=120, env=env)
    assert p.returncode != 0
    assert not (tmp_path / "o" / "word_counts.csv").exists()
    p = subprocess.run([MPIRUN, "-np", "2", cli, str(csv), "--processes", "2", "--output-dir", str(tmp_path / "o")],
                       capture_output=True, timeout=120, env=env)
    assert p.returncode != 0 and b"--processes cannot be combined" in p.stderr


# ---------------------------------------------------------------- RCCL transport
# host/msa_rccl.c against the in-process HIP / RCCL stand-ins of
# host/test_stub (host memory, a thread per rank, RCCL's send/recv matching):
# the transport's bookkeeping -- not RCCL itself, which the GPU tests run.
RCCL_BIN = os.path.join(PKG, "bin", "msa_rccl_test")


@pytest.fixture(scope="module")
def rccl_bin():
    if not os.path.exists(RCCL_BIN):
        subprocess.run(["make", "-C", PKG, "bin/msa_rccl_test"], check=True, capture_output=True, timeout=120)
    return RCCL_BIN


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rccl_transport_exchanges(rccl_bin, world):
    """All-gathers and all-to-all-v rounds where some rank pairs exchange
    nothing (an empty send or receive must not be posted: RCCL would wait for
    it), on the transport's own stream and on an external one (no host wait);
    every pool buffer and stream released at the end."""
    p = subprocess.run([rccl_bin, "exchange", str(world)], capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr


def test_rccl_transport_pool(rccl_bin):
    """The device buffer pool: a free buffer that fits is reused, at most 16
    are in use (a 17th request fails), and the smallest free one is evicted to
    make room for a larger request."""
    p = subprocess.run([rccl_bin, "pool"], capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert b"more than 16 transport buffers in use" in p.stderr


@pytest.mark.parametrize("what,msg", [("initfail", b"ncclCommInitRank"), ("mallocfail", b"hipMalloc")])
def test_rccl_transport_failures(rccl_bin, what, msg):
    """msa_tr_rccl failing to set up its communicator returns NULL with
    nothing left allocated; an exchange buffer the device cannot provide
    fails that request only."""
    p = subprocess.run([rccl_bin, what], capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert msg in p.stderr
