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
