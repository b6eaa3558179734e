"""CPU: the C ABI surface of libmsa_hip (no kernel launches without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO


def header_symbols():
    with open(os.path.join(REPO, "include", "msa_hip.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*|void \*)\s*\**(msa_\w+)\s*\(", txt, re.M)))


def test_header_declares_what_binding_knows(msa_mod):
    assert header_symbols() == sorted(msa_mod.EXPORTS)


def test_library_exports_every_declared_symbol(msa_mod):
    lib = ctypes.CDLL(msa_mod.LIB_PATH)
    for name in header_symbols():
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", msa_mod.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (msa_\w+)", nm))
    assert set(header_symbols()) <= exported


def test_library_is_gfx950(msa_mod):
    """The kernels are gfx950 code objects (no other offload target)."""
    blob = open(msa_mod.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_no_gpu_means_loud_failure(msa_mod):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(msa_mod.MsaError) as e:
        msa_mod.Context(0)
    assert e.value.code == -2  # MSA_ERR_HIP


def test_generator_is_deterministic(msa_mod):
    a = msa_mod.gen_corpus(500, mode="zipf", seed=5)
    b = msa_mod.gen_corpus(500, mode="zipf", seed=5)
    c = msa_mod.gen_corpus(500, mode="zipf", seed=6)
    assert a == b and a != c
    assert a.startswith(b"artist,song,link,text\n")


def test_generator_modes(msa_mod):
    t = msa_mod.gen_corpus(300, mode="torture", seed=2)
    h = msa_mod.gen_corpus(300, mode="highcard", seed=2)
    z = msa_mod.gen_corpus(300, mode="zipf", seed=2, crlf=True)
    assert b"\r\n" in z
    assert len(h) > 0 and len(t) > 0


def test_table_csv_format(msa_mod):
    got = msa_mod.table_csv_bytes([(b'a"b', 3), (b"c", 1)], "word")
    assert got == b'word,count\n"a""b",3\n"c",1\n'
    assert msa_mod.table_csv_bytes([(b"x", 2), (b"y", 1)], "artist", limit=1) == b'artist,count\n"x",2\n'


def test_cli_bench_mode_arguments(tmp_path):
    """The C host's bench mode (bench.py --driver chost) refuses a run without
    a synthetic corpus, before any rank or GPU starts (no GPU needed)."""
    import subprocess

    cli = os.path.join(PKG, "bin", "parallel_spotify")
    p = subprocess.run([cli, "-", "--bench-steps", "2", "--output-dir", str(tmp_path / "o")], capture_output=True,
                       timeout=60)
    assert p.returncode != 0
    assert b"--bench-steps needs --synthetic-songs" in p.stderr
