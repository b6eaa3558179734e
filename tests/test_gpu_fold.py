"""GPU: the folded split scan (k_scan_fold, msa_k3.hip; MSA_FOLD=1) -- the
reader's chunk functions (K1), their scan (K2) and the record structure pass
(k_scan_struct) in one pass with a decoupled look-back over tiles of four
chunks.  Measured as fast as the three-kernel path, not faster, so
it is opt-in; these tests hold it to the same bytes as the reference at np=1
(read_csv_record / parse_csv_line / process_lyrics,
/root/reference/src/parallel_spotify.c:258-304, 350-394, 549-633): the
torture and edge corpora, the real reference's golden outputs, corpora of
thousands of tiles (look-backs across several 64-tile windows), and a fresh
context whose first split guesses the record count too low and runs again."""
import os

import pytest

from test_gpu_parity import EDGE, check_against_oracle, gpu_outputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fctx(msa_mod):
    old = os.environ.get("MSA_FOLD")
    os.environ["MSA_FOLD"] = "1"
    try:
        c = msa_mod.Context(0)  # the library reads the setting when the context is made
    finally:
        if old is None:
            os.environ.pop("MSA_FOLD")
        else:
            os.environ["MSA_FOLD"] = old
    yield c
    c.close()


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_fold_torture(msa_mod, fctx, tmp_path, seed):
    data = msa_mod.gen_corpus(1500, mode="torture", seed=seed)
    check_against_oracle(msa_mod, fctx, data, tmp_path, f"fold_torture{seed}")


@pytest.mark.parametrize("name", sorted(EDGE))
def test_fold_edge_cases(msa_mod, fctx, tmp_path, name):
    check_against_oracle(msa_mod, fctx, EDGE[name], tmp_path, f"fold_{name}")


@pytest.mark.parametrize("mode,songs,crlf", [("zipf", 3000, False), ("zipf", 2000, True), ("highcard", 3000, False)])
def test_fold_small_corpora(msa_mod, fctx, tmp_path, mode, songs, crlf):
    data = msa_mod.gen_corpus(songs, mode=mode, seed=17, vocab=20000, n_artists=500, crlf=crlf)
    check_against_oracle(msa_mod, fctx, data, tmp_path, f"fold_{mode}{songs}{int(crlf)}")


@pytest.mark.parametrize("mode", ["zipf", "highcard"])
def test_fold_many_tiles(msa_mod, fctx, tmp_path, mode):
    """~50 MB: ~800 tiles of 64 KiB, more workgroups than tiles per window."""
    data = msa_mod.gen_corpus(200_000, mode=mode, seed=23)
    check_against_oracle(msa_mod, fctx, data, tmp_path, f"fold_{mode}_many")
    # again on the same context: new status epoch, tickets continue
    check_against_oracle(msa_mod, fctx, data, tmp_path, f"fold_{mode}_many_again")


def test_fold_first_split_guess_too_low(msa_mod, tmp_path, monkeypatch):
    """A fresh context guesses a record per 64 bytes; a corpus of shorter
    records overflows that guess, and the split runs again with the count the
    folded scan returned."""
    monkeypatch.setenv("MSA_FOLD", "1")
    rows = b"".join(b"A%d,s,l,w%d x\n" % (i % 7, i % 11) for i in range(300_000))
    data = b"artist,song,link,text\n" + rows
    assert len(data) / 300_000 < 64
    with msa_mod.Context(0) as c:
        check_against_oracle(msa_mod, c, data, tmp_path, "fold_short_records")


def test_fold_golden_reference_np1(msa_mod, fctx):
    """Every golden case of the real reference (`mpirun -np 1`), folded."""
    from conftest import GOLDEN
    from test_oracle import CASES, golden

    for case in CASES:
        res, files = golden(case, 1)
        data = open(os.path.join(GOLDEN, case, "input.csv"), "rb").read()
        if res["returncode"] != 0:
            fctx.load_csv(data)
            with pytest.raises(msa_mod.MsaError) as e:
                fctx.run()
            assert e.value.code in (-3, -4), case
            continue
        got = gpu_outputs(msa_mod, fctx, data)
        assert got["metrics"] == {k: res[k] for k in ("processes", "total_songs", "total_words")}, case
        assert got["word_counts.csv"] == files["word_counts.csv"], case
        assert got["top_artists.csv"] == files["top_artists.csv"], case
        assert got["split"] == files["split"], case
