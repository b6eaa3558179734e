"""GPU: the bucketed aggregation of the token pass's miss logs
(msa_k3.hip, msa_launch_miss_buckets), forced with MSA_MISS_BUCKETS=1 on
corpora (it is opt-in: measured slower than k_miss_agg).

The logs are bucketed by a second key hash, each bucket counted exactly in one
workgroup's LDS table and each distinct key inserted once (a claim and one
count add); entries that find that table full take the atomic insert.  The word
counts must equal the reference's (process_lyrics + the hash table,
/root/reference/src/parallel_spotify.c:350-394) on a high-cardinality corpus
whose tables all grow, on a Zipfian one (frequent words arrive as flushed
entries carrying counts), and on the CSV torture corpora."""
import pytest

from test_gpu_parity import check_against_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["highcard", "zipf", "torture"])
def test_miss_buckets_forced(msa_mod, tmp_path, monkeypatch, case):
    monkeypatch.setenv("MSA_MISS_BUCKETS", "1")
    if case == "highcard":
        data = msa_mod.gen_corpus(150_000, mode="highcard", seed=31)
    elif case == "zipf":
        data = msa_mod.gen_corpus(60_000, mode="zipf", seed=12)
    else:
        data = msa_mod.gen_corpus(1500, mode="torture", seed=3)
    with msa_mod.Context(0) as c:  # the library reads the setting when the context is made
        check_against_oracle(msa_mod, c, data, tmp_path, f"mb_{case}")
        # a second run on the same context: the tables, logs and buckets are reused
        check_against_oracle(msa_mod, c, data, tmp_path, f"mb_{case}_again")


def test_miss_buckets_auto_switch(msa_mod, tmp_path, monkeypatch):
    """The automatic choice with a low threshold: the first split aggregates
    with k_miss_agg, the next ones bucketed -- both byte-identical."""
    monkeypatch.setenv("MSA_MISS_BUCKETS", "2")
    monkeypatch.setenv("MSA_MISS_BUCKETS_MIN", "1000")
    data = msa_mod.gen_corpus(40_000, mode="highcard", seed=9)
    with msa_mod.Context(0) as c:
        for k in range(3):
            check_against_oracle(msa_mod, c, data, tmp_path, f"mb_auto{k}")
