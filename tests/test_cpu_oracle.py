"""CPU tier: pin the oracle (our C restatement) to the reference.

* against the committed golden fixtures, which were produced by the reference
  library compiled from /root/reference (tests/golden/gen_golden.py);
* directly against that compiled reference when it is present here;
* the product library's host tables against the oracle's (no GPU needed).
"""
import os

import numpy as np
import pytest

import oracle_lib as ol

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _keys(prefix):
    with np.load(os.path.join(GOLDEN, "golden_small.npz")) as z:
        return sorted(k for k in z.files if k.startswith(prefix))


@pytest.mark.parametrize("key", _keys("enc_"))
def test_oracle_encode_vs_golden(key):
    k, r, b = (int(x) for x in key.split("_")[1:])
    if k * b > 4_000_000:
        pytest.skip("large for the scalar oracle")
    with np.load(os.path.join(GOLDEN, "golden_small.npz")) as z:
        expect = z[key]
    got = ol.oracle().encode(ol.pcg_bytes(2, 0, k, b), r)
    assert np.array_equal(got, expect)


@pytest.mark.parametrize("key", _keys("decout_"))
def test_oracle_decode_vs_golden(key):
    tag = "_".join(key.split("_")[1:])
    k, r, b, loss = (int(x) for x in tag.split("_"))
    with np.load(os.path.join(GOLDEN, "golden_small.npz")) as z:
        lo, lr, expect = z["declo_" + tag].tolist(), z["declr_" + tag].tolist(), z[key]
    got = ol.oracle().decode(ol.pcg_bytes(2, 1, k, b), ol.pcg_bytes(2, 2, r, b), lo, lr)
    for j, i in enumerate(lo):
        assert np.array_equal(got[i], expect[j])


def test_oracle_roundtrip_benchmark_pattern():
    k, r, b = 300, 100, 128
    data = ol.pcg_bytes(2, 0, k, b)
    rec = ol.oracle().encode(data, r)
    lo, lr = ol.benchmark_losses(k, r, 80, seed=2, trial=0, data_bytes=k * b)
    got = ol.oracle().decode(data, rec, lo, lr)
    for i in lo:
        assert np.array_equal(got[i], data[i])


@pytest.mark.skipif(ol.reference() is None, reason="reference not compiled here (make -C oracle ref)")
@pytest.mark.parametrize("k,r,b", [(2, 2, 64), (77, 31, 128), (128, 128, 64), (200, 56, 64), (129, 100, 64),
                                   (1000, 500, 64), (3000, 1, 64), (1, 1, 64)])
def test_oracle_vs_compiled_reference(k, r, b):
    rng = np.random.default_rng(k * 1000 + r)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    ref = ol.reference()
    assert np.array_equal(ol.oracle().encode(data, r), ref.encode(data, r))
    junk = rng.integers(0, 256, (r, b), dtype=np.uint8)
    loss = min(r, k)
    lo = sorted(rng.choice(k, loss, replace=False).tolist())
    lr = sorted(rng.choice(r, r - loss, replace=False).tolist())
    a = ol.oracle().decode(data, junk, lo, lr)
    e = ref.decode(data, junk, lo, lr)
    for i in lo:
        assert np.array_equal(a[i], e[i])


def test_pcg_matches_reference_generator():
    # first outputs of PCGRandom.Seed(2, 0) (tests/benchmark.cpp:134-156), scalar vs vectorised
    g = ol.PCGRandom(2, 0)
    scalar = [g.next() for _ in range(10000)]
    assert scalar == ol.pcg_stream(2, 0, 10000).tolist()


def test_shuffle_deck_is_permutation():
    for count in (1, 2, 5, 128, 200, 256, 257, 1000, 4001):
        deck = ol.shuffle_deck16(ol.PCGRandom(2, 0), count)
        assert sorted(deck) == list(range(count))


@pytest.mark.parametrize("field", [8, 16])
@pytest.mark.parametrize("which", [0, 1, 2, 3])
def test_library_tables_match_oracle(field, which):
    import leopard_amd
    got = leopard_amd.table(field, which)
    expect = ol.oracle_table(field == 16, which)
    assert np.array_equal(got, expect)
