"""GPU sweeps modelled on the reference's own test driver (tests/benchmark.cpp):

* exhaustive small codes, tests/benchmark.cpp:603-618: every K in [1, 256] and
  every R in [1, K] (all 32896 codes), loss = R.  The encoder output is
  compared with the CPU oracle byte for byte, and the decode of the benchmark's
  loss pattern (ShuffleDeck16, tests/benchmark.cpp:440-467) must return the
  originals.  Split by K range so that every test finishes in seconds.
* random codes, tests/benchmark.cpp:572-600: the reference driver's PCG-drawn
  (K, R, loss) for "small" (K <= 128) and "large" (K <= 32768) codes.

Buffers are 64 bytes (the reference's minimum) so that the oracle keeps up."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

B = 64


def _roundtrip(leo, data_d, data_np, k, r, loss, seed, trial):
    rec_d = leo.encode(data_d, r).clone()
    torch.cuda.synchronize()
    assert np.array_equal(rec_d.cpu().numpy(), ol.oracle().encode(data_np, r)), (k, r, "encode")
    lo, lr = ol.benchmark_losses(k, r, loss, seed=seed, trial=trial)
    got = leo.decode(data_d, rec_d, lo, lr)
    torch.cuda.synchronize()
    if lo:
        idx = torch.tensor(lo, device="cuda")
        assert torch.equal(torch.stack([got[i] for i in lo]), data_d.index_select(0, idx)), (k, r, loss)


K_RANGES = [(1, 64), (65, 96), (97, 128), (129, 150), (151, 170), (171, 190), (191, 208), (209, 224), (225, 240),
            (241, 256)]


@pytest.mark.parametrize("k0,k1", K_RANGES)
def test_exhaustive_small_codes(leo, k0, k1):
    """tests/benchmark.cpp:603-618: every code with k0 <= K <= k1, every R <= K."""
    pool = ol.pcg_bytes(3, 0, 256, B)
    pool_d = torch.from_numpy(pool).cuda()
    n = 0
    for k in range(k0, k1 + 1):
        for r in range(1, k + 1):
            _roundtrip(leo, pool_d[:k], pool[:k], k, r, r, seed=3, trial=k * 1000 + r)
            n += 1
    assert n == sum(k for k in range(k0, k1 + 1))


def _random_codes(max_k, count, seed):
    """(K, R, loss) as the reference driver draws them (tests/benchmark.cpp:575-599):
    K = Next() % max + 1, R = Next() % K + 1, loss = Next() % R + 1."""
    prng = ol.PCGRandom(seed, 8)
    out = []
    for _ in range(count):
        k = prng.next() % max_k + 1
        r = prng.next() % k + 1
        loss = prng.next() % r + 1
        out.append((k, r, loss))
    return out


@pytest.mark.parametrize("k,r,loss", _random_codes(128, 48, 2))
def test_random_small_codes(leo, k, r, loss):
    data = ol.pcg_bytes(5, k, k, B)
    _roundtrip(leo, torch.from_numpy(data).cuda(), data, k, r, loss, seed=5, trial=r)


@pytest.mark.parametrize("k,r,loss", _random_codes(32768, 6, 2))
def test_random_large_codes(leo, k, r, loss):
    data = ol.hash_bytes(k, k, B)
    _roundtrip(leo, torch.from_numpy(data).cuda(), data, k, r, loss, seed=7, trial=r)
