"""CPU tier for the multi-GPU path: column sharding across
ranks with no data-path collective.

Two gloo ranks each code only their own 64-byte-aligned column range of the
object (with the CPU oracle standing in for the per-rank device call, which
`-m gpu` tests cover through leo_amd_*_slice); the test then gathers the
shards (test-side only) and checks they equal coding the whole object.  Also
covers the shard arithmetic and the max-over-ranks timing helper that
bench.py uses for N > 1.
"""
import os
import socket

import numpy as np
import pytest

from leopard_amd.sharding import BLOCK, column_shards, max_over_ranks, shard_for_rank


@pytest.mark.parametrize("nbytes", [64, 128, 640, 65536, 64000])
@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_column_shards_cover_exactly(nbytes, parts):
    sh = column_shards(nbytes, parts)
    assert len(sh) == parts
    off = 0
    for o, n in sh:
        assert o == off and n % BLOCK == 0 and o % BLOCK == 0
        off += n
    assert off == nbytes
    sizes = [n for _, n in sh]
    assert max(sizes) - min(sizes) <= BLOCK
    assert [shard_for_rank(nbytes, p, parts) for p in range(parts)] == sh


def test_column_shards_rejects_unaligned():
    with pytest.raises(ValueError):
        column_shards(100, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# (K, R, B): GF(2^8) and GF(2^16) (K + R > 256), B splitting unevenly over 2 ranks
CASES = [(20, 10, 640), (128, 128, 1024), (300, 100, 320)]


def _rank_main(rank, world, port, results):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import oracle_lib as ol
        codec = ol.oracle()
        out = []
        for (k, r, b) in CASES:
            data = ol.pcg_bytes(5, 1, k, b)
            off, size = shard_for_rank(b, rank, world)
            rec_shard = codec.encode(np.ascontiguousarray(data[:, off:off + size]), r)
            lost = list(range(0, min(k, r), 2))
            full_rec = codec.encode(data, r)
            dec_shard = codec.decode(np.ascontiguousarray(data[:, off:off + size]),
                                     np.ascontiguousarray(full_rec[:, off:off + size]), lost, [])
            # test-side gather (the product path has no collective)
            parts = [None] * world
            dist.all_gather_object(parts, (off, rec_shard, dec_shard))
            if rank == 0:
                parts.sort(key=lambda x: x[0])
                rec = np.concatenate([p[1] for p in parts], axis=1)
                dec = {i: np.concatenate([p[2][i] for p in parts]) for i in lost}
                out.append(bool(np.array_equal(rec, full_rec))
                           and all(np.array_equal(dec[i], data[i]) for i in lost))
        elapsed = max_over_ranks(0.5 + rank)
        if rank == 0:
            results.put((out, elapsed))
    finally:
        dist.destroy_process_group()


def test_two_rank_column_sharding_matches_whole_object():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(rk, 2, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, elapsed = q.get(timeout=5)
    assert ok == [True] * len(CASES)
    assert elapsed == 1.5  # max over ranks of 0.5 + rank
