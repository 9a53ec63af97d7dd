"""Column sharding of one encode/decode across ranks (one process per GPU).

Every Leopard operation is column-independent: byte j of a piece only meets
byte j of the other pieces (GF(2^8)), or the pair (j, j+32) of its 64-byte
block (GF(2^16) ALTMAP, reference LeopardFF16.cpp:315-332).  A call over
``buffer_bytes`` therefore splits into 64-byte-aligned column ranges that
ranks process independently with ``leo_amd_encode_slice`` /
``leo_amd_decode_slice`` -- no data-path collective.
The only cross-rank traffic is control: a barrier and the max of the elapsed
times, over whatever process group the caller provides (gloo or RCCL).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

BLOCK = 64  # leo_encode/leo_decode require buffer_bytes % 64 == 0 (reference leopard.h:158)


def column_shards(buffer_bytes: int, parts: int) -> List[Tuple[int, int]]:
    """Split [0, buffer_bytes) into `parts` contiguous 64-byte-aligned ranges
    (offset, size) differing by at most one block; empty ranges are possible
    when there are fewer blocks than parts."""
    if buffer_bytes % BLOCK:
        raise ValueError("buffer_bytes must be a multiple of 64")
    if parts < 1:
        raise ValueError("parts must be >= 1")
    blocks = buffer_bytes // BLOCK
    base, extra = divmod(blocks, parts)
    out, off = [], 0
    for p in range(parts):
        n = (base + (1 if p < extra else 0)) * BLOCK
        out.append((off, n))
        off += n
    return out


def shard_for_rank(buffer_bytes: int, rank: int, world: int) -> Tuple[int, int]:
    return column_shards(buffer_bytes, world)[rank]


def encode_shard(buffer_bytes: int, rank: int, world: int, original_count: int, recovery_count: int,
                 original_data: Sequence[int], work_data: Sequence[int]):
    """This rank's column range of leo_encode (device pointers of the whole pieces)."""
    import leopard_amd as leo
    off, size = shard_for_rank(buffer_bytes, rank, world)
    if size == 0:
        return leo.LeopardResult.Success
    wc = leo.leo_encode_work_count(original_count, recovery_count)
    return leo.leo_amd_encode_slice(buffer_bytes, off, size, original_count, recovery_count, wc,
                                    original_data, work_data)


def decode_shard(buffer_bytes: int, rank: int, world: int, original_count: int, recovery_count: int,
                 original_data: Sequence[Optional[int]], recovery_data: Sequence[Optional[int]],
                 work_data: Sequence[int]):
    """This rank's column range of leo_decode."""
    import leopard_amd as leo
    off, size = shard_for_rank(buffer_bytes, rank, world)
    if size == 0:
        return leo.LeopardResult.Success
    wc = leo.leo_decode_work_count(original_count, recovery_count)
    return leo.leo_amd_decode_slice(buffer_bytes, off, size, original_count, recovery_count, wc,
                                    original_data, recovery_data, work_data)


def max_over_ranks(value: float, group=None) -> float:
    """Max of a per-rank float (e.g. elapsed seconds) over the process group."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    device = "cpu"
    if dist.get_backend(group) == dist.Backend.NCCL:  # RCCL reduces device tensors only
        device = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
