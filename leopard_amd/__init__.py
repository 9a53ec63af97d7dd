"""leopard_amd -- MI355X-native Leopard-RS erasure coding, Python view of the C ABI.

The product is ``lib/libleopard_amd.so``, a drop-in replacement exporting the
reference's C interface (include/leopard.h; reference leopard.h:105-234).  This
module binds it with ctypes and mirrors the reference API one-to-one:

    leo_init()                        leopard.h:105-106
    leo_result_string(result)         leopard.h:127
    leo_encode_work_count(K, R)       leopard.h:143
    leo_encode(B, K, R, wc, orig, work)            leopard.h:180
    leo_decode_work_count(K, R)       leopard.h:202
    leo_decode(B, K, R, wc, orig, rec, work)       leopard.h:227

Buffers are passed as sequences of integer addresses (None for a lost piece),
exactly like the C arrays of pointers.  Addresses may be host memory or HIP
device memory (e.g. ``tensor.data_ptr()`` of a CUDA/HIP torch tensor).

Convenience wrappers for torch tensors (``encode``, ``decode``) sit on top and
go through the same C entry points.  There is no CPU fallback: if the shared
library is missing this module raises at import, and without a gfx950 GPU
``leo_init()`` returns ``LeopardResult.Platform``.
"""
from __future__ import annotations

import ctypes
import enum
import os
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LEOPARD_AMD_LIB") or os.path.join(_HERE, "lib", "libleopard_amd.so")
LEO_VERSION = 2

__all__ = [
    "LEO_VERSION", "LeopardResult", "leo_init", "leo_result_string", "leo_encode_work_count", "leo_encode",
    "leo_decode_work_count", "leo_decode", "leo_amd_encode_slice", "leo_amd_decode_slice", "leo_amd_encode_batch",
    "leo_amd_decode_batch", "register_host", "unregister_host", "set_fanout", "set_stream", "release_stream",
    "set_async", "set_device", "device_count", "table", "last_error", "encode", "decode", "LIB_PATH", "lib",
]


class LeopardResult(enum.IntEnum):
    """leopard.h:113-124"""
    Success = 0
    NeedMoreData = -1
    TooMuchData = -2
    InvalidSize = -3
    InvalidCounts = -4
    InvalidInput = -5
    Platform = -6
    CallInitialize = -7


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {_HERE}` (hipcc, gfx950)")
    try:  # share torch's HIP runtime when torch is around (same soname, one runtime per process)
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the C ABI
        pass
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    u, i, u64, vp = ctypes.c_uint, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p
    pp = ctypes.POINTER(vp)
    sig = {
        "leo_init_": (i, [i]),
        "leo_result_string": (ctypes.c_char_p, [i]),
        "leo_encode_work_count": (u, [u, u]),
        "leo_decode_work_count": (u, [u, u]),
        "leo_encode": (i, [u64, u, u, u, pp, pp]),
        "leo_decode": (i, [u64, u, u, u, pp, pp, pp]),
        "leo_amd_encode_slice": (i, [u64, u64, u64, u, u, u, pp, pp]),
        "leo_amd_decode_slice": (i, [u64, u64, u64, u, u, u, pp, pp, pp]),
        "leo_amd_encode_batch": (i, [u, u64, u, u, u, ctypes.POINTER(pp), ctypes.POINTER(pp)]),
        "leo_amd_decode_batch": (i, [u, u64, u, u, u, ctypes.POINTER(pp), ctypes.POINTER(pp), ctypes.POINTER(pp)]),
        "leo_amd_register_host": (i, [vp, u64]),
        "leo_amd_unregister_host": (i, [vp]),
        "leo_amd_set_stream": (None, [vp]),
        "leo_amd_set_async": (None, [i]),
        "leo_amd_set_device": (None, [i]),
        "leo_amd_set_fanout": (None, [i]),
        "leo_amd_release_stream": (None, [vp]),
        "leo_amd_device_count": (i, []),
        "leo_amd_table": (i, [i, i, vp, u]),
        "leo_amd_last_error": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("LEOPARD_AMD_LIB") and not hasattr(lib, name):
            continue  # an older experiment build (tools/ A/B runs) may lack later extensions
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def _ptrs(seq: Sequence[Optional[int]]):
    arr = (ctypes.c_void_p * max(len(seq), 1))()
    for k, p in enumerate(seq):
        arr[k] = None if p is None else int(p)
    return arr


def leo_init(version: int = LEO_VERSION) -> LeopardResult:
    return LeopardResult(lib.leo_init_(version))


def leo_result_string(result) -> str:
    return lib.leo_result_string(int(result)).decode()


def leo_encode_work_count(original_count: int, recovery_count: int) -> int:
    return lib.leo_encode_work_count(original_count, recovery_count)


def leo_decode_work_count(original_count: int, recovery_count: int) -> int:
    return lib.leo_decode_work_count(original_count, recovery_count)


def leo_encode(buffer_bytes, original_count, recovery_count, work_count, original_data, work_data) -> LeopardResult:
    od = None if original_data is None else _ptrs(original_data)
    wd = None if work_data is None else _ptrs(work_data)
    return LeopardResult(lib.leo_encode(buffer_bytes, original_count, recovery_count, work_count, od, wd))


def leo_decode(buffer_bytes, original_count, recovery_count, work_count, original_data, recovery_data,
               work_data) -> LeopardResult:
    od = None if original_data is None else _ptrs(original_data)
    rd = None if recovery_data is None else _ptrs(recovery_data)
    wd = None if work_data is None else _ptrs(work_data)
    return LeopardResult(lib.leo_decode(buffer_bytes, original_count, recovery_count, work_count, od, rd, wd))


def leo_amd_encode_slice(buffer_bytes, byte_offset, slice_bytes, original_count, recovery_count, work_count,
                         original_data, work_data) -> LeopardResult:
    return LeopardResult(lib.leo_amd_encode_slice(buffer_bytes, byte_offset, slice_bytes, original_count,
                                                  recovery_count, work_count, _ptrs(original_data),
                                                  _ptrs(work_data)))


def leo_amd_decode_slice(buffer_bytes, byte_offset, slice_bytes, original_count, recovery_count, work_count,
                         original_data, recovery_data, work_data) -> LeopardResult:
    return LeopardResult(lib.leo_amd_decode_slice(buffer_bytes, byte_offset, slice_bytes, original_count,
                                                  recovery_count, work_count, _ptrs(original_data),
                                                  _ptrs(recovery_data), _ptrs(work_data)))


def _ptr_arrays(seqs):
    """List of pointer sequences -> (void**)[count] (keeps the arrays alive in .keep)."""
    arrs = [_ptrs(q) for q in seqs]
    outer = (ctypes.POINTER(ctypes.c_void_p) * max(len(arrs), 1))(
        *[ctypes.cast(a, ctypes.POINTER(ctypes.c_void_p)) for a in arrs])
    outer.keep = arrs
    return outer


def _batch_lists(**lists):
    """Every per-object list of a batch call must name the same objects: the C
    side reads object_count entries of each outer array."""
    counts = {name: len(v) for name, v in lists.items()}
    if len(set(counts.values())) != 1:
        raise ValueError(f"batch lists differ in length: {counts}")
    return next(iter(counts.values()))


def leo_amd_encode_batch(buffer_bytes, original_count, recovery_count, work_count, original_data,
                         work_data) -> LeopardResult:
    """original_data / work_data: one pointer sequence per object (include/leopard_amd.h)."""
    count = _batch_lists(original_data=original_data, work_data=work_data)
    return LeopardResult(lib.leo_amd_encode_batch(count, buffer_bytes, original_count, recovery_count,
                                                  work_count, _ptr_arrays(original_data), _ptr_arrays(work_data)))


def leo_amd_decode_batch(buffer_bytes, original_count, recovery_count, work_count, original_data, recovery_data,
                         work_data) -> LeopardResult:
    count = _batch_lists(original_data=original_data, recovery_data=recovery_data, work_data=work_data)
    return LeopardResult(lib.leo_amd_decode_batch(count, buffer_bytes, original_count, recovery_count,
                                                  work_count, _ptr_arrays(original_data), _ptr_arrays(recovery_data),
                                                  _ptr_arrays(work_data)))


def register_host(ptr: int, nbytes: int) -> LeopardResult:
    """Pin + map a caller-owned host range (include/leopard_amd.h)."""
    return LeopardResult(lib.leo_amd_register_host(ctypes.c_void_p(ptr), nbytes))


def unregister_host(ptr: int) -> LeopardResult:
    return LeopardResult(lib.leo_amd_unregister_host(ctypes.c_void_p(ptr)))


def set_stream(stream_handle: Optional[int]) -> None:
    """HIP stream (integer handle, e.g. torch.cuda.current_stream().cuda_stream) for this thread."""
    lib.leo_amd_set_stream(None if not stream_handle else ctypes.c_void_p(stream_handle))


def release_stream(stream_handle: Optional[int]) -> None:
    """Free this thread's library scratch for a HIP stream (-1: every stream), after
    the work the library queued on it; call before destroying the stream."""
    lib.leo_amd_release_stream(None if not stream_handle else ctypes.c_void_p(stream_handle))


def set_async(enable: bool) -> None:
    lib.leo_amd_set_async(1 if enable else 0)


def set_device(device: int) -> None:
    lib.leo_amd_set_device(int(device))


def set_fanout(ranges: int) -> None:
    """Host-memory calls split their columns over `ranges` device workers (-1 = every device)."""
    lib.leo_amd_set_fanout(int(ranges))


def device_count() -> int:
    return lib.leo_amd_device_count()


def table(field: int, which: int):
    """Host-side tables (no GPU needed): which = 0 log, 1 exp, 2 FFT skew, 3 LogWalsh."""
    import numpy as np
    n = 1 << field
    out = np.zeros(n, dtype=np.uint16)
    got = lib.leo_amd_table(field, which, out.ctypes.data, n)
    if got < 0:
        raise ValueError(f"leo_amd_table({field}, {which}) -> {got}")
    return out[:got].copy()


def last_error() -> str:
    return lib.leo_amd_last_error().decode()


# ---------------------------------------------------------------- torch glue --

def _check(res, what):
    res = LeopardResult(res)
    if res != LeopardResult.Success:
        raise RuntimeError(f"{what}: {res.name} ({leo_result_string(res)}) {last_error()}")


def encode(original, recovery_count: int, work=None):
    """original: uint8 tensor [K, B] (device or host).  Returns work[:R] (recovery)."""
    import torch
    k, nbytes = original.shape
    wc = leo_encode_work_count(k, recovery_count)
    if work is None:
        work = torch.empty((max(wc, 1), nbytes), dtype=torch.uint8, device=original.device)
    res = leo_encode(nbytes, k, recovery_count, wc, [original[i].data_ptr() for i in range(k)],
                     [work[i].data_ptr() for i in range(wc)])
    _check(res, "leo_encode")
    return work[:recovery_count]


def decode(original, recovery, lost_originals, lost_recovery=(), work=None):
    """Rebuild lost originals.  original [K, B] / recovery [R, B] tensors; the
    indices listed as lost are passed as NULL.  Returns {i: work[i]}."""
    import torch
    k, nbytes = original.shape
    r = recovery.shape[0]
    wc = leo_decode_work_count(k, r)
    if work is None:
        work = torch.empty((wc, nbytes), dtype=torch.uint8, device=original.device)
    lo, lr = set(int(i) for i in lost_originals), set(int(i) for i in lost_recovery)
    res = leo_decode(nbytes, k, r, wc, [None if i in lo else original[i].data_ptr() for i in range(k)],
                     [None if i in lr else recovery[i].data_ptr() for i in range(r)],
                     [work[i].data_ptr() for i in range(wc)])
    _check(res, "leo_decode")
    return {i: work[i] for i in sorted(lo)}
