"""Test-side access to the CPU checkers (TEST INFRASTRUCTURE ONLY).

* ``oracle/liboracle.so``        -- our plain-C restatement of Leopard's algorithm.
* ``oracle/_ref/libleopard_ref.so`` -- the reference library compiled from
  /root/reference by ``oracle/Makefile`` (present where it was built; it travels
  to the GPU box as a prebuilt .so).

Both expose Leopard's encode/decode calling convention (arrays of piece
pointers, leopard.h:180-234), so the same numpy helpers drive either.

Also restates the reference benchmark's data generator and loss pattern
(tests/benchmark.cpp:134-156 PCGRandom, :290-372 ShuffleDeck16, :440-467 losses)
so parity tests use exactly the reference's synthetic inputs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libleopard_ref.so")

_VP = ctypes.c_void_p


def _bind(lib, prefix):
    getattr(lib, prefix + "encode_work_count").restype = ctypes.c_uint
    getattr(lib, prefix + "encode_work_count").argtypes = [ctypes.c_uint, ctypes.c_uint]
    getattr(lib, prefix + "decode_work_count").restype = ctypes.c_uint
    getattr(lib, prefix + "decode_work_count").argtypes = [ctypes.c_uint, ctypes.c_uint]
    enc = getattr(lib, prefix + "encode")
    enc.restype = ctypes.c_int
    enc.argtypes = [ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                    ctypes.POINTER(_VP), ctypes.POINTER(_VP)]
    dec = getattr(lib, prefix + "decode")
    dec.restype = ctypes.c_int
    dec.argtypes = [ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                    ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.POINTER(_VP)]


class CpuCodec:
    """Uniform wrapper over the oracle or the compiled reference."""

    def __init__(self, path: str, prefix: str, init_name: str, init_args=()):
        self.path = path
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        self.prefix = prefix
        _bind(self.lib, prefix)
        init = getattr(self.lib, init_name)
        init.restype = ctypes.c_int
        rc = init(*init_args)
        if rc != 0:
            raise RuntimeError(f"{path}: init failed rc={rc}")

    def encode_work_count(self, k, r):
        return getattr(self.lib, self.prefix + "encode_work_count")(k, r)

    def decode_work_count(self, k, r):
        return getattr(self.lib, self.prefix + "decode_work_count")(k, r)

    def encode_raw(self, nbytes, k, r, work_count, orig_ptrs, work_ptrs):
        oa = (_VP * len(orig_ptrs))(*orig_ptrs)
        wa = (_VP * len(work_ptrs))(*work_ptrs)
        return getattr(self.lib, self.prefix + "encode")(nbytes, k, r, work_count, oa, wa)

    def decode_raw(self, nbytes, k, r, work_count, orig_ptrs, rec_ptrs, work_ptrs):
        oa = (_VP * len(orig_ptrs))(*orig_ptrs)
        ra = (_VP * len(rec_ptrs))(*rec_ptrs)
        wa = (_VP * len(work_ptrs))(*work_ptrs)
        return getattr(self.lib, self.prefix + "decode")(nbytes, k, r, work_count, oa, ra, wa)

    # ---- numpy conveniences -------------------------------------------------
    def encode(self, data: np.ndarray, r: int) -> np.ndarray:
        """data: uint8 [K, B] -> recovery uint8 [R, B]."""
        k, nbytes = data.shape
        data = np.ascontiguousarray(data)
        wc = self.encode_work_count(k, r)
        work = np.zeros((max(wc, 1), nbytes), dtype=np.uint8)
        orig = [data[i].ctypes.data for i in range(k)]
        wp = [work[i].ctypes.data for i in range(wc)]
        rc = self.encode_raw(nbytes, k, r, wc, orig, wp)
        if rc != 0:
            raise RuntimeError(f"encode rc={rc}")
        return work[:r].copy()

    def decode(self, data: np.ndarray, recovery: np.ndarray, lost_orig, lost_rec) -> dict:
        """Returns {i: uint8[B]} for each lost original i."""
        k, nbytes = data.shape
        r = recovery.shape[0]
        data = np.ascontiguousarray(data)
        recovery = np.ascontiguousarray(recovery)
        wc = self.decode_work_count(k, r)
        work = np.zeros((wc, nbytes), dtype=np.uint8)
        lo, lr = set(lost_orig), set(lost_rec)
        orig = [None if i in lo else data[i].ctypes.data for i in range(k)]
        rec = [None if i in lr else recovery[i].ctypes.data for i in range(r)]
        wp = [work[i].ctypes.data for i in range(wc)]
        rc = self.decode_raw(nbytes, k, r, wc, orig, rec, wp)
        if rc != 0:
            raise RuntimeError(f"decode rc={rc}")
        return {i: work[i].copy() for i in sorted(lo)}


def build_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), os.path.abspath(ORACLE_SO)])
    return ORACLE_SO


_oracle = None
_ref = None


def oracle() -> CpuCodec:
    global _oracle
    if _oracle is None:
        build_oracle()
        _oracle = CpuCodec(ORACLE_SO, "orc_", "orc_init")
        _oracle.lib.orc_table.restype = ctypes.c_int
        _oracle.lib.orc_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return _oracle


def oracle_table(ff16: bool, which: int) -> np.ndarray:
    """which: 0 log, 1 exp, 2 skew, 3 logwalsh."""
    o = oracle()
    n = (65536 if ff16 else 256) - (1 if which == 2 else 0)
    out = np.zeros(n, dtype=np.uint16)
    got = o.lib.orc_table(int(ff16), which, out.ctypes.data)
    assert got == n
    return out


def reference() -> CpuCodec | None:
    """The compiled reference, or None when it was not built (never built on the GPU box)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = CpuCodec(REF_SO, "leo_", "leo_init_", (2,))
    return _ref


# ---------------------------------------------------------------------------
# The reference benchmark's synthetic data (tests/benchmark.cpp)

class PCGRandom:
    """PCG32 exactly as tests/benchmark.cpp:134-156."""
    M = 6364136223846793005
    MASK = (1 << 64) - 1

    def __init__(self, y: int, x: int = 0):
        self.state = 0
        self.inc = ((y << 1) | 1) & self.MASK
        self.next()
        self.state = (self.state + x) & self.MASK
        self.next()

    def next(self) -> int:
        old = self.state
        self.state = (old * self.M + self.inc) & self.MASK
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF


def pcg_stream(seed: int, trial: int, n: int) -> np.ndarray:
    """n successive PCG outputs (uint32) -- vectorised by jumping is not needed
    at test sizes; uses an LCG skip-ahead for speed on large n."""
    g = PCGRandom(seed, trial)
    # LCG advance in numpy: compute successive states with uint64 wraparound.
    out = np.empty(n, dtype=np.uint32)
    state = np.uint64(g.state)
    inc = np.uint64(g.inc)
    mult = np.uint64(PCGRandom.M)
    # Precompute states in blocks using the affine-map power trick.
    block = 4096
    a_pows = np.empty(block, dtype=np.uint64)
    c_pows = np.empty(block, dtype=np.uint64)
    a, c = np.uint64(1), np.uint64(0)
    with np.errstate(over="ignore"):
        for i in range(block):
            a_pows[i], c_pows[i] = a, c
            a, c = a * mult, c * mult + inc
        a_blk, c_blk = a, c
        pos = 0
        while pos < n:
            cnt = min(block, n - pos)
            states = a_pows[:cnt] * state + c_pows[:cnt]
            xs = (((states >> np.uint64(18)) ^ states) >> np.uint64(27)) & np.uint64(0xFFFFFFFF)
            rot = (states >> np.uint64(59)).astype(np.uint64)
            xs32 = xs.astype(np.uint64)
            val = ((xs32 >> rot) | (xs32 << ((np.uint64(32) - rot) & np.uint64(31)))) & np.uint64(0xFFFFFFFF)
            out[pos:pos + cnt] = val.astype(np.uint32)
            state = a_blk * state + c_blk
            pos += cnt
    return out


def pcg_bytes(seed: int, trial: int, pieces: int, nbytes: int) -> np.ndarray:
    """uint8 [pieces, nbytes]: one PCG Next() per byte, low 8 bits, pieces in order
    (the convention of SURVEY.md section 8(c) KATs)."""
    return (pcg_stream(seed, trial, pieces * nbytes) & 0xFF).astype(np.uint8).reshape(pieces, nbytes)


def shuffle_deck16(prng: PCGRandom, count: int):
    """tests/benchmark.cpp:290-372 (including its unrolled switch semantics)."""
    deck = [0] * max(count, 1)
    deck[0] = 0
    ii = 1
    if count <= 256:
        while True:
            rv = prng.next()
            rem = count - ii
            if rem >= 4:
                for sh in (0, 8, 16, 24):
                    jj = ((rv >> sh) & 0xFF) % ii
                    deck[ii] = deck[jj]
                    deck[jj] = ii
                    ii += 1
                continue
            shifts = {3: (0, 8, 16), 2: (8, 16), 1: (16,), 0: ()}[rem]
            for sh in shifts:
                jj = ((rv >> sh) & 0xFF) % ii
                deck[ii] = deck[jj]
                deck[jj] = ii
                ii += 1
            return deck[:count]
    while True:
        rv = prng.next()
        rem = count - ii
        if rem >= 2:
            for sh in (0, 16):
                jj = ((rv >> sh) & 0xFFFF) % ii
                deck[ii] = deck[jj]
                deck[jj] = ii
                ii += 1
            continue
        if rem == 1:
            jj = (rv & 0xFFFF) % ii
            deck[ii] = deck[jj]
            deck[jj] = ii
        return deck[:count]


def benchmark_losses(k: int, r: int, loss_count: int, seed: int = 2, trial: int = 0, data_bytes: int | None = None):
    """The loss pattern of tests/benchmark.cpp:440-467: the PCG stream continues
    after data generation; originals lost = first loss_count of ShuffleDeck16(K),
    recoveries lost = first (R - loss_count) of ShuffleDeck16(R).

    data_bytes: number of PCG draws consumed by data generation before the
    shuffles (pieces*bytes for our raw fill).  Pass 0 to start fresh."""
    prng = PCGRandom(seed, trial)
    if data_bytes:
        # advance by data_bytes draws
        st = pcg_advance(prng, data_bytes)
    lost_o = shuffle_deck16(prng, k)[:loss_count]
    lost_r = shuffle_deck16(prng, r)[: r - loss_count]
    return sorted(lost_o), sorted(lost_r)


def pcg_advance(prng: PCGRandom, n: int):
    """Advance an LCG by n steps in O(log n)."""
    M = PCGRandom.MASK
    acc_mult, acc_plus = 1, 0
    cur_mult, cur_plus = PCGRandom.M, prng.inc
    while n > 0:
        if n & 1:
            acc_mult = (acc_mult * cur_mult) & M
            acc_plus = (acc_plus * cur_mult + cur_plus) & M
        cur_plus = ((cur_mult + 1) * cur_plus) & M
        cur_mult = (cur_mult * cur_mult) & M
        n >>= 1
    prng.state = (acc_mult * prng.state + acc_plus) & M
    return prng


def fnv1a64(buf) -> str:
    """FNV-1a 64 over bytes (vectorised in chunks via Python int math)."""
    h = 0xCBF29CE484222325
    p = 0x100000001B3
    mv = memoryview(np.ascontiguousarray(buf).reshape(-1).view(np.uint8))
    for b in mv.tobytes():
        h ^= b
        h = (h * p) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


# ---------------------------------------------------------------------------
# Counter-hash fill: cheap to reproduce on the GPU (torch) and on the CPU
# (numpy) for the multi-GB BASELINE shapes.  byte (p, j) depends only on the
# global index g = p * B + j and the seed.

def _hash32_np(g: np.ndarray, seed: int) -> np.ndarray:
    x = (g.astype(np.uint64) * np.uint64(2654435761) + np.uint64(seed * 0x632BE5AB)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return (x & np.uint64(0xFF)).astype(np.uint8)


def hash_bytes(seed: int, pieces: int, nbytes: int) -> np.ndarray:
    out = np.empty((pieces, nbytes), dtype=np.uint8)
    flat = out.reshape(-1)
    step = 1 << 24
    for s in range(0, flat.size, step):
        e = min(flat.size, s + step)
        flat[s:e] = _hash32_np(np.arange(s, e, dtype=np.uint64), seed)
    return out


def hash_bytes_torch(seed: int, pieces: int, nbytes: int, device):
    """Same bytes as hash_bytes(), generated on `device` (int64 arithmetic,
    masked to 32 bits after every multiply, so wraparound does not matter)."""
    import torch
    out = torch.empty((pieces, nbytes), dtype=torch.uint8, device=device)
    flat = out.view(-1)
    step = 1 << 26
    M = 0xFFFFFFFF
    for s in range(0, flat.numel(), step):
        e = min(flat.numel(), s + step)
        g = torch.arange(s, e, dtype=torch.int64, device=device)
        x = (g * 2654435761 + seed * 0x632BE5AB) & M
        x = x ^ (x >> 16)
        x = (x * 0x85EBCA6B) & M
        x = x ^ (x >> 13)
        x = (x * 0xC2B2AE35) & M
        x = x ^ (x >> 16)
        flat[s:e] = (x & 0xFF).to(torch.uint8)
    return out
