#!/usr/bin/env python3
"""Benchmark: device-resident Leopard-RS encode + decode through the C ABI.

Metric (BASELINE.json): device-resident encode+decode GB/s of input bytes.
One *step* = one leo_encode of a batch plus one worst-case leo_decode of the
same batch (every original lost, decoded from the R recovery pieces), both
called through the drop-in C ABI with device pointers, in async mode.  Step s
runs on HIP stream s % S (--streams, default 3 objects in flight: a single
64 KiB-piece call fills each CU with one workgroup, and concurrent objects
fill the phases where one call waits on memory or barriers); the same steps on
one stream are reported as "serial".  value = (input bytes K*B per step,
summed over ranks) / time.

Workload (configs[1]): 128 originals + 128 recovery pieces of 65536 bytes,
GF(2^8).  Every rank owns its own 64 KiB-per-piece column shard of a larger
object (64-byte column blocks never interact, so no collective is needed);
per-GPU work is fixed as N grows -> "scaling": "weak".  To defeat the 256 MiB
Infinity Cache the step walks over >= 16 distinct buffer sets (> 2x MALL).

Roofline: the dominant kernel is timed alone with HIP events on the stream it
runs on (back-to-back calls queued behind a spin kernel); achieved =
algorithmic bytes per launch ((K_surv + lost) * B for decode, (K + R) * B for
encode) / mean launch duration, against the 8 TB/s HBM3E peak.
traffic = HBM bytes per launch from the committed rocprofv3 PMC pass
(tools/pmc_traffic.py), when present for this workload.

cpu_baseline: the reference library compiled from its sources
(oracle/_ref/libleopard_ref.so, AVX2, single thread -- FF8 has no OpenMP) timed
on this host on a bounded sample of the same workload; falls back to our
scalar oracle port if the reference build is absent.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--R", type=int, default=128)
    ap.add_argument("--bytes", type=int, default=65536)
    ap.add_argument("--sets", type=int, default=0, help="buffer sets rotated (0 = enough for >512 MiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the GF(2^16) configs (32768+32768 and 1000+200 x 64 KiB)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory (PCIe-inclusive) rate")
    ap.add_argument("--streams", type=int, default=3,
                    help="objects in flight: step s runs on HIP stream s %% S (1 = strictly serial steps)")
    return ap.parse_args()


def hash_fill_cuda(torch, seed, pieces, nbytes, device):
    """Synthetic piece bytes on the device: a 32-bit counter hash of the global
    byte index (same bytes as tests/oracle_lib.hash_bytes)."""
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


class Sets:
    """Pre-built pointer arrays (ctypes) for rotating buffer sets."""

    def __init__(self, leo, torch, k, r, nbytes, nsets, device):
        self.k, self.r, self.nbytes = k, r, nbytes
        self.enc_wc = leo.leo_encode_work_count(k, r)
        self.dec_wc = leo.leo_decode_work_count(k, r)
        VP = ctypes.c_void_p
        self.orig, self.rec, self.enc_work, self.dec_work = [], [], [], []
        self.p_orig, self.p_encw, self.p_null, self.p_rec, self.p_decw = [], [], [], [], []
        for s in range(nsets):
            o = hash_fill_cuda(torch, 7 + s, k, nbytes, device)
            ew = torch.zeros((self.enc_wc, nbytes), dtype=torch.uint8, device=device)
            dw = torch.zeros((self.dec_wc, nbytes), dtype=torch.uint8, device=device)
            self.orig.append(o)
            self.enc_work.append(ew)
            self.dec_work.append(dw)
            self.p_orig.append((VP * k)(*[o[i].data_ptr() for i in range(k)]))
            self.p_encw.append((VP * self.enc_wc)(*[ew[i].data_ptr() for i in range(self.enc_wc)]))
            self.p_null.append((VP * k)())  # every original lost
            self.p_rec.append((VP * r)(*[ew[i].data_ptr() for i in range(r)]))
            self.p_decw.append((VP * self.dec_wc)(*[dw[i].data_ptr() for i in range(self.dec_wc)]))
        self.n = nsets


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")  # control plane only (barrier, max-time); no data-path collective
    # one process per GPU; more ranks than GPUs (a functional rehearsal on a
    # smaller box) share devices round-robin
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)

    import leopard_amd as leo
    from leopard_amd.sharding import max_over_ranks
    assert leo.leo_init() == 0, leo.last_error()
    lib = leo.lib
    stream = torch.cuda.current_stream(device)
    leo.set_stream(stream.cuda_stream)
    leo.set_async(True)

    k, r, nbytes = args.K, args.R, args.bytes
    per_set = (k + leo.leo_encode_work_count(k, r) + leo.leo_decode_work_count(k, r)) * nbytes
    nsets = args.sets or max(16, -(-(512 << 20) // per_set))
    sets = Sets(leo, torch, k, r, nbytes, nsets, device)
    torch.cuda.synchronize()

    def enc(i):
        return lib.leo_encode(nbytes, k, r, sets.enc_wc, sets.p_orig[i], sets.p_encw[i])

    def dec(i):
        return lib.leo_decode(nbytes, k, r, sets.dec_wc, sets.p_null[i], sets.p_rec[i], sets.p_decw[i])

    # correctness gate before timing: a decode must reproduce the originals
    assert enc(0) == 0 and dec(0) == 0, leo.last_error()
    torch.cuda.synchronize()
    assert torch.equal(sets.dec_work[0][:k], sets.orig[0]), "decode mismatch"
    for i in range(sets.n):
        assert enc(i) == 0
    torch.cuda.synchronize()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    # Objects in flight: step s (encode of buffer set i, then the decode of its
    # recovery pieces) runs on stream s % S, so up to S independent objects are
    # coded concurrently -- how a storage node keeps the GPU busy with stripes
    # whose single calls are too small to fill 256 CUs.  Steps on one stream
    # stay ordered; buffer sets rotate over >= 16 sets, so concurrent steps
    # never share buffers.
    streams = [torch.cuda.Stream(device) for _ in range(max(1, args.streams))]

    def run_steps(nsteps, nstreams):
        for s in range(nsteps):
            i = s % sets.n
            leo.set_stream(streams[s % nstreams].cuda_stream)
            if enc(i) != 0 or dec(i) != 0:
                raise RuntimeError(leo.last_error())

    def timed(nstreams):
        run_steps(args.warmup, nstreams)
        barrier()
        t0 = time.perf_counter()
        run_steps(args.steps, nstreams)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        el = max_over_ranks(t1 - t0)
        if world > 1:
            barrier()
        return el

    elapsed = timed(len(streams))
    elapsed_serial = timed(1) if len(streams) > 1 else elapsed
    leo.set_stream(stream.cuda_stream)

    # Per-launch kernel duration with HIP events on the launch stream: a spin
    # kernel holds the stream while the host enqueues n back-to-back calls (one
    # kernel each on the FF8 path) between one event pair, so the pair holds
    # only GPU time; back-to-back kernels start as the previous one ends
    # (rocprofv3 trace: median gap 0), so time / n is the mean launch duration.
    def time_calls(fn, n=100):
        for j in range(10):
            fn(j % sets.n)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(50_000_000)
        e0.record(stream)
        for j in range(n):
            fn(j % sets.n)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / n

    t_enc = time_calls(enc)
    t_dec = time_calls(dec)
    in_bytes = k * nbytes
    algo_enc = (k + r) * nbytes
    algo_dec = (r + k) * nbytes  # R surviving pieces read + K lost originals written (full loss)
    dominant = ("decode", algo_dec, t_dec) if t_dec >= t_enc else ("encode", algo_enc, t_enc)

    secondary = None
    if not args.no_secondary and rank == 0:
        secondary = [run_secondary(leo, torch, device, kk, rr, ll) for kk, rr, ll in
                     ((32768, 32768, 32768), (1000, 200, 200))]
    host = host_e2e(leo, k, r, nbytes) if rank == 0 and not args.no_host else None

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(k, r, nbytes, args.cpu_seconds)

    traffic = pmc_traffic(dominant[0], k, r, nbytes)
    if rank == 0:
        value = world * in_bytes * args.steps / elapsed / 1e9
        achieved = dominant[1] / dominant[2] / 1e9
        out = {
            "metric": "device-resident encode+decode GB/s (input bytes/s) at 128+128 and 32768+32768 pieces",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-hash bytes on device)",
            "config": {"workload": f"{k}+{r} x {nbytes} B pieces, GF(2^8), encode + full-loss decode per step, "
                                   f"device-resident, {sets.n} rotating buffer sets, "
                                   f"{len(streams)} objects in flight",
                       "original_count": k, "recovery_count": r, "buffer_bytes": nbytes, "losses": k,
                       "field": "FF8" if leo.leo_decode_work_count(k, r) <= 256 else "FF16",
                       "objects_in_flight": len(streams),
                       "sharding": "64-byte column blocks per rank, no collective"},
            "serial": {"value": round(world * in_bytes * args.steps / elapsed_serial / 1e9, 3),
                       "ms_per_step": round(elapsed_serial / args.steps * 1e3, 4),
                       "note": "same steps, one stream (each step waits for the previous)"},
            "encode_GBps": round(in_bytes / t_enc / 1e9, 3),
            "decode_GBps": round(in_bytes / t_dec / 1e9, 3),
            "encode_us": round(t_enc * 1e6, 3),
            "decode_us": round(t_dec * 1e6, 3),
            "roofline": {"bound": "hbm", "kernel": dominant[0], "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic.get("bytes"), "traffic_source": traffic.get("source"),
                         "algorithmic_bytes_per_launch": dominant[1]},
            "cpu_baseline": cpu,
            "host_e2e": host,
        }
        if secondary:
            out["secondary"] = secondary
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_secondary(leo, torch, device, k, r, loss):
    """GF(2^16) configs of BASELINE.json (configs[3], configs[2]) at 64 KiB:
    encode, then decode with `loss` originals lost (the benchmark's
    ShuffleDeck16 pattern, tests/benchmark.cpp:440-467) -- a few calls each."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as ol
    nbytes = 65536
    lib = leo.lib
    VP = ctypes.c_void_p
    o = hash_fill_cuda(torch, 7, k, nbytes, device)
    ew = torch.empty((leo.leo_encode_work_count(k, r), nbytes), dtype=torch.uint8, device=device)
    dw = torch.empty((leo.leo_decode_work_count(k, r), nbytes), dtype=torch.uint8, device=device)
    lo, lr = ol.benchmark_losses(k, r, loss, seed=2, trial=0)
    los, lrs = set(lo), set(lr)
    po = (VP * k)(*[o[i].data_ptr() for i in range(k)])
    pe = (VP * ew.shape[0])(*[ew[i].data_ptr() for i in range(ew.shape[0])])
    pn = (VP * k)(*[None if i in los else o[i].data_ptr() for i in range(k)])
    pr = (VP * r)(*[None if i in lrs else ew[i].data_ptr() for i in range(r)])
    pd = (VP * dw.shape[0])(*[dw[i].data_ptr() for i in range(dw.shape[0])])
    s = torch.cuda.current_stream(device)
    leo.set_stream(s.cuda_stream)

    def t(fn, n=3):
        assert fn() == 0, leo.last_error()
        s.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(n):
            assert fn() == 0, leo.last_error()
        b.record(s)
        b.synchronize()
        return a.elapsed_time(b) / 1e3 / n

    te = t(lambda: lib.leo_encode(nbytes, k, r, ew.shape[0], po, pe))
    td = t(lambda: lib.leo_decode(nbytes, k, r, dw.shape[0], pn, pr, pd))
    idx = torch.tensor(lo, device=device)
    ok = bool(torch.equal(dw.index_select(0, idx), o.index_select(0, idx)))
    inb = k * nbytes
    res = {"workload": f"{k}+{r} x {nbytes} B, GF(2^16), {loss} originals lost", "encode_GBps": round(inb / te / 1e9, 3),
           "decode_GBps": round(inb / td / 1e9, 3), "encode_decode_GBps": round(inb / (te + td) / 1e9, 3),
           "encode_ms": round(te * 1e3, 3), "decode_ms": round(td * 1e3, 3), "roundtrip_ok": ok}
    del o, ew, dw
    torch.cuda.empty_cache()
    return res


def host_e2e(leo, k, r, nbytes, steps=20):
    """PCIe-inclusive rate: the same encode + full-loss decode step through the
    C ABI with caller-owned pageable host buffers (the reference's contract).
    The library stages them through its pinned two-slot ring.  Not `value`."""
    import numpy as np
    data = np.frombuffer(np.random.default_rng(7).bytes(k * nbytes), dtype=np.uint8).reshape(k, nbytes)
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    work = np.zeros((wc, nbytes), dtype=np.uint8)
    dwork = np.zeros((dwc, nbytes), dtype=np.uint8)
    po = [data[i].ctypes.data for i in range(k)]
    pe = [work[i].ctypes.data for i in range(wc)]
    pr = [work[i].ctypes.data for i in range(r)]
    pd = [dwork[i].ctypes.data for i in range(dwc)]
    lost = [None] * k

    def step():
        assert leo.leo_encode(nbytes, k, r, wc, po, pe) == 0, leo.last_error()
        assert leo.leo_decode(nbytes, k, r, dwc, lost, pr, pd) == 0, leo.last_error()

    step()
    t0 = time.perf_counter()
    t_enc = 0.0
    for _ in range(steps):
        a = time.perf_counter()
        assert leo.leo_encode(nbytes, k, r, wc, po, pe) == 0, leo.last_error()
        t_enc += time.perf_counter() - a
        assert leo.leo_decode(nbytes, k, r, dwc, lost, pr, pd) == 0, leo.last_error()
    dt = time.perf_counter() - t0
    ok = bool(np.array_equal(dwork[:k], data))
    inb = k * nbytes
    return {"value": round(inb * steps / dt / 1e9, 3), "unit": "GB/s", "encode_GBps": round(inb * steps / t_enc / 1e9, 3),
            "decode_GBps": round(inb * steps / (dt - t_enc) / 1e9, 3), "roundtrip_ok": ok,
            "sample": f"{steps} steps, pageable numpy buffers, H2D + kernels + D2H per call"}


def pmc_traffic(kernel, k, r, nbytes):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (tools/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md HBM
    section), when one exists for this workload; else None."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_traffic.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        e = d.get("workloads", {}).get(f"{k}+{r}x{nbytes}", {}).get(kernel)
        if e:
            return {"bytes": e["hbm_bytes_per_launch"], "source": os.path.relpath(path, REPO)}
    return {}


def cpu_baseline(k, r, nbytes, seconds):
    """Reference AVX2 library (or our scalar port) on the host, 1 thread."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as ol
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    codec, kind = ol.reference(), "reference"
    if codec is None:
        codec, kind = ol.oracle(), "port"
    data = ol.hash_bytes(7, k, nbytes)
    wc_e = codec.encode_work_count(k, r)
    wc_d = codec.decode_work_count(k, r)
    work = np.zeros((wc_e, nbytes), dtype=np.uint8)
    dwork = np.zeros((wc_d, nbytes), dtype=np.uint8)
    po = [data[i].ctypes.data for i in range(k)]
    pe = [work[i].ctypes.data for i in range(wc_e)]
    pn = [None] * k
    pr = [work[i].ctypes.data for i in range(r)]
    pd = [dwork[i].ctypes.data for i in range(wc_d)]
    # warm (first touch)
    assert codec.encode_raw(nbytes, k, r, wc_e, po, pe) == 0
    assert codec.decode_raw(nbytes, k, r, wc_d, pn, pr, pd) == 0
    t_enc = t_dec = 0.0
    steps = 0
    start = time.perf_counter()
    while steps < 3 or time.perf_counter() - start < seconds:
        a = time.perf_counter()
        codec.encode_raw(nbytes, k, r, wc_e, po, pe)
        b = time.perf_counter()
        codec.decode_raw(nbytes, k, r, wc_d, pn, pr, pd)
        c = time.perf_counter()
        t_enc += b - a
        t_dec += c - b
        steps += 1
    assert np.array_equal(dwork[:k], data)
    inb = k * nbytes
    return {"value": round(inb * steps / (t_enc + t_dec) / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
            "sample": f"{steps} encode+decode steps of {k}+{r} x {nbytes} B (full loss), warm buffers, "
                      f"{t_enc + t_dec:.1f} s; encode {inb * steps / t_enc / 1e9:.3f} GB/s, "
                      f"decode {inb * steps / t_dec / 1e9:.3f} GB/s"}


if __name__ == "__main__":
    main()
