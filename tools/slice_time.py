#!/usr/bin/env python3
"""Per-rank cost of the configs[4] column split on one GPU (performance
diagnostics only): encode + full-loss decode of 32768 + 32768 pieces, one
column shard of B / N bytes, (a) as pieces of that width (what a bench.py rank
allocates since round 6) and (b) as a slice of 64 KiB pieces (the round-5
layout), against the whole object.  HIP events around back-to-back calls.
usage: slice_time.py [N ...]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import hash_fill_cuda, ptrs  # noqa: E402

VP = ctypes.c_void_p


def main():
    k = r = 32768
    b = 65536
    ns = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    assert leo.leo_init() == 0
    st = torch.cuda.current_stream()
    leo.set_stream(st.cuda_stream)
    leo.set_async(True)
    lib = leo.lib
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    pn = (VP * k)()

    def run(width, pitch, off, reps=4):
        data = hash_fill_cuda(torch, 7, k, pitch, "cuda")
        work = torch.empty((wc, pitch), dtype=torch.uint8, device="cuda")
        dwork = torch.empty((dwc, pitch), dtype=torch.uint8, device="cuda")
        po, pw, pr, pd = ptrs(data), ptrs(work), ptrs(work, r), ptrs(dwork)

        def step():
            assert lib.leo_amd_encode_slice(pitch, off, width, k, r, wc, po, pw) == 0, leo.last_error()
            assert lib.leo_amd_decode_slice(pitch, off, width, k, r, dwc, pn, pr, pd) == 0, leo.last_error()
        step()
        torch.cuda.synchronize()
        ok = bool(torch.equal(dwork[:k, off:off + width], data[:, off:off + width]))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            step()
        e1.record(st)
        e1.synchronize()
        del data, work, dwork
        torch.cuda.empty_cache()
        return e0.elapsed_time(e1) / reps, ok

    whole, ok = run(b, b, 0)
    print(f"whole object: {whole:.3f} ms per encode + decode (roundtrip_ok={ok})", flush=True)
    for n in ns:
        w = b // n
        own, ok1 = run(w, w, 0)
        sl, ok2 = run(w, b, 0)
        print(f"N={n}: shard of {w} B: own {w}-B pieces {own:.3f} ms ({whole / own / n:.3f} of ideal 1/N), "
              f"slice of 64 KiB pieces {sl:.3f} ms ({whole / sl / n:.3f}); roundtrip_ok={ok1 and ok2}", flush=True)


if __name__ == "__main__":
    main()
