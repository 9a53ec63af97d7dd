#!/usr/bin/env python3
"""Step throughput (encode + full-loss decode, device-resident) with 1..S
objects in flight on S HIP streams.  usage: conc.py K R B [S ...]"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import Sets  # noqa: E402


def main():
    k, r, b = (int(x) for x in sys.argv[1:4])
    streams_list = [int(x) for x in sys.argv[4:]] or [1, 2, 3]
    assert leo.leo_init() == 0
    leo.set_async(True)
    sets = Sets(leo, torch, k, r, b, 16, "cuda")
    lib = leo.lib
    for ns in streams_list:
        streams = [torch.cuda.Stream() for _ in range(ns)]
        handles = [s.cuda_stream for s in streams]

        def run(steps):
            for s in range(steps):
                i = s % sets.n
                leo.set_stream(handles[s % ns])
                assert lib.leo_encode(b, k, r, sets.enc_wc, sets.p_orig[i], sets.p_encw[i]) == 0
                assert lib.leo_decode(b, k, r, sets.dec_wc, sets.p_null[i], sets.p_rec[i], sets.p_decw[i]) == 0

        run(50)
        torch.cuda.synchronize()
        steps = 400
        t0 = time.perf_counter()
        run(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{k}+{r} x {b}: {ns} stream(s): {dt / steps * 1e6:7.2f} us/step  {k * b * steps / dt / 1e9:8.2f} GB/s",
              flush=True)
    torch.cuda.synchronize()
    assert torch.equal(sets.dec_work[0][:k], sets.orig[0])


if __name__ == "__main__":
    main()
