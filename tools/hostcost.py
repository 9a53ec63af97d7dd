#!/usr/bin/env python3
"""Host cost per leo_encode / leo_decode call (device pointers, async): calls
queued behind a spin kernel, so the GPU never back-pressures the host."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import Sets  # noqa: E402


def main():
    k, r, b = 128, 128, 65536
    assert leo.leo_init() == 0
    leo.set_async(True)
    st = torch.cuda.current_stream()
    leo.set_stream(st.cuda_stream)
    sets = Sets(leo, torch, k, r, b, 16, "cuda")
    lib = leo.lib
    enc = lambda i: lib.leo_encode(b, k, r, sets.enc_wc, sets.p_orig[i], sets.p_encw[i])
    dec = lambda i: lib.leo_decode(b, k, r, sets.dec_wc, sets.p_null[i], sets.p_rec[i], sets.p_decw[i])
    nop = lambda i: lib.leo_encode_work_count(k, r)
    setst = lambda i: leo.set_stream(st.cuda_stream)
    for name, fn in [("work_count (ctypes floor)", nop), ("set_stream", setst), ("encode", enc), ("decode", dec)]:
        for j in range(20):
            fn(j % 16)
        torch.cuda.synchronize()
        torch.cuda._sleep(200_000_000)
        n = 200
        t0 = time.perf_counter()
        for j in range(n):
            fn(j % 16)
        dt = (time.perf_counter() - t0) / n
        torch.cuda.synchronize()
        print(f"{name:28s} {dt * 1e6:7.2f} us/call", flush=True)


if __name__ == "__main__":
    main()
