#!/usr/bin/env python3
"""Host enqueue cost of leo_amd_encode_batch / decode_batch (slab-laid
objects, async mode): wall time of N back-to-back calls while a spin kernel
holds the stream, so no call waits for the GPU.  usage: batch_hostcost.py [K R B OBJ]"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import Sets  # noqa: E402

VP = ctypes.c_void_p
PP = ctypes.POINTER(VP)


def main():
    k, r, b, cnt = (int(x) for x in sys.argv[1:5]) if len(sys.argv) > 4 else (128, 128, 65536, 16)
    assert leo.leo_init() == 0
    leo.set_async(True)
    s = torch.cuda.current_stream()
    leo.set_stream(s.cuda_stream)
    sets = Sets(leo, torch, k, r, b, cnt, "cuda")
    lib = leo.lib
    mk = lambda arrs: (PP * len(arrs))(*[ctypes.cast(a, PP) for a in arrs])  # noqa: E731
    bo, bw = mk(sets.p_orig[:cnt]), mk(sets.p_encw[:cnt])
    bn, br, bd = mk(sets.p_null[:cnt]), mk(sets.p_rec[:cnt]), mk(sets.p_decw[:cnt])
    enc = lambda: lib.leo_amd_encode_batch(cnt, b, k, r, sets.enc_wc, bo, bw)  # noqa: E731
    dec = lambda: lib.leo_amd_decode_batch(cnt, b, k, r, sets.dec_wc, bn, br, bd)  # noqa: E731
    for fn in (enc, dec):
        for _ in range(5):
            assert fn() == 0, leo.last_error()
    torch.cuda.synchronize()
    n = 20
    for name, fn in (("encode_batch", enc), ("decode_batch", dec), ("encode_batch", enc)):
        torch.cuda._sleep(400_000_000)  # the stream stays busy while the host enqueues
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        dt = (time.perf_counter() - t0) / n
        torch.cuda.synchronize()
        print(f"{k}+{r}x{b} x{cnt} objects: {name} host enqueue {dt * 1e6:.1f} us per call", flush=True)


if __name__ == "__main__":
    main()
