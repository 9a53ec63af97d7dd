#!/usr/bin/env python3
"""Quick per-call timing of leo_encode / leo_decode (device pointers, async,
back-to-back on one stream, HIP events).  usage: kbench.py [K R B ...]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import hash_fill_cuda  # noqa: E402


def run(k, r, b, sets=int(os.environ.get('KB_SETS', '16')), n=int(os.environ.get('KB_N', '100')),
        warm=int(os.environ.get('KB_WARM', '300'))):
    VP = ctypes.c_void_p
    lib = leo.lib
    ewc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    S = []
    for s in range(sets):
        o = hash_fill_cuda(torch, 7 + s, k, b, "cuda")
        ew = torch.zeros((ewc, b), dtype=torch.uint8, device="cuda")
        dw = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
        S.append((o, ew, dw, (VP * k)(*[o[i].data_ptr() for i in range(k)]),
                  (VP * ewc)(*[ew[i].data_ptr() for i in range(ewc)]),
                  (VP * k)(*([None] * min(k, r) + [o[i].data_ptr() for i in range(min(k, r), k)])),
                  (VP * r)(*[ew[i].data_ptr() for i in range(r)]), (VP * dwc)(*[dw[i].data_ptr() for i in range(dwc)])))
    enc = lambda i: lib.leo_encode(b, k, r, ewc, S[i][3], S[i][4])
    dec = lambda i: lib.leo_decode(b, k, r, dwc, S[i][5], S[i][6], S[i][7])
    for i in range(sets):
        assert enc(i) == 0, leo.last_error()
    torch.cuda.synchronize()
    rc = dec(0)
    torch.cuda.synchronize()
    lost = min(k, r)  # the first min(K, R) originals are lost
    ok = rc == 0 and torch.equal(S[0][2][:lost], S[0][0][:lost])
    st = torch.cuda.current_stream()

    def t(fn):
        for j in range(warm):
            fn(j % sets)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for j in range(n):
            fn(j % sets)
        z.record(st)
        z.synchronize()
        return a.elapsed_time(z) / n * 1e3

    te, td = t(enc), t(dec)
    print(f"{k}+{r} x {b}: encode {te:8.2f} us ({k*b/te/1e3:7.1f} GB/s in, {(k+r)*b/te/1e3:7.1f} GB/s algo)  "
          f"decode {td:8.2f} us ({k*b/td/1e3:7.1f} GB/s in)  roundtrip_ok={ok}", flush=True)


def main():
    assert leo.leo_init() == 0
    leo.set_stream(torch.cuda.current_stream().cuda_stream)
    leo.set_async(True)
    args = [int(x) for x in sys.argv[1:]] or [128, 128, 65536]
    for i in range(0, len(args), 3):
        run(*args[i:i + 3])


if __name__ == "__main__":
    main()
