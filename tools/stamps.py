#!/usr/bin/env python3
"""Phase timeline of the FF8 kernels from an LAMD_STAMPS build (diagnostics only).

usage: LEOPARD_AMD_LIB=leopard_amd/ablate/stamps/libleopard_amd.so python tools/stamps.py K R B
Prints, per stamp index, min / median / max over waves of (stamp - earliest entry) in us
(s_memrealtime, 100 MHz), for one encode and one full-loss decode."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import hash_fill_cuda  # noqa: E402


def show(name, buf, nwaves, nst):
    t = buf[: nwaves * 8].view(nwaves, 8)[:, :nst].cpu().double()
    t0 = t[:, 0].min()
    print(name)
    for k in range(nst):
        col = (t[:, k] - t0) / 100.0  # us
        s, _ = col.sort()
        print(f"  stamp {k}: min {s[0]:7.2f}  p10 {s[len(s)//10]:7.2f}  med {s[len(s)//2]:7.2f}  p90 {s[len(s)*9//10]:7.2f}  max {s[-1]:7.2f} us")


def main():
    k, r, b = (int(x) for x in sys.argv[1:4])
    assert leo.leo_init() == 0
    lib = leo.lib
    lib.leo_amd_debug_stamps.argtypes = [ctypes.c_void_p]
    stamps = torch.zeros(1 << 22, dtype=torch.int64, device="cuda")
    assert lib.leo_amd_debug_stamps(stamps.data_ptr()) == 0
    leo.set_stream(torch.cuda.current_stream().cuda_stream)
    leo.set_async(True)
    VP = ctypes.c_void_p
    ewc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    o = hash_fill_cuda(torch, 7, k, b, "cuda")
    ew = torch.zeros((ewc, b), dtype=torch.uint8, device="cuda")
    dw = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
    po = (VP * k)(*[o[i].data_ptr() for i in range(k)])
    pe = (VP * ewc)(*[ew[i].data_ptr() for i in range(ewc)])
    pn = (VP * k)()
    pr = (VP * r)(*[ew[i].data_ptr() for i in range(r)])
    pd = (VP * dwc)(*[dw[i].data_ptr() for i in range(dwc)])
    T = (leo.leo_encode_work_count(k, r) // 2 - 1).bit_length()
    for _ in range(200):
        lib.leo_encode(b, k, r, ewc, po, pe)
    torch.cuda.synchronize()
    stamps.zero_()
    lib.leo_encode(b, k, r, ewc, po, pe)
    torch.cuda.synchronize()
    waves_enc = int((stamps.view(-1, 8)[:, 0] != 0).sum())
    show(f"encode {k}+{r} x {b}: {waves_enc} waves", stamps, waves_enc, 6)
    for _ in range(200):
        lib.leo_decode(b, k, r, dwc, pn, pr, pd)
    torch.cuda.synchronize()
    stamps.zero_()
    lib.leo_decode(b, k, r, dwc, pn, pr, pd)
    torch.cuda.synchronize()
    waves_dec = int((stamps.view(-1, 8)[:, 0] != 0).sum())
    show(f"decode {k}+{r} x {b}: {waves_dec} waves", stamps, waves_dec, 7)
    assert torch.equal(dw[:k], o)


if __name__ == "__main__":
    main()
