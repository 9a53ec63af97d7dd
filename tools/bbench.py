#!/usr/bin/env python3
"""Batched-launch timing: leo_amd_encode_batch / leo_amd_decode_batch (full
loss) over OBJ objects, each timed alone with HIP events on the call stream
(back-to-back launches behind a spin kernel).  Reports us per launch, us per
object and the algorithmic HBM rate ((K + R) * B per object) against 8 TB/s.
usage: bbench.py K R B OBJ [OBJ ...]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import Sets  # noqa: E402

VP = ctypes.c_void_p
PP = ctypes.POINTER(VP)


def main():
    k, r, b = (int(x) for x in sys.argv[1:4])
    counts = [int(x) for x in sys.argv[4:]] or [16]
    assert leo.leo_init() == 0
    leo.set_async(True)
    s = torch.cuda.current_stream()
    leo.set_stream(s.cuda_stream)
    nsets = max(counts) * 2
    sets = Sets(leo, torch, k, r, b, nsets, "cuda")
    lib = leo.lib
    for cnt in counts:
        mk = lambda arrs: (PP * len(arrs))(*[ctypes.cast(a, PP) for a in arrs])  # noqa: E731
        groups = []
        for g in range(2):
            ids = [g * cnt + o for o in range(cnt)]
            groups.append((mk([sets.p_orig[i] for i in ids]), mk([sets.p_encw[i] for i in ids]),
                           mk([sets.p_null[i] for i in ids]), mk([sets.p_rec[i] for i in ids]),
                           mk([sets.p_decw[i] for i in ids]), ids))

        def enc(g):
            bo, bw, _, _, _, _ = groups[g]
            assert lib.leo_amd_encode_batch(cnt, b, k, r, sets.enc_wc, bo, bw) == 0, leo.last_error()

        def dec(g):
            _, _, bn, br, bd, _ = groups[g]
            assert lib.leo_amd_decode_batch(cnt, b, k, r, sets.dec_wc, bn, br, bd) == 0, leo.last_error()

        for g in range(2):
            enc(g)
            dec(g)
        torch.cuda.synchronize()
        for g in range(2):
            for i in groups[g][5]:  # BB_NOCHECK=1: ablation builds (wrong results by design)
                assert os.environ.get("BB_NOCHECK") or torch.equal(sets.dec_work[i][:k], sets.orig[i]), "decode mismatch"

        def t(fn, n=20):
            for j in range(4):
                fn(j & 1)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(20_000_000)
            e0.record(s)
            for j in range(n):
                fn(j & 1)
            e1.record(s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / 1e3 / n

        te, td = t(enc), t(dec)
        algo = (k + r) * b
        print(f"{k}+{r}x{b} objects={cnt}: encode {te * 1e6:8.1f} us/launch {te / cnt * 1e6:6.2f} us/obj "
              f"{algo * cnt / te / 1e9:7.1f} GB/s ({algo * cnt / te / 8e12:.3f}) | decode {td * 1e6:8.1f} us/launch "
              f"{td / cnt * 1e6:6.2f} us/obj {algo * cnt / td / 1e9:7.1f} GB/s ({algo * cnt / td / 8e12:.3f})",
              flush=True)


if __name__ == "__main__":
    main()
