#!/usr/bin/env python3
"""In-kernel shader clock of the FF8 slab batch kernel (LAMD_CLOCK build,
diagnostics only): >= 2 s of back-to-back 16-object encode launches, then the
last launch's per-workgroup (s_memtime, s_memrealtime) pairs give the clock
(MI355X_MICROARCH.md "DVFS give-back" item 6) and the workgroup lifetimes.
usage: LEOPARD_AMD_LIB=leopard_amd/exp/clock/libleopard_amd.so python tools/clock.py [K R B OBJ]"""
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
    k, r, b, cnt = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else [128, 128, 65536, 16]))
    assert leo.leo_init() == 0
    lib = leo.lib
    lib.leo_amd_debug_clock.argtypes = [VP]
    nwg = (b // 256) * cnt
    buf = torch.zeros(nwg * 4, dtype=torch.int64, device="cuda")
    assert lib.leo_amd_debug_clock(buf.data_ptr()) == 0
    leo.set_async(True)
    s = torch.cuda.current_stream()
    leo.set_stream(s.cuda_stream)
    sets = Sets(leo, torch, k, r, b, cnt, "cuda")
    mk = lambda arrs: (PP * len(arrs))(*[ctypes.cast(a, PP) for a in arrs])  # noqa: E731
    bo, bw = mk(sets.p_orig[:cnt]), mk(sets.p_encw[:cnt])
    t0 = time.time()
    n = 0
    while time.time() - t0 < 2.5:
        for _ in range(50):
            assert lib.leo_amd_encode_batch(cnt, b, k, r, sets.enc_wc, bo, bw) == 0, leo.last_error()
        n += 50
        torch.cuda.synchronize()
    v = buf.view(nwg, 4).cpu().double()
    dc, dr = v[:, 2] - v[:, 0], (v[:, 3] - v[:, 1])
    clk = (dc / dr * 100.0).sort().values  # MHz
    life = (dr / 100.0).sort().values  # us
    span = (v[:, 3].max() - v[:, 1].min()) / 100.0
    q = lambda t, f: float(t[int(f * (len(t) - 1))])  # noqa: E731
    print(f"{k}+{r}x{b} objects={cnt} launches={n}: clock MHz p10 {q(clk, .1):.0f} med {q(clk, .5):.0f} p90 {q(clk, .9):.0f}; "
          f"workgroup life us p10 {q(life, .1):.2f} med {q(life, .5):.2f} p90 {q(life, .9):.2f}; launch span {span:.1f} us; "
          f"workgroups {nwg}")


if __name__ == "__main__":
    main()
