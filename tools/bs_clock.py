#!/usr/bin/env python3
"""In-kernel shader clock of the bit-sliced slab kernel (rs_ff8_bs.hip built
with -DLAMD_CLOCK, diagnostics only): >= 2 s of back-to-back 64-object
encode launches of 128 + 128 x 65536 B, then the last launch's per-wave
(s_memtime, s_memrealtime) pairs give the shader clock under this kernel's load
and each persistent wave's lifetime.
usage: LEOPARD_AMD_LIB=leopard_amd/exp/<clock build>/libleopard_amd.so python tools/bs_clock.py [OBJ]"""
import ctypes
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import Sets  # noqa: E402

VP = ctypes.c_void_p
PP = ctypes.POINTER(VP)


def main():
    k, r, b = 128, 128, 65536
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    assert leo.leo_init() == 0
    lib = leo.lib
    lib.leo_amd_debug_bs_clock.argtypes = [VP]
    ntiles = (b // 256) * cnt
    buf = torch.zeros(ntiles * 4, dtype=torch.int64, device="cuda")
    assert lib.leo_amd_debug_bs_clock(buf.data_ptr()) == 0
    leo.set_async(True)
    s = torch.cuda.current_stream()
    leo.set_stream(s.cuda_stream)
    sets = Sets(leo, torch, k, r, b, cnt, "cuda")
    mk = lambda arrs: (PP * len(arrs))(*[ctypes.cast(a, PP) for a in arrs])  # noqa: E731
    bo, bw = mk(sets.p_orig[:cnt]), mk(sets.p_encw[:cnt])
    t0 = time.time()
    n = 0
    dur = float(os.environ.get("BS_CLOCK_S", "2.5"))
    samples = []

    def sample():  # BS_CLOCK_SMI=1: board power and clocks under the load (read-only queries)
        time.sleep(1.0)
        for cmd in (["amd-smi", "metric", "-p", "-c"], ["rocm-smi", "--showpower", "--showclocks"]):
            try:
                samples.append(subprocess.run(cmd, capture_output=True, text=True, timeout=20).stdout)
            except Exception as e:  # noqa: BLE001
                samples.append(f"{cmd[0]}: {e}")

    th = threading.Thread(target=sample) if os.environ.get("BS_CLOCK_SMI") else None
    if th:
        th.start()
    while time.time() - t0 < dur:
        buf.zero_()
        for _ in range(20):
            assert lib.leo_amd_encode_batch(cnt, b, k, r, sets.enc_wc, bo, bw) == 0, leo.last_error()
        n += 20
        torch.cuda.synchronize()
    if th:
        th.join()
        for o in samples:
            print("\n".join(ln for ln in o.splitlines() if ln.strip() and "amdgpu.ids" not in ln)[:3000])
    v = buf.view(ntiles, 4).cpu().double()
    v = v[v[:, 3] > 0]  # one row per persistent wave (indexed by its first tile)
    dc, dr = v[:, 2] - v[:, 0], (v[:, 3] - v[:, 1])
    clk = (dc / dr * 100.0).sort().values  # MHz
    life = (dr / 100.0).sort().values  # us
    start = ((v[:, 1] - v[:, 1].min()) / 100.0).sort().values
    span = (v[:, 3].max() - v[:, 1].min()) / 100.0
    q = lambda t, f: float(t[int(f * (len(t) - 1))])  # noqa: E731
    print(f"{k}+{r}x{b} objects={cnt} launches={n} waves={len(v)}: clock MHz p10 {q(clk, .1):.0f} med {q(clk, .5):.0f} "
          f"p90 {q(clk, .9):.0f}; wave life us p10 {q(life, .1):.1f} med {q(life, .5):.1f} p90 {q(life, .9):.1f}; "
          f"start us p90 {q(start, .9):.1f} max {float(start[-1]):.1f}; launch span {span:.1f} us")


if __name__ == "__main__":
    main()
