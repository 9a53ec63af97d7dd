#!/usr/bin/env python3
"""Board power and shader clocks while one codec call shape runs back to back
(performance diagnostics only): leo_encode or leo_decode (first min(K, R)
originals lost) of K + R x B device pieces for S seconds on one stream, with
amd-smi (read-only) sampled from a helper thread one second in.  Prints the
calls per second and the sampled socket power / per-XCD GFX clocks.
usage: smi_probe.py K R B encode|decode [S]"""
import ctypes
import os
import re
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import hash_fill_cuda  # noqa: E402


def main():
    k, r, b = (int(x) for x in sys.argv[1:4])
    kind = sys.argv[4]
    dur = float(sys.argv[5]) if len(sys.argv) > 5 else 6.0
    VP = ctypes.c_void_p
    assert leo.leo_init() == 0
    leo.set_stream(torch.cuda.current_stream().cuda_stream)
    leo.set_async(True)
    lib = leo.lib
    ewc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    o = hash_fill_cuda(torch, 7, k, b, "cuda")
    ew = torch.zeros((ewc, b), dtype=torch.uint8, device="cuda")
    dw = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
    po = (VP * k)(*[o[i].data_ptr() for i in range(k)])
    pe = (VP * ewc)(*[ew[i].data_ptr() for i in range(ewc)])
    lost = min(k, r)
    pn = (VP * k)(*([None] * lost + [o[i].data_ptr() for i in range(lost, k)]))
    pr = (VP * r)(*[ew[i].data_ptr() for i in range(r)])
    pd = (VP * dwc)(*[dw[i].data_ptr() for i in range(dwc)])
    assert lib.leo_encode(b, k, r, ewc, po, pe) == 0, leo.last_error()
    fn = (lambda: lib.leo_encode(b, k, r, ewc, po, pe)) if kind == "encode" else \
         (lambda: lib.leo_decode(b, k, r, dwc, pn, pr, pd))
    torch.cuda.synchronize()
    samples = []

    def sample():
        time.sleep(1.0)
        samples.append(subprocess.run(["amd-smi", "metric", "-p", "-c"], capture_output=True, text=True,
                                      timeout=30).stdout)

    th = threading.Thread(target=sample)
    t0 = time.time()
    th.start()
    n = 0
    while time.time() - t0 < dur:
        for _ in range(4):
            assert fn() == 0, leo.last_error()
        n += 4
        torch.cuda.synchronize()
    el = time.time() - t0
    th.join()
    txt = samples[0] if samples else ""
    pw = re.findall(r"SOCKET_POWER:\s*(\d+)", txt)
    clk = [int(c) for c in re.findall(r"GFX_\d+:\s*\n\s*CLK:\s*(\d+)", txt)]
    print(f"{k}+{r} x {b} {kind}: {n / el:.1f} calls/s ({el / n * 1e6:.1f} us per call); socket power {pw} W; "
          f"GFX clocks MHz {clk}", flush=True)


if __name__ == "__main__":
    main()
