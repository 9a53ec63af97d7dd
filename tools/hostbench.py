#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) encode / full-loss decode rates through the C
ABI with pageable numpy buffers.  usage: hostbench.py K R B [K R B ...]
(LEO_AMD_SLOT_MB / LEO_AMD_HOST_THREADS tune the library's staging ring)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import leopard_amd as leo  # noqa: E402


def run(k, r, b, steps=10):
    data = np.frombuffer(np.random.default_rng(7).bytes(k * b), dtype=np.uint8).reshape(k, b)
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    work = np.zeros((wc, b), dtype=np.uint8)
    dwork = np.zeros((dwc, b), dtype=np.uint8)
    po = [data[i].ctypes.data for i in range(k)]
    pe = [work[i].ctypes.data for i in range(wc)]
    pr = [work[i].ctypes.data for i in range(r)]
    pd = [dwork[i].ctypes.data for i in range(dwc)]
    lost = [None] * min(k, r) + po[min(k, r):]
    enc = lambda: leo.leo_encode(b, k, r, wc, po, pe)
    dec = lambda: leo.leo_decode(b, k, r, dwc, lost, pr, pd)
    assert enc() == 0 and dec() == 0, leo.last_error()
    assert np.array_equal(dwork[:min(k, r)], data[:min(k, r)])
    te = td = 0.0
    for _ in range(steps):
        t0 = time.perf_counter(); enc(); t1 = time.perf_counter(); dec(); t2 = time.perf_counter()
        te += t1 - t0; td += t2 - t1
    inb = k * b * steps
    print(f"{k}+{r} x {b}: encode {inb / te / 1e9:6.2f} GB/s  decode {inb / td / 1e9:6.2f} GB/s  "
          f"step {inb / (te + td) / 1e9:6.2f} GB/s  (slot={os.environ.get('LEO_AMD_SLOT_MB', '32')} MiB, "
          f"threads={os.environ.get('LEO_AMD_HOST_THREADS', 'auto')})", flush=True)


def main():
    assert leo.leo_init() == 0
    a = [int(x) for x in sys.argv[1:]] or [128, 128, 65536]
    for i in range(0, len(a), 3):
        run(*a[i:i + 3])


if __name__ == "__main__":
    main()
