"""Probe: device memory per fresh stream -- runtime stream state vs library scratch.
Run on the GPU box: python tools/memprobe2.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import leopard_amd as leo  # noqa: E402
import oracle_lib as ol  # noqa: E402

MiB = 1 << 20


def free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return torch.cuda.mem_get_info()[0]


assert leo.leo_init() == 0
k, r, b = 1000, 200, 4096
rng = np.random.default_rng(1)
data = rng.integers(0, 256, (k, b), dtype=np.uint8)
rec = ol.oracle().encode(data, r)
lost = sorted(rng.choice(k, r, replace=False).tolist())
dd, dr = torch.from_numpy(data).cuda(), torch.from_numpy(rec).cuda()
wc = leo.leo_decode_work_count(k, r)
work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
los = set(lost)


def dec():
    return leo.leo_decode(b, k, r, wc, [None if i in los else dd[i].data_ptr() for i in range(k)],
                          [dr[i].data_ptr() for i in range(r)], [work[i].data_ptr() for i in range(wc)])


assert dec() == 0
for _ in range(64):
    with torch.cuda.stream(torch.cuda.Stream()):
        work.add_(0)
leo.release_stream(-1)
f0 = free()
print("base", f0 / MiB)
for j in range(40):
    s = torch.cuda.Stream()
    leo.set_stream(s.cuda_stream)
    assert dec() == 0
    s.synchronize()
    a = (f0 - free()) / MiB
    leo.release_stream(s.cuda_stream)
    c = (f0 - free()) / MiB
    print(f"stream {j} {s.cuda_stream:#x}: after decode {a}, after release {c}", flush=True)
leo.set_stream(None)
leo.release_stream(-1)
print("after release all", (f0 - free()) / MiB)
for j in range(3):
    s = torch.cuda.Stream()
    leo.set_stream(s.cuda_stream)
    assert dec() == 0
    leo.set_stream(None)
    print(f"again {j}: {(f0 - free()) / MiB}", flush=True)
leo.release_stream(-1)
print("end", (f0 - free()) / MiB)
