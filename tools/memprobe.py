"""Probe: device memory accounting of the library's scratch (stream-ordered
pool vs hipMalloc), and whether hipFree blocks on other streams' work.
Run on the GPU box: python tools/memprobe.py"""
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import leopard_amd as leo  # noqa: E402
import oracle_lib as ol  # noqa: E402

MiB = 1 << 20
hip = ctypes.CDLL("libamdhip64.so")


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


f0 = free()
print("start free MiB", f0 / MiB)
assert dec() == 0
f1 = free()
print("after first call (main thread):", (f0 - f1) / MiB, "MiB used")
leo.release_stream(-1)
f2 = free()
print("after release_stream(-1):", (f0 - f2) / MiB)
for j in range(3):
    t = threading.Thread(target=dec)
    t.start()
    t.join()
    a = (f0 - free()) / MiB
    time.sleep(0.5)
    print(f"after thread {j}: right after join {a}, 0.5 s later {(f0 - free()) / MiB}")

pool = ctypes.c_void_p()
hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0)
for case in ("free on other stream", "free on other stream + device sync + trim", "free on own stream"):
    A, svc, p = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(A))
    hip.hipStreamCreateWithFlags(ctypes.byref(svc), 1)
    g0 = free()
    hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(32 * MiB), A)
    hip.hipStreamSynchronize(A)
    if case.startswith("free on own"):
        hip.hipFreeAsync(p, A)
        hip.hipStreamSynchronize(A)
    else:
        hip.hipFreeAsync(p, svc)
        hip.hipStreamSynchronize(svc)
    hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
    g1 = free()
    extra = ""
    if "device sync" in case:
        hip.hipDeviceSynchronize()
        hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
        extra = f", after device sync + trim {(g0 - free()) / MiB}"
    hip.hipStreamDestroy(A)
    hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
    print(f"{case}: held after free+trim {(g0 - g1) / MiB}{extra}, after destroying A + trim {(g0 - free()) / MiB}")

# raw pool behaviour
p = ctypes.c_void_p()
s = ctypes.c_void_p()
hip.hipStreamCreate(ctypes.byref(s))
g0 = free()
for sz in (16 * MiB, 64 * MiB):
    hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(sz), s)
    hip.hipStreamSynchronize(s)
    g1 = free()
    hip.hipFreeAsync(p, s)
    hip.hipStreamSynchronize(s)
    g2 = free()
    pool = ctypes.c_void_p()
    hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0)
    rc = hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
    g3 = free()
    print(f"pool {sz // MiB} MiB: alloc {(g0 - g1) / MiB}, after free {(g0 - g2) / MiB}, after trim (rc {rc}) "
          f"{(g0 - g3) / MiB}")

# does hipFree wait for another stream's work?
q = ctypes.c_void_p()
hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(64 * MiB))
torch.cuda.synchronize()
other = torch.cuda.Stream()
with torch.cuda.stream(other):
    torch.cuda._sleep(200_000_000)  # ~100 ms on the other stream
t0 = time.perf_counter()
hip.hipFree(q)
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"hipFree returned after {1e3 * (t1 - t0):.1f} ms while another stream slept ~100 ms")
hip.hipMallocAsync(ctypes.byref(q), ctypes.c_size_t(64 * MiB), s)
hip.hipStreamSynchronize(s)
with torch.cuda.stream(other):
    torch.cuda._sleep(200_000_000)
t0 = time.perf_counter()
hip.hipFreeAsync(q, s)
hip.hipStreamSynchronize(s)
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"hipFreeAsync+sync(own stream) returned after {1e3 * (t1 - t0):.1f} ms")
