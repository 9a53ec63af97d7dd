"""Phase timeline of k_enc16n (rs_ff16_small.hip) from an LAMD_STAMPS build.
usage: LEOPARD_AMD_LIB=leopard_amd/exp/stamps/libleopard_amd.so python tools/stamps16.py K R B"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import hash_fill_cuda  # noqa: E402

k, r, b = (int(x) for x in sys.argv[1:4])
assert leo.leo_init() == 0
lib = leo.lib
lib.leo_amd_debug_stamps16.argtypes = [ctypes.c_void_p]
stamps = torch.zeros(1 << 22, dtype=torch.int64, device="cuda")
assert lib.leo_amd_debug_stamps16(stamps.data_ptr()) == 0
VP = ctypes.c_void_p
ewc = leo.leo_encode_work_count(k, r)
o = hash_fill_cuda(torch, 7, k, b, "cuda")
ew = torch.zeros((ewc, b), dtype=torch.uint8, device="cuda")
po = (VP * k)(*[o[i].data_ptr() for i in range(k)])
pe = (VP * ewc)(*[ew[i].data_ptr() for i in range(ewc)])
for _ in range(20):
    lib.leo_encode(b, k, r, ewc, po, pe)
torch.cuda.synchronize()
stamps.zero_()
lib.leo_encode(b, k, r, ewc, po, pe)
torch.cuda.synchronize()
nwaves = (b // 128) * 8
t = stamps[: nwaves * 8].view(nwaves, 8).cpu().double()
t0 = t[:, 0].min()
for kk in range(8):
    col = ((t[:, kk] - t0) / 100.0).sort()[0]
    n = len(col)
    print(f"stamp {kk}: min {col[0]:7.2f} p10 {col[n//10]:7.2f} med {col[n//2]:7.2f} p90 {col[n*9//10]:7.2f} max {col[-1]:7.2f} us")
d = (t[:, 1:] - t[:, :-1]) / 100.0
print("per-wave phase durations (median us):", [round(float(x), 2) for x in d.median(dim=0)[0]])
