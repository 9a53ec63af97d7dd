"""Phase timeline of k_dec16n_one (rs_ff16_small.hip) from an LAMD_STAMPS build:
one decode at K+R x B with the benchmark loss pattern (bench.run_shape's).
Per wave 32 stamps: 0 start, 1 first tile staged, per input tile i: 2+3i scale +
IFFT done, 3+3i fold done, 4+3i next tile's loads / tables waited for; 26+k
output tile k done (FFT + reveal + store).
usage: LEOPARD_AMD_LIB=leopard_amd/exp/stamps/libleopard_amd.so python tools/stamps16one.py K R B LOSS"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
import oracle_lib as ol  # noqa: E402
from bench import hash_fill_cuda, ptrs  # noqa: E402

k, r, b, loss = (int(x) for x in sys.argv[1:5])
assert leo.leo_init() == 0
lib = leo.lib
lib.leo_amd_debug_stamps16.argtypes = [ctypes.c_void_p]
stamps = torch.zeros(1 << 24, dtype=torch.int64, device="cuda")
assert lib.leo_amd_debug_stamps16(stamps.data_ptr()) == 0
ewc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
o = hash_fill_cuda(torch, 7, k, b, "cuda")
ew = torch.zeros((ewc, b), dtype=torch.uint8, device="cuda")
dw = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
assert lib.leo_encode(b, k, r, ewc, ptrs(o), ptrs(ew)) == 0
lo, lr = ol.benchmark_losses(k, r, loss, seed=2, trial=0)
po, pr, pd = ptrs(o, lost=lo), ptrs(ew, r, lost=lr), ptrs(dw)
for _ in range(200):
    assert lib.leo_decode(b, k, r, dwc, po, pr, pd) == 0
torch.cuda.synchronize()
stamps.zero_()
assert lib.leo_decode(b, k, r, dwc, po, pr, pd) == 0
torch.cuda.synchronize()
base = (2 << 22) // 32
v = stamps.view(-1, 32)[base:].cpu().double()
v = v[v[:, 0] > 0]
t0 = v[:, 0].min()
v = torch.where(v > 0, (v - t0) / 100.0, torch.full_like(v, float("nan")))  # s_memrealtime: 100 MHz -> us
print(f"waves {len(v)}; kernel span {float(torch.nan_to_num(v, nan=0).max()):.2f} us")


def q(x):
    x = x[~torch.isnan(x)]
    if len(x) == 0:
        return "-"
    p = torch.quantile(x, torch.tensor([0.1, 0.5, 0.9], dtype=torch.double))
    return f"p10 {float(p[0]):7.2f}  median {float(p[1]):7.2f}  p90 {float(p[2]):7.2f}"


print(f"  first tile staged             {q(v[:, 1] - v[:, 0])}")
prev = v[:, 1]
for i in range(8):
    if torch.isnan(v[:, 2 + 3 * i]).all():
        break
    print(f"  tile {i}: scale + IFFT        {q(v[:, 2 + 3 * i] - prev)}")
    print(f"  tile {i}: fold                {q(v[:, 3 + 3 * i] - v[:, 2 + 3 * i])}")
    print(f"  tile {i}: wait next           {q(v[:, 4 + 3 * i] - v[:, 3 + 3 * i])}")
    prev = v[:, 4 + 3 * i]
for kk in range(4):
    if torch.isnan(v[:, 26 + kk]).all():
        continue
    print(f"  output {kk}: FFT+reveal        {q(v[:, 26 + kk] - prev)}")
    prev = v[:, 26 + kk]
