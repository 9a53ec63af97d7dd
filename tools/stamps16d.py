"""Phase timeline of k_dec16n_fin (rs_ff16_small.hip) from an LAMD_STAMPS build:
one decode at K+R x B with the benchmark loss pattern (bench.run_shape's).
usage: LEOPARD_AMD_LIB=leopard_amd/exp/stamps/libleopard_amd.so python tools/stamps16d.py K R B LOSS"""
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
for _ in range(20):
    assert lib.leo_decode(b, k, r, dwc, po, pr, pd) == 0
torch.cuda.synchronize()
stamps.zero_()
assert lib.leo_decode(b, k, r, dwc, po, pr, pd) == 0
torch.cuda.synchronize()
NS = 5
allv = stamps.view(-1, 8)[:, :NS].cpu().double()
t0 = allv[allv[:, 0] > 0][:, 0].min()
for name, lo_, hi_, phases in (("pass 1 (k_dec16n_lo)", 0, (1 << 22) // 8,
                                "loads+tables, scale, IFFT, store"),
                               ("pass 2 (k_dec16n_fin)", (1 << 22) // 8, None,
                                "tables+first U, fold loop, FFT, reveal+store")):
    v = allv[lo_:hi_]
    v = v[v[:, 0] > 0]
    print(f"{name}: {k}+{r} x {b}, {loss} lost: {len(v)} waves stamped")
    for kk in range(NS):
        col = ((v[:, kk] - t0) / 100.0).sort()[0]
        n = len(col)
        print(f"  stamp {kk}: min {col[0]:7.2f} p10 {col[n//10]:7.2f} med {col[n//2]:7.2f} p90 {col[n*9//10]:7.2f} max {col[-1]:7.2f} us")
    d = (v[:, 1:] - v[:, :-1]) / 100.0
    print(f"  per-wave phase durations (median us): {phases}:", [round(float(x), 2) for x in d.median(dim=0)[0]])
