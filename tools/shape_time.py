"""Per-call GPU time of encode / decode at given shapes (bench.run_shape).
usage: python tools/shape_time.py K,R,B,LOSS [K,R,B,LOSS ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import leopard_amd as leo  # noqa: E402

assert leo.leo_init() == 0, leo.last_error()
dev = torch.device("cuda", 0)
leo.set_stream(torch.cuda.current_stream(dev).cuda_stream)
leo.set_async(True)  # as bench.py: calls queue behind the spin kernel (a synchronous call would time the host)
shapes = sys.argv[1:] or ["1000,200,65536,200", "32768,32768,65536,32768"]
# warm the GPU up first (clocks ramp under sustained load; a cold first shape reads slow)
_w = bench.hash_fill_cuda(torch, 1, 128, 1 << 16, dev)
_ww = torch.empty((256, 1 << 16), dtype=torch.uint8, device=dev)
import time as _t  # noqa: E402
_t0 = _t.perf_counter()
while _t.perf_counter() - _t0 < float(os.environ.get("WARM_S", "2")):
    for _ in range(50):
        leo.encode(_w, 128, _ww)
    torch.cuda.synchronize()
del _w, _ww
for spec in shapes:
    k, r, b, loss = (int(x) for x in spec.split(","))
    res = bench.run_shape(leo, torch, dev, k, r, b, loss, n=10)
    print(json.dumps(res), flush=True)
