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
shapes = sys.argv[1:] or ["1000,200,65536,200", "32768,32768,65536,32768"]
for spec in shapes:
    k, r, b, loss = (int(x) for x in spec.split(","))
    res = bench.run_shape(leo, torch, dev, k, r, b, loss, n=10)
    print(json.dumps(res), flush=True)
