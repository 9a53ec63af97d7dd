#!/usr/bin/env python3
"""GF(2^16) batch vs single calls (bench.ff16_batch) at several piece sizes:
usage: ff16batch.py K R LOSS OBJECTS B [B ...]   (us per object)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
import bench  # noqa: E402


def main():
    k, r, loss, objs = (int(x) for x in sys.argv[1:5])
    assert leo.leo_init() == 0
    leo.set_async(True)
    dev = torch.device("cuda", 0)
    for b in (int(x) for x in sys.argv[5:]):
        res = bench.ff16_batch(leo, torch, dev, k=k, r=r, nbytes=b, objects=objs, loss=loss)
        print(json.dumps({"bytes": b, **{x: res[x] for x in res if x.endswith("per_object") or x == "roundtrip_ok"}}),
              flush=True)


if __name__ == "__main__":
    main()
