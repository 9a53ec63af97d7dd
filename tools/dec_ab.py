#!/usr/bin/env python3
"""Encode / decode timing of (K, R, B, loss) shapes through bench.run_shape
(benchmark loss pattern, HIP events).  usage: dec_ab.py K R B LOSS [K R B LOSS ...]
Environment switches (LEO_AMD_FF8_SPLIT=0, ...) select the decoder variant."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
from bench import run_shape  # noqa: E402


def main():
    v = [int(x) for x in sys.argv[1:]]
    assert leo.leo_init() == 0
    leo.set_async(True)  # as bench.py: calls do not wait for their kernels
    tag = " ".join(f"{k}={os.environ[k]}" for k in sorted(os.environ) if k.startswith("LEO_AMD_"))
    for i in range(0, len(v), 4):
        k, r, b, loss = v[i:i + 4]
        res = run_shape(leo, torch, "cuda", k, r, b, loss, n=int(os.environ.get("AB_N", "20")))
        print(json.dumps({"env": tag, **res}), flush=True)


if __name__ == "__main__":
    main()
