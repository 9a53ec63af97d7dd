#!/usr/bin/env python3
"""bench.py's host_e2e leg alone (PCIe-inclusive encode + full-loss decode on
caller-owned host buffers, pageable and registered).  usage: hoste2e.py [K R B]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import leopard_amd as leo  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    k, r, b = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (128, 128, 65536)
    assert leo.leo_init() == 0
    print(json.dumps(bench.host_e2e(leo, k, r, b)), flush=True)
