#!/usr/bin/env python3
"""FF8 encoder lane-group forms (run with LEO_AMD_FF8_G=1 or 2) vs the oracle; exit 1 on any mismatch.
Used by tests/test_gpu_parity.py::test_encoder_lane_group_forms and as a debug aid."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
import oracle_lib as ol  # noqa: E402

leo.leo_init()
failed = 0
for (k, r, b) in [(50, 20, 64), (50, 20, 256), (100, 20, 256), (32, 20, 256), (40, 20, 256), (64, 32, 256),
                  (128, 128, 1024), (100, 100, 64 * 9), (200, 55, 512), (20, 12, 2048), (7, 5, 128)]:
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    exp = ol.oracle().encode(data, r)
    dev = torch.from_numpy(data).cuda()
    got = leo.encode(dev, r).cpu().numpy()
    bad = np.argwhere(got != exp)
    rows = sorted(set(bad[:, 0].tolist())) if len(bad) else []
    cols = sorted(set((bad[:, 1] // 4).tolist())) if len(bad) else []
    failed += len(rows) > 0
    print(f"slab {k}+{r}x{b}: bad rows {rows[:24]} dword cols {cols[:20]}{'...' if len(cols) > 20 else ''}", flush=True)
sys.exit(1 if failed else 0)
