#!/usr/bin/env python3
"""Run one encode/decode case on the GPU and compare with the oracle (debug aid).
usage: probe_case.py K R B LOSS [seed]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import leopard_amd as leo  # noqa: E402
import oracle_lib as ol  # noqa: E402


def main():
    assert leo.leo_init() == 0
    args = sys.argv[1:]
    for i in range(0, len(args), 4):
        case(*(int(x) for x in args[i:i + 4]))


def case(k, r, b, loss, seed=1):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    rec = ol.oracle().encode(data, r)
    dt = torch.from_numpy(data).cuda()
    got_rec = leo.encode(dt, r).cpu().numpy()
    enc_ok = np.array_equal(got_rec, rec)
    if not enc_ok:
        rows = [i for i in range(r) if not np.array_equal(got_rec[i], rec[i])]
        cols = sorted(set(np.nonzero((got_rec != rec).any(axis=0))[0].tolist()))
        print(f"  encode bad rows {len(rows)}: {rows[:40]} ... bad cols {len(cols)}: {cols[:32]}")
    lo = sorted(rng.choice(k, loss, replace=False).tolist())
    lr = sorted(rng.choice(r, r - loss, replace=False).tolist())
    try:
        res = leo.decode(dt, torch.from_numpy(rec).cuda(), lo, lr)
        torch.cuda.synchronize()
        bad = [i for i in lo if not np.array_equal(res[i].cpu().numpy(), data[i])]
        print(f"case {k} {r} {b} {loss}: enc_ok={enc_ok} dec_bad={len(bad)}/{len(lo)} {bad[:8]}")
    except Exception as e:  # noqa: BLE001
        print(f"case {k} {r} {b} {loss}: enc_ok={enc_ok} decode error {e}")
        sys.exit(3)
    if bad:
        d = res[bad[0]].cpu().numpy() != data[bad[0]]
        print(f"  first bad piece {bad[0]}: bad cols {np.nonzero(d)[0][:32].tolist()}")


if __name__ == "__main__":
    main()
