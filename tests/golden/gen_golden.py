#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

The reference library is compiled from /root/reference by ``make -C oracle ref``
into oracle/_ref/libleopard_ref.so (its own sources, untouched; nothing copied
into this repo).  This script drives its C ABI (leopard.h:143-234) on synthetic
inputs from the reference benchmark's PCG generator (tests/benchmark.cpp:134-156)
and stores only inputs' seeds and outputs:

* golden_small.npz   full recovery bytes for small (K, R, B) shapes, FF8 and FF16,
                     plus decoder outputs on NON-codeword inputs (random
                     "recovery" bytes), which pins the decoder's exact linear map
                     and not just its round-trip property.
* golden_digests.json SHA-256 of the recovery bytes for the BASELINE.json shapes
                     (128+128, 1000+200 at B=64000/65536 and 32768+32768 at 65536),
                     for PCG inputs ("digests") and for counter-hash inputs
                     ("hash_digests": oracle_lib.hash_bytes, seed 7, which the GPU
                     tests regenerate on the device in milliseconds).

Input convention: piece i, byte j = low 8 bits of the (i*B + j)-th PCG32 output
after PCGRandom.Seed(seed, trial) -- seed 2 as in tests/benchmark.cpp:53.

Run:  make -C oracle ref && python tests/golden/gen_golden.py [--big]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402

# (K, R, B): FF8 and FF16 shapes covering K==1, R==1, K % m != 0, R not a power
# of two, multi-chunk encoders, the FF8/FF16 boundary (n = 256 vs 512).
SMALL_ENC = [
    (1, 1, 64), (2, 2, 64), (3, 1, 64), (3, 2, 64), (7, 5, 128), (16, 16, 64), (17, 16, 192),
    (100, 20, 64), (128, 128, 128), (130, 126, 64), (200, 55, 64), (255, 1, 64), (64, 64, 320),
    (129, 127, 64), (300, 37, 128), (1000, 200, 64), (5000, 3000, 64), (60000, 1000, 64),
    (33, 9, 64), (250, 6, 64),
]
# Decoder on non-codeword inputs: (K, R, B, losses)
SMALL_DEC = [
    (2, 2, 64, 1), (7, 5, 128, 5), (100, 20, 64, 20), (128, 128, 64, 128), (130, 126, 64, 100),
    (200, 55, 64, 55), (129, 127, 64, 127), (300, 37, 128, 30), (1000, 200, 64, 200),
    (5000, 3000, 64, 3000),
]
BIG = [(128, 128, 65536), (128, 128, 64000), (1000, 200, 65536), (1000, 200, 64000), (32768, 32768, 65536)]


def key(*a):
    return "_".join(str(int(x)) for x in a)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also digest the BASELINE shapes (needs ~10 GB RAM)")
    ap.add_argument("--big-decode", action="store_true",
                    help="only add the decoder digests at the BASELINE shapes to golden_digests.json")
    args = ap.parse_args()
    ref = ol.reference()
    if ref is None:
        sys.exit("build the reference first: make -C oracle ref")
    if args.big_decode:
        big_decode(ref)
        return

    out = {}
    for (k, r, b) in SMALL_ENC:
        d = ol.pcg_bytes(2, 0, k, b)
        out["enc_" + key(k, r, b)] = ref.encode(d, r)
        print("enc", k, r, b, flush=True)
    for (k, r, b, loss) in SMALL_DEC:
        d = ol.pcg_bytes(2, 1, k, b)
        rec = ol.pcg_bytes(2, 2, r, b)  # not a codeword: pins the exact decoder map
        lo, lr = ol.benchmark_losses(k, r, loss, seed=2, trial=3)
        res = ref.decode(d, rec, lo, lr)
        out["declo_" + key(k, r, b, loss)] = np.array(lo, dtype=np.int32)
        out["declr_" + key(k, r, b, loss)] = np.array(lr, dtype=np.int32)
        out["decout_" + key(k, r, b, loss)] = np.stack([res[i] for i in lo])
        print("dec", k, r, b, loss, flush=True)
    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), **out)

    if args.big:
        dig = {}
        for (k, r, b) in BIG:
            d = ol.pcg_bytes(2, 0, k, b)
            rec = ref.encode(d, r)
            dig[key(k, r, b)] = hashlib.sha256(rec.tobytes()).hexdigest()
            print("big", k, r, b, dig[key(k, r, b)], flush=True)
            del d, rec
        hdig = {}
        for (k, r, b) in BIG:
            d = ol.hash_bytes(7, k, b)
            rec = ref.encode(d, r)
            hdig[key(k, r, b)] = hashlib.sha256(rec.tobytes()).hexdigest()
            print("big-hash", k, r, b, hdig[key(k, r, b)], flush=True)
            del d, rec
        with open(os.path.join(HERE, "golden_digests.json"), "w") as f:
            json.dump({"convention": "sha256 of recovery pieces 0..R-1 concatenated; inputs pcg_bytes(2,0,K,B) "
                                     "for 'digests', hash_bytes(7,K,B) for 'hash_digests'",
                       "digests": dig, "hash_digests": hdig}, f, indent=1)


def big_decode(ref):
    """Decoder digests at the BASELINE shapes on NON-codeword inputs (pins the
    decoder's exact map at full size, not only its round trip): originals
    hash_bytes(7, K, B), "recovery" pieces hash_bytes(8, R, B), the benchmark's
    loss pattern with loss = R (benchmark_losses(K, R, R, seed=2, trial=0):
    R originals lost, every recovery piece kept); digest = sha256 of the
    rebuilt originals concatenated in loss order."""
    path = os.path.join(HERE, "golden_digests.json")
    with open(path) as f:
        doc = json.load(f)
    dd = doc.setdefault("decode_hash_digests", {})
    for (k, r, b) in BIG:
        d = ol.hash_bytes(7, k, b)
        rec = ol.hash_bytes(8, r, b)
        lo, lr = ol.benchmark_losses(k, r, r, seed=2, trial=0)
        res = ref.decode(d, rec, lo, lr)
        h = hashlib.sha256()
        for i in lo:
            h.update(res[i].tobytes())
        dd[key(k, r, b)] = h.hexdigest()
        print("big-decode", k, r, b, dd[key(k, r, b)], flush=True)
        del d, rec, res
    doc["decode_convention"] = ("decode_hash_digests: sha256 of the lost originals (benchmark_losses(K, R, R, seed=2, "
                                "trial=0) order) rebuilt from originals hash_bytes(7,K,B) and non-codeword recovery "
                                "pieces hash_bytes(8,R,B)")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
