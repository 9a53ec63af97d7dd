#!/usr/bin/env python3
"""Tabulate tools/gpu_ab.sh output of tools/shape_time.py: one row per shape,
encode / decode µs per build or environment.  usage: ab_shapes.py FILE"""
import json
import sys

cur, rows = None, {}
for line in open(sys.argv[1]):
    if line.startswith('=='):
        cur = line.split(maxsplit=1)[1].strip()
    elif line.startswith('{'):
        d = json.loads(line)
        rows.setdefault(d['workload'], []).append((cur, d['encode_us'], d['decode_us']))
for w, v in rows.items():
    print(w)
    for c, e, d in v:
        print(f"    {c:40s} encode {e:7.2f}  decode {d:7.2f}")
