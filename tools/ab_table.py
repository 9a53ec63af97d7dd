"""Compact table of a tools/gpu_ab_shapes.sh log: variant, workload, encode / decode us."""
import json
import sys

var = "?"
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("=="):
        var = line[3:]
    elif line.startswith("{"):
        try:
            d = json.loads(line)
        except ValueError:
            continue
        print(f"{var:10s} {d['workload'][:44]:44s} enc {d['encode_us']:9.2f} dec {d['decode_us']:9.2f} ok={d['roundtrip_ok']}")
