#!/usr/bin/env python3
"""Run bench.py (headline only unless extra args say otherwise) in a child
process and print one short line: value, GPU time per launch, spans, frac.
  python3 tools/bench_brief.py [bench.py args...]   (for tools/gpu_ab.sh CMD)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = sys.argv[1:] or ["--steps", "100", "--warmup", "10", "--no-host", "--no-cpu-baseline", "--no-sharded",
                        "--no-secondary"]
p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True)
if p.returncode != 0:
    sys.stderr.write(p.stderr[-3000:])
    sys.exit(p.returncode)
d = json.loads(p.stdout.strip().splitlines()[-1])
r = d["roofline"]
print("value %.1f GB/s  launch %.1f us  spans %s / %s us  frac %.4f" % (
    d["value"], r["launch_us"], r.get("launch_span_encode_us"), r.get("launch_span_decode_us"), r["frac"]))
keys = ["single_call_us", "configs2_encode_us", "configs2_decode_us", "configs3_encode_ms", "configs3_decode_ms",
        "configs1_16loss_decode_us", "ff16_batch_speedup_encode", "ff16_batch_speedup_decode"]
extra = ["%s %s" % (k, r[k]) for k in keys if k in r]
if "breadth_100x10_decode_us" in d:
    extra.append("breadth_100x10_decode_us %s" % d["breadth_100x10_decode_us"])
for sec in d.get("secondary") or []:
    if sec.get("kind") == "ff16_batch":
        extra.append("ff16 batch us/object enc %s dec %s" % (sec["batch_encode_us_per_object"],
                                                            sec["batch_decode_us_per_object"]))
if extra:
    print("  " + "; ".join(extra))
