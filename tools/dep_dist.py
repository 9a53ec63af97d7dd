#!/usr/bin/env python3
"""Dependency distance histogram of the VALU stream of one kernel in a hipcc
-save-temps .s file: for each VALU instruction, how many VALU instructions
back its nearest source VGPR was written (1 = the previous one).  A wave
issues a VALU op at most every 4 cycles and a dependent op waits the
producer's latency, so at two waves per SIMD short distances stall the SIMD.
usage: dep_dist.py file.s kernel_substring"""
import re
import sys
from collections import Counter

REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs(text):
    out = []
    for m in REG.finditer(text):
        if m.group(1):
            out.append(int(m.group(1)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines, on = [], False
    for ln in open(path):
        if not on and not ln[:1].isspace() and name in ln and ":" in ln and not ln.startswith("."):
            on = True
            continue
        if on:
            if "s_endpgm" in ln:
                break
            lines.append(ln.strip())
    last = {}
    hist = Counter()
    n = 0
    for ln in lines:
        if not ln.startswith("v_"):
            continue
        parts = ln.split(None, 1)
        if len(parts) < 2:
            continue
        ops = parts[1].split(",")
        dst, srcs = regs(ops[0]), regs(",".join(ops[1:]))
        d = min((n - last[r] for r in srcs if r in last), default=99)
        hist[min(d, 8)] += 1
        for r in dst:
            last[r] = n
        n += 1
    tot = sum(hist.values())
    print(f"{n} VALU instructions; nearest-producer distance: " +
          " ".join(f"{k if k < 8 else '8+'}:{100 * v / tot:.1f}%" for k, v in sorted(hist.items())))


if __name__ == "__main__":
    main()
