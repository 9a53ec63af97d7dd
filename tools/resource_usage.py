#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output per kernel."""
import re, subprocess, sys

def main():
    src = sys.argv[1]
    extra = sys.argv[2:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
           "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: +(.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
        name = name.replace("lamd::(anonymous namespace)::", "").replace("lamd::", "")
        print(f"{name[:60]:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} sgpr={r.get('SGPRs','?'):>3} "
              f"scratch={r.get('ScratchSize [bytes/lane]','?'):>5} vspill={r.get('VGPRs Spill','?'):>5} "
              f"sspill={r.get('SGPRs Spill','?'):>4} occ={r.get('Occupancy [waves/SIMD]','?')} lds={r.get('LDS Size [bytes/block]','?')}")

if __name__ == "__main__":
    main()
