#!/usr/bin/env python3
"""Per (kernel, grid) average duration from a rocprofv3 kernel_trace.csv, the
idle gap after each library kernel, and for runs of consecutive launches whose
name contains BUSY (default k_ff8_bs_slab; no other kernel between them) the
GPU time per launch, (last end - first start) / launches, beside the mean
kernel duration: the two differ when launches on two streams overlap."""
import os
import csv
import sys
from collections import defaultdict


def main():
    for f in sys.argv[1:]:
        agg = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "lamd" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].replace("lamd::(anonymous namespace)::", "").replace("lamd::", "")
            name = name.split("(")[0] if "(" in name else name
            grid = (r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Grid_Size_Y", ""), r.get("Workgroup_Size_X", r.get("Workgroup_Size")))
            agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f)
        for (name, grid), v in sorted(agg.items()):
            v.sort()
            print(f"  {name:40s} grid={grid} n={len(v):4d} avg={sum(v)/len(v):8.2f} us  med={v[len(v)//2]:8.2f}")
        # idle time from a library kernel's end to the next kernel's start (any kernel)
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        gaps = defaultdict(list)
        for a, b in zip(rows, rows[1:]):
            if "lamd" not in a["Kernel_Name"]:
                continue
            name = a["Kernel_Name"].replace("lamd::(anonymous namespace)::", "").split("(")[0]
            gaps[name].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
        for name, v in sorted(gaps.items()):
            v.sort()
            print(f"  gap after {name:32s} n={len(v):4d} med={v[len(v)//2]:8.2f} us  (negative: the next kernel started first)")
        key = os.environ.get("BUSY", "k_ff8_bs_slab")
        runs, cur = [], []
        for r in rows:
            if key in r["Kernel_Name"]:
                cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            elif cur:
                runs.append(cur)
                cur = []
        if cur:
            runs.append(cur)
        for run in runs:
            if len(run) < 4:
                continue
            busy = (max(e for _, e in run) - run[0][0]) / len(run) / 1e3
            span = sum(e - s for s, e in run) / len(run) / 1e3
            print(f"  run of {len(run):4d} {key} launches: GPU time per launch {busy:8.2f} us, "
                  f"mean kernel duration {span:8.2f} us")


if __name__ == "__main__":
    main()
