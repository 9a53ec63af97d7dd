#!/usr/bin/env python3
"""Per (kernel, grid) average duration from a rocprofv3 kernel_trace.csv."""
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


if __name__ == "__main__":
    main()
