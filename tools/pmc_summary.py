#!/usr/bin/env python3
"""Average PMC counter values per kernel from rocprofv3 --pmc csv outputs."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    dirs = sys.argv[1:] or sorted(glob.glob("gpurun_out/pmc*/"))
    agg = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(d.rstrip("/") + "/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"]
                if "lamd" not in name:
                    continue
                short = name.replace("lamd::(anonymous namespace)::", "").replace("lamd::", "").split("(")[0][:60]
                short += f"  grid={row.get('Grid_Size', '')}"
                agg[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in agg.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
