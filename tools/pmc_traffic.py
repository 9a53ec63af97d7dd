#!/usr/bin/env python3
"""HBM traffic per launch of the encode / decode kernels from rocprofv3 PMC passes.

GPU box:  KB_ARGS="128 128 65536" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE
          python3 tools/pmc_traffic.py 128 128 65536 gpurun_out/pmc1 gpurun_out/pmc2 > profiles/<round>/pmc_traffic.json
Batched launches:  PMC_TOOL=bbench KB_ARGS="128 128 65536 16" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE
          python3 tools/pmc_traffic.py --objects 16 128 128 65536 gpurun_out/pmc1 gpurun_out/pmc2

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of coalesced streaming reads (MI355X_MICROARCH.md, HBM section),
so HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  For these kernels the x2
calibration checks out against the algorithmic read bytes (one dword per lane
per piece, every piece read once).  bench.py reports it as roofline.traffic."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def kernel_kind(name):
    # the GF(2^8) encoder tile also runs full-loss decodes of K = R = m codes:
    # its last template argument is the form (rs_args.h: 1 dense encode, 2 dense decode)
    m = re.search(r"k_ff8_bs_slab<([^>]*)>", name)  # bit-sliced dense tile: form (first argument) 1 encode, 2 decode
    if m:
        return "decode" if m.group(1).split(",")[0].strip() == "2" else "encode"
    m = re.search(r"k_ff8_enc(?:_slab|_batch)?<([^>]*)>", name)
    if m:
        return "decode" if m.group(1).split(",")[-1].strip() == "2" else "encode"
    if "k_enc" in name:
        return "encode"
    if "k_ff8_dec" in name or "k_dec" in name:
        return "decode"
    return None


def main():
    args = sys.argv[1:]
    objects = 1
    if args[0] == "--objects":  # batched launches (tools/bbench.py): bytes of every object of a launch
        objects = int(args[1])
        args = args[2:]
    k, r, b = (int(x) for x in args[:3])
    dirs = args[3:]
    loss = calls = None
    while dirs and dirs[0].startswith("--"):
        opt, val = dirs[0][2:].split("=", 1)
        if opt == "loss":  # originals lost in the decode (its algorithmic bytes)
            loss = int(val)
        elif opt == "calls":  # calls of each kind in the run: bytes per call = all dispatches' bytes / calls
            calls = int(val)
        dirs = dirs[1:]
    # per kernel (a call of a multi-pass path launches each of its kernels once):
    # average over dispatches, then the call's bytes = sum over its kernels
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(d.rstrip("/") + "/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                kind = kernel_kind(row["Kernel_Name"])
                if kind is None:
                    continue
                if k + r > 256 and "k_ff8_" in row["Kernel_Name"]:
                    continue  # a GF(2^16) shape: the tool's GF(2^8) warm-up launches are not its kernels
                name = re.sub(r"^.*::(k_\w+<[^>]*>).*$", r"\1", row["Kernel_Name"])
                vals[(kind, name)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for (kind, name), cs in sorted(vals.items()):
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        e = out.setdefault(kind, {"kernel": "", "FETCH_SIZE_KiB": 0.0, "WRITE_SIZE_KiB": 0.0, "dispatches": 0,
                                  "hbm_bytes_per_launch": 0})
        e["kernel"] = (e["kernel"] + " + " if e["kernel"] else "") + name
        e["FETCH_SIZE_KiB"] = round(e["FETCH_SIZE_KiB"] + fetch, 1)
        e["WRITE_SIZE_KiB"] = round(e["WRITE_SIZE_KiB"] + write, 1)
        e["dispatches"] += len(cs["FETCH_SIZE"])
        if calls:  # several dispatches of a kernel per call (column slices): total / calls
            e["hbm_bytes_per_launch"] += int((2 * sum(cs["FETCH_SIZE"]) + sum(cs["WRITE_SIZE"])) * 1024 / calls)
        else:
            e["hbm_bytes_per_launch"] += int((2 * fetch + write) * 1024)
    for kind, e in out.items():
        # encode (K + R) * B; decode (K_surv + R_recv + lost) * B, which is
        # (K + loss) * B when exactly `loss` recovery pieces are received (the benchmark's pattern)
        if kind == "decode":
            # originals lost in the counted decodes (kbench.py: the first min(K, R)); bench.py
            # attaches these bytes only to a decode of the same kernels and loss count
            e["loss"] = loss if loss is not None else min(k, r)
        if kind == "decode" and loss is not None:
            e["algorithmic_bytes_per_launch"] = objects * (k + loss) * b
        else:
            e["algorithmic_bytes_per_launch"] = objects * (k + r) * b
    key = f"{k}+{r}x{b}" + (f"/batch{objects}" if objects > 1 else "")
    print(json.dumps({"workloads": {key: out},
                      "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; (2*FETCH+WRITE) KiB"},
                     indent=1))


if __name__ == "__main__":
    main()
