#!/usr/bin/env python3
"""Per-dispatch averages of every counter in rocprofv3 counter_collection CSVs
under a directory, grouped by kernel: python tools/pmc_summary.py gpurun_out/k3v0"""
import collections
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        continue
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"]].append(r)
    for kern, rs in sorted(by.items()):
        agg = collections.defaultdict(float)
        for r in rs:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp = len(set(r["Dispatch_Id"] for r in rs))
        print(f, "dispatches", disp, "kernel", kern[:90], "vgpr", rs[0]["VGPR_Count"],
              "agpr", rs[0].get("Accum_VGPR_Count"), "lds", rs[0]["LDS_Block_Size"])
        for k, v in sorted(agg.items()):
            print(f"   {k:36s} {v / disp:.4g}")
