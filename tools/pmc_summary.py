#!/usr/bin/env python3
"""Per-dispatch averages of every counter in rocprofv3 counter_collection CSVs
under a directory: python tools/pmc_summary.py gpurun_out/k3v0"""
import collections
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        continue
    agg = collections.defaultdict(float)
    for r in rows:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
    disp = len(set(r["Dispatch_Id"] for r in rows))
    print(f, "dispatches", disp, "kernel", rows[0]["Kernel_Name"][:60], "vgpr", rows[0]["VGPR_Count"],
          "agpr", rows[0].get("Accum_VGPR_Count"), "lds", rows[0]["LDS_Block_Size"])
    for k, v in sorted(agg.items()):
        print(f"   {k:36s} {v / disp:.4g}")
