#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs per kernel (sum over dispatches of the named kernel)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_exact"
agg = defaultdict(float)
disp = set()
for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add((f, r["Dispatch_Id"]))
print(f"kernel~{pat}: {len(disp)} dispatch-passes")
for k in sorted(agg):
    print(f"  {k:28s} {agg[k]:.6g}")
