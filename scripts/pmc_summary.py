#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: per kernel, mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        key = (row["Dispatch_Id"], row["Counter_Name"])
        vals[k][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
for k, cs in vals.items():
    print(k)
    for c, lst in sorted(cs.items()):
        per = defaultdict(float)
        for d, v in lst:
            per[d] += v  # sum over dimensions (XCD/SE/...) within a dispatch
        mean = sum(per.values()) / len(per)
        print(f"   {c:24s} {mean:16.4g}   ({len(per)} dispatches)")
