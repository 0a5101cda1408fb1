#!/usr/bin/env python3
"""Average duration of each pv:: kernel over the LAST `steps` dispatches of a rocprofv3
kernel trace (the timed region of bench.py: warmup dispatches excluded), to set beside
bench.py's hipEvent averages.  usage: prof_timed.py run_kernel_trace.csv [steps]"""
import csv
import json
import sys
from collections import defaultdict

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if "pv::" not in n:
        continue
    d[n.split("(")[0].replace("void ", "")].append(
        (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
out = {}
for k, v in d.items():
    v.sort()
    last = [dur for _, dur in v[-steps:]]
    out[k] = {"dispatches": len(v), "timed": len(last), "avg_ms": sum(last) / len(last) / 1e6}
print(json.dumps(out, indent=1))
