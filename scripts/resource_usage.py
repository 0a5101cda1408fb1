#!/usr/bin/env python3
"""Summarise `make resource-usage` remarks: one line per kernel (VGPR, AGPR, spills,
occupancy, LDS).  Usage: make -C phase-vocoder_amd/csrc resource-usage 2>&1 | python3 scripts/resource_usage.py"""
import re
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    body = m.group(1)
    if body.startswith("Function Name:"):
        cur = {"name": body.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "Occupancy [waves/SIMD]"]
for r in rows:
    n = r["name"].replace("_ZN2pv", "").replace("EEEvNS_", "|").split("|")[0]
    print(f"{n:40s} " + " ".join(f"{k.split()[0][:5]}{'-sp' if 'Spill' in k else ''}={r.get(k, '?'):>4s}" for k in keys))
