#!/usr/bin/env python3
"""Print the key fields of bench JSON lines and rocprofv3 kernel stats (session helper)."""
import csv
import json
import sys

for f in sys.argv[1:]:
    if f.endswith(".csv"):
        for r in csv.DictReader(open(f)):
            if "pv::" in r["Name"]:
                print(f"  {r['Name'][:64]:64s} n={r['Calls']:>4s} avg={float(r['AverageNs']) / 1e6:.4f} "
                      f"min={float(r['MinNs']) / 1e6:.4f} ms")
        continue
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d["roofline"]
    v = r.get("valu") or {}
    chk = d.get("rms_vs_oracle") or {}
    print(f"{f}: value={d['value']:.4g} ms/step={d['ms_per_step']:.4f} dom={r['kernel']} frac={r['frac']:.4f} "
          f"bound={r['bound']} issue={v.get('issue_frac_at_peak_clock')} rms={chk.get('max')}")
    print("  ", {k: round(x["avg_ms"], 4) for k, x in d.get("kernels", {}).items()})
