#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_session.sh
with scripts/prof_kernels.py --calib) -> profiles/traffic.json, the `roofline.traffic`
bench.py reports.

Units and gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and
WRITE_SIZE are KiB per dispatch (summed over XCDs here); FETCH_SIZE counts half of the
bytes of a coalesced streaming read.  The phase-vocoder kernels use 8-byte-per-lane global
loads/stores, a width the guide leaves uncalibrated, so the factors are measured in the
same run on the batched FFT (pv_fft_c2c, N = 512), which reads and writes exactly
8 * 512 * 131072 bytes with the same access width: fetch_factor = known / FETCH bytes,
write_factor = known / WRITE bytes."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/traffic.json"
CALIB_BYTES = 8 * 512 * 131072
NAMES = {"k_std_analysis": "analysis", "k_synthesis": "synthesis", "k_carry": "carry",
         "k_seam": "seam", "k_runsum": "runsum", "k_compat_analysis": "compat_analysis",
         "k_fft": "fft", "k_fused": "fused"}

per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        c = row["Counter_Name"]
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("pv::", "")
        per[k][c][row["Dispatch_Id"]] += float(row["Counter_Value"])


def mean(d):
    return sum(d.values()) / max(len(d), 1)


fft = [k for k in per if k.startswith("k_fft<512")]
if not fft:
    sys.exit("no k_fft<512> calibration dispatches found (run prof_kernels.py --calib)")
fetch_f = CALIB_BYTES / (mean(per[fft[0]]["FETCH_SIZE"]) * 1024)
write_f = CALIB_BYTES / (mean(per[fft[0]]["WRITE_SIZE"]) * 1024)
res = {"_calibration": {"kernel": fft[0], "known_bytes": CALIB_BYTES,
                        "fetch_factor": fetch_f, "write_factor": write_f,
                        "source": root}}
for k, cs in per.items():
    base = k.split("<")[0]
    name = NAMES.get(base, base)
    rd = mean(cs["FETCH_SIZE"]) * 1024 * fetch_f
    wr = mean(cs["WRITE_SIZE"]) * 1024 * write_f
    res[name if name not in res else k] = {"kernel": k, "read_bytes_per_launch": rd,
                                           "write_bytes_per_launch": wr,
                                           "bytes_per_launch": rd + wr}
res["_layout"] = os.environ.get("PV_TRAFFIC_LAYOUT", "packed")   # its spectrum row layout
wl = os.environ.get("PV_TRAFFIC_WORKLOAD", "c3")                  # what prof_kernels.py ran
# profiles/traffic.json holds one entry per workload: {"c3": {...}, "c4": {...}}
allw = {}
if os.path.exists(out):
    try:
        allw = json.load(open(out))
        if "_workload" in allw:  # the single-workload form of earlier rounds
            allw = {allw["_workload"]: allw}
    except ValueError:
        allw = {}
allw[wl] = res
json.dump(allw, open(out, "w"), indent=1)
print(json.dumps({wl: res}, indent=1))
