#!/usr/bin/env python3
"""Round 5 diagnostic: minimax fits of atan(a) = a P(a^2) on [0, 1] with 8 and 9 fp32
coefficients (linear programming, scipy HiGHS), each evaluated through the contract's fp32
atan2 (atan2_eval.c: seed + cubic + Newton reciprocal, Horner in fmaf, octant fix-ups) over
2e7 random bins.  Result: 8 coefficients 3.5e-7 rad worst, 9
coefficients 3.1e-7, the contract's 10: 2.95e-7 — the 3e-7 bound holds only with 10.
  gcc -O2 -ffp-contract=off -o /tmp/atan2_eval scripts/atan_fit/atan2_eval.c -lm
  python3 scripts/atan_fit/fit.py /tmp/atan2_eval"""
import subprocess
import sys

import numpy as np
from scipy.optimize import linprog


def fit(ncoef, npts=6000, scale=1e6):
    a = np.linspace(0, 1, npts)
    s = a * a
    f = np.arctan(a)
    A = np.stack([a * s ** j for j in range(ncoef)], 1) * scale
    n = ncoef
    c = np.zeros(n + 1)
    c[-1] = 1
    Aub = np.vstack([np.hstack([A, -np.ones((len(a), 1))]), np.hstack([-A, -np.ones((len(a), 1))])])
    bub = np.concatenate([f * scale, -f * scale])
    Aeq = np.zeros((1, n + 1))
    Aeq[0, 0] = scale
    r = linprog(c, A_ub=Aub, b_ub=bub, A_eq=Aeq, b_eq=[scale], bounds=[(None, None)] * (n + 1), method="highs")
    return r.x[:n], r.x[n] / scale


if __name__ == "__main__":
    ev = sys.argv[1] if len(sys.argv) > 1 else None
    contract = ["0x1.000000p+0", "-0x1.5554eep-2", "0x1.9986ecp-3", "-0x1.23c87ap-3", "0x1.bd9028p-4",
                "-0x1.506f6cp-4", "0x1.c2c9f4p-5", "-0x1.d2ca58p-6", "0x1.398008p-7", "-0x1.8ba68ap-10"]
    if ev:
        print("contract (10):", subprocess.run([ev] + contract, capture_output=True, text=True).stdout.strip())
    for n in (8, 9):
        co, t = fit(n)
        h = [float(np.float32(x)).hex() for x in co]
        print(n, "coefficients: minimax", t, h)
        if ev:
            print("   ", subprocess.run([ev] + h, capture_output=True, text=True).stdout.strip())
