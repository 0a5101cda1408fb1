#!/usr/bin/env python3
"""In-kernel clock of the analysis kernel (MI355X_MICROARCH.md, DVFS give-back item 6):
Δs_memtime / Δs_memrealtime × 100 MHz stamped by every wave around its frame loop, in a
diagnostic build only (make -C phase-vocoder_amd/csrc variant NAME=clk DEFS=-DPV_CLOCK_PROBE;
the product kernel executes no stamp).  Runs the config-3 batch back to back for >= 2 s on
random-phase synthetic data first, then reads the stamps of the last analysis launch.

  PV_LIB_PATH=phase-vocoder_amd/build/variants/libpv_clk.so python scripts/clock_stamp.py [c3|c4] [random|zeros]

"zeros" runs the same instruction stream on all-zero input (MI355X_MICROARCH.md DVFS item 1:
less switching energy per instruction): a power-capped kernel then holds a higher clock
and runs faster at unchanged cycles; a latency- or bandwidth-bound one does not.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-vocoder_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import synth_channels_np, cpu_share
    from pvamd import PhaseVocoder, STANDARD, TIME_SHIFT, PITCH_SHIFT, _lib
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    N, eff, scale = (1024, TIME_SHIFT, 0.5) if wl == "c3" else (2048, PITCH_SHIFT, 1.5)
    C, n = 1024, 441000
    data = sys.argv[2] if len(sys.argv) > 2 else "random"
    if data == "zeros":
        x = torch.zeros(C, n, device="cuda")
    else:
        x = torch.from_numpy(synth_channels_np(C, n, 20240, cpu_share()[0])).cuda()
    pv = PhaseVocoder(N, eff, scale, 4, mode=STANDARD, max_channels=C, max_frames=1722)
    spec, out = pv.alloc_spec(C, pv.num_frames(n)), pv.alloc_out(C, pv.num_frames(n))
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < 3.0:
        pv.process(x, spec=spec, out=out)
        torch.cuda.synchronize()
        steps += 1
    dt = (time.perf_counter() - t0) / steps
    L = _lib.lib()
    L.pv_debug_clock.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    nruns = -(-pv.num_frames(n) // pv.frames_per_run)
    buf = np.zeros(2 * C * nruns, np.uint64)
    _lib.check(L.pv_debug_clock(pv._h, buf.ctypes.data, buf.size), "pv_debug_clock")
    dm, dr = buf[0::2].astype(np.float64), buf[1::2].astype(np.float64)
    ok = dr > 0
    ghz = dm[ok] / dr[ok] * 0.1
    print(json.dumps({"workload": wl, "data": data, "waves": int(ok.sum()), "steps": steps, "ms_per_step": dt * 1e3,
                      "clock_GHz_median": float(np.median(ghz)), "clock_GHz_p10": float(np.percentile(ghz, 10)),
                      "clock_GHz_p90": float(np.percentile(ghz, 90)),
                      "wave_loop_us_median": float(np.median(dr[ok]) * 0.01)}))


if __name__ == "__main__":
    main()
