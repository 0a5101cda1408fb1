#!/usr/bin/env python3
"""Per-kernel times of the batched path for a few (N, effect, scale) at 1024 channels x 10 s:
how much the pitch map (synthesis MODE 2) costs against a stretch (MODE 0) of the same N.
Diagnostic (not a bench line)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-vocoder_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import pv_frames, synth_channels  # noqa: E402
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder  # noqa: E402


def run(N, effect, scale, C=1024, n=441000, steps=10):
    x = synth_channels(torch, C, n, 20240, torch.device("cuda:0"))
    pv = PhaseVocoder(N, effect, scale, 4, mode=STANDARD, max_channels=C, max_frames=pv_frames(n, N // 4))
    frames = pv.num_frames(n)
    spec, out = pv.alloc_spec(C, frames), pv.alloc_out(C, frames)
    for _ in range(3):
        pv.process(x, spec=spec, out=out)
    torch.cuda.synchronize()
    pv.profile(True)
    pv.profile_reset()
    for _ in range(steps):
        pv.process(x, spec=spec, out=out)
    torch.cuda.synchronize()
    prof = pv.profile_read()
    pv.profile(False)
    ks = " ".join(f"{k}={v[0] / max(v[1], 1):.3f}" for k, v in prof.items())
    print(f"N={N} {effect}{scale}: {ks}", flush=True)


for N, eff, sc in [(2048, PITCH_SHIFT, 1.5), (2048, TIME_SHIFT, 1.0), (2048, PITCH_SHIFT, 2.0),
                   (1024, PITCH_SHIFT, 1.5), (1024, TIME_SHIFT, 0.5)]:
    run(N, eff, sc)
