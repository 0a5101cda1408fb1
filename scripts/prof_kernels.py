#!/usr/bin/env python3
"""Standalone driver for rocprofv3 counter passes: config 3 (1024 ch x 10 s, N=1024,
hop=256, PV_STANDARD stretch 0.5, packed rows as bench.py) through pv_process, `--reps`
times; --N / --effect / --scale / --mode / --layout select the other workloads."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-vocoder_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--channels", type=int, default=1024)
    ap.add_argument("--effect", default="t")
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--mode", default="standard")
    ap.add_argument("--calib", action="store_true")
    ap.add_argument("--layout", choices=["packed", "natural"], default="packed")
    ap.add_argument("--n", type=int, default=441000, help="samples per channel (c2: 2646000)")
    ap.add_argument("--write-spec", action="store_true",
                    help="hand the spectrum back (bench.py's --write-spec); by default STANDARD "
                         "runs as bench.py does, without (REF_COMPAT always writes the caller's rows)")
    args = ap.parse_args()
    import torch
    from bench import synth_channels_np
    from pvamd import PhaseVocoder
    from pvamd._lib import PV_SPEC_NATURAL, PV_SPEC_PACKED
    n = args.n
    layout = PV_SPEC_PACKED if (args.layout == "packed" and args.mode == "standard") else PV_SPEC_NATURAL
    pv = PhaseVocoder(args.N, args.effect, args.scale, 4, mode=args.mode,
                      max_channels=args.channels, max_frames=n // (args.N // 4) + 2, spec_layout=layout)
    # host-generated input + plain copy: no torch compute kernels in the profiled process
    x = torch.from_numpy(synth_channels_np(args.channels, n, 20240)).to("cuda:0")
    frames = pv.num_frames(n)
    want = args.write_spec or args.mode != "standard"
    spec = pv.alloc_spec(args.channels, frames) if want else None
    out = pv.alloc_out(args.channels, frames)
    for _ in range(args.reps):
        pv.process(x, spec=spec, out=out, spectrum=want)
    torch.cuda.synchronize()
    if args.calib:
        # traffic calibration: the batched FFT reads and writes exactly 8*n*batch bytes with
        # the same 8-byte-per-lane global loads / stores as the phase-vocoder kernels
        from pvamd.fft import fft
        a = torch.zeros((131072, 512), dtype=torch.complex64, device="cuda:0")
        b = torch.empty_like(a)
        for _ in range(args.reps):
            fft(a, out=b)
        torch.cuda.synchronize()
        print("calib bytes", a.numel() * 8)
    print("done", frames)


if __name__ == "__main__":
    main()
