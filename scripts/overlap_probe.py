#!/usr/bin/env python3
"""Does running two channel halves of the config-3 batch on two HIP streams beat running
them back to back?  Diagnostic for the multi-stream pv_process schedule.
Prints ms per full batch for: serial (one handle, all channels), two handles on one stream,
two handles on two streams, K chunks round-robin over two streams."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-vocoder_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import pv_frames, synth_channels  # noqa: E402
from pvamd import STANDARD, TIME_SHIFT, PhaseVocoder  # noqa: E402


def main():
    C, n, N, hd = 1024, 441000, 1024, 4
    chunks = int(os.environ.get("CHUNKS", "4"))
    dev = torch.device("cuda:0")
    x = synth_channels(torch, C, n, 20240, dev)
    mf = pv_frames(n, N // hd)
    full = PhaseVocoder(N, TIME_SHIFT, 0.5, hd, mode=STANDARD, max_channels=C, max_frames=mf)
    frames = full.num_frames(n)
    spec = full.alloc_spec(C, frames)
    out = full.alloc_out(C, frames)
    cc = C // chunks
    hs = [PhaseVocoder(N, TIME_SHIFT, 0.5, hd, mode=STANDARD, max_channels=cc, max_frames=mf)
          for _ in range(chunks)]
    s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def serial():
        full.process(x, spec=spec, out=out)

    def one_stream():
        for i, h in enumerate(hs):
            sl = slice(i * cc, (i + 1) * cc)
            h.process(x[sl], spec=spec[sl], out=out[sl])

    def two_streams():
        cur = torch.cuda.current_stream(dev)
        for st in s:
            st.wait_stream(cur)
        for i, h in enumerate(hs):
            sl = slice(i * cc, (i + 1) * cc)
            h.process(x[sl], spec=spec[sl], out=out[sl], stream=s[i % 2].cuda_stream)
        for st in s:
            cur.wait_stream(st)

    for name, fn in [("serial", serial), ("chunks_one_stream", one_stream),
                     ("chunks_two_streams", two_streams)] * 2:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        print(f"{name:22s} chunks={chunks} {dt * 1e3:.3f} ms  {C * frames / dt:.4g} frames/s", flush=True)


if __name__ == "__main__":
    main()
