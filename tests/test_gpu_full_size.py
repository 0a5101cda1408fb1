"""Parity at BASELINE.json's full sizes through size-independent properties (the oracle
cannot redo a 1.7-million-frame batch in a test): the per-GPU workloads of configs 2, 3 and
4 run whole, and

* every output sample is finite and the output has exactly pv_output_length samples, the
  length the oracle's output has too (no truncation before the comparison);
* a channel's result does not depend on the batch it is in: channels run alone, and the
  upper half of the channels run as their own batch (what one rank of the multi-GPU shard
  does), equal the full batch bit for bit at the same run length (PV_RUN_FRAMES: the run
  length sets where the overlap-add sums are split into run seams, so it sets their
  rounding);
* a second run is bit-identical (no atomics, no order-dependent reductions);
* 16 channels spread over the batch (first and last included, bench.py's check_channels)
  match the CPU oracle within the north_star tolerance;
* spectrum magnitudes are >= 0 and phases lie in [-pi, pi]."""
import os
import sys

import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from pvamd import _lib
from test_gpu_parity import RMS_TOL, rms

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import check_channels, cpu_share, synth_channels_np  # noqa: E402

pytestmark = pytest.mark.gpu

WORKLOADS = {  # BASELINE configs: (N, effect, scale, channels per GPU, seconds)
    "c3": (1024, TIME_SHIFT, 0.5, 1024, 10.0),
    "c4": (2048, PITCH_SHIFT, 1.5, 1024, 10.0),
    "c2": (1024, PITCH_SHIFT, 2.0, 1, 60.0),
}


@pytest.mark.parametrize("wl", ["c3", "c4", "c2"])
def test_full_size_properties(cuda, monkeypatch, wl):
    import torch
    N, effect, scale, C, seconds = WORKLOADS[wl]
    n = int(round(seconds * 44100))
    hop = N // 4
    x_host = synth_channels_np(C, n, 20240, cpu_share()[0])
    x = torch.from_numpy(x_host).cuda()
    frames_max = n // hop + 2
    pv = PhaseVocoder(N, effect, scale, 4, mode=STANDARD, max_channels=C, max_frames=frames_max,
                      spec_layout=_lib.PV_SPEC_PACKED)
    fr = pv.num_frames(n)
    spec, out = pv.alloc_spec(C, fr), pv.alloc_out(C, fr)
    pv.process(x, spec=spec, out=out)
    torch.cuda.synchronize()
    olen = pv.output_length(fr)
    hs = pv.outHopSize
    assert olen == fr * hs + (N - hs)         # the full overlap-add length (pv.h pv_output_length)
    assert out.shape == (C, olen)
    full = out
    assert bool(torch.isfinite(full).all())
    ref_bits = full.cpu().numpy().view(np.uint32).copy()

    # determinism: a second run, same buffers
    pv.process(x, spec=spec, out=out)
    torch.cuda.synchronize()
    assert np.array_equal(out[:, :olen].cpu().numpy().view(np.uint32), ref_bits)

    # spectrum ranges (packed rows: slot 0 of lane 0 carries two sign-coded real bins)
    sp = pv.unpack_spec(spec)[:, :fr]
    assert bool((sp[..., 0] >= 0).all())
    assert bool((sp[..., 1].abs() <= np.float32(np.pi)).all())

    # batch independence: single channels, and the upper half as its own batch, at the
    # batch's run length
    monkeypatch.setenv("PV_RUN_FRAMES", str(pv.frames_per_run))
    for c in sorted({0, C // 2, C - 1}):
        one = PhaseVocoder(N, effect, scale, 4, mode=STANDARD, max_channels=1, max_frames=frames_max,
                           spec_layout=_lib.PV_SPEC_PACKED)
        o1, _ = one.process(x[c:c + 1].contiguous())
        assert np.array_equal(o1[0, :olen].cpu().numpy().view(np.uint32), ref_bits[c]), f"channel {c}"
    if C > 1:
        h = C // 2
        half = PhaseVocoder(N, effect, scale, 4, mode=STANDARD, max_channels=C - h, max_frames=frames_max,
                            spec_layout=_lib.PV_SPEC_PACKED)
        oh, _ = half.process(x[h:].contiguous())
        assert np.array_equal(oh[:, :olen].cpu().numpy().view(np.uint32), ref_bits[h:])

    # the oracle on 16 channels spread over the batch, whole rows (same length, no truncation)
    idx = check_channels(C)
    ref, _ = pvref.std_process_batch(x_host[idx], N, 4, ord(effect), scale, fr, cpu_share()[0])
    g = full[idx].cpu().numpy()
    assert ref.shape == g.shape == (len(idx), olen)
    for j, c in enumerate(idx):
        assert rms(g[j], ref[j]) <= RMS_TOL, f"channel {c}"
