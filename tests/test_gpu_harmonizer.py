"""GPU parity of the harmoniser (pv_harmon*, README.md:50 "multiple pitch shifts on a
single input"): every voice equals the CPU oracle's pitch shift of the input and the
GPU's own single-voice pv_process, bit for bit; the mix is the gain-weighted sum."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, Harmonizer, PhaseVocoder

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5


def synth(n, seed, sr=44100):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sr
    x = np.zeros(n)
    for _ in range(3):
        x += 0.1 * np.sin(2 * np.pi * rng.uniform(55, 4000) * t + rng.uniform(0, 2 * np.pi))
    x += rng.uniform(-1e-3, 1e-3, n)
    return x.astype(np.float32)


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


@pytest.mark.parametrize("N,ratios", [(1024, [1.25, 1.5, 0.75]), (512, [2.0, 1.0]),
                                      (2048, [1.5, 0.5, 1.125, 1.0])])
def test_harmonizer_voices_and_mix(cuda, monkeypatch, N, ratios):
    import torch
    C = 3
    xs = np.stack([synth(40000, 70 + c) for c in range(C)])
    hz = Harmonizer(N, ratios, 4, max_channels=C, max_frames=400)
    gains = [0.5 / (k + 1) for k in range(len(ratios))]
    voices, mix, _ = hz.harmonize(torch.from_numpy(xs).cuda(), gains=gains)
    v = voices.cpu().numpy()
    # the voices run the split path; a single pv_process would take the fused (integer ratio)
    # launch with its own run length (same values up to the seams, tests/test_gpu_fused.py)
    monkeypatch.setenv("PV_FUSED", "0")
    for k, r in enumerate(ratios):
        pv = PhaseVocoder(N, PITCH_SHIFT, r, 4, mode=STANDARD, max_channels=C, max_frames=400)
        single, _ = pv.process(torch.from_numpy(xs).cuda())
        assert np.array_equal(v[k], single.cpu().numpy()), f"voice {k} differs from pv_process"
        ref = pvref.std_process(xs[1], N, 4, ord("p"), r)
        assert rms(v[k][1], ref) <= RMS_TOL
    want = sum(g * v[k].astype(np.float64) for k, g in enumerate(gains))
    assert np.max(np.abs(mix.cpu().numpy() - want)) <= 1e-6


def test_harmonizer_spectrum_is_the_single_voice_spectrum(cuda, monkeypatch):
    """The shared analysis writes the same rows, bit for bit, as a PhaseVocoder of the
    first voice's ratio (same contract, same kernels)."""
    import torch
    monkeypatch.setenv("PV_FUSED", "0")
    C = 2
    xs = np.stack([synth(30000, 90 + c) for c in range(C)])
    hz = Harmonizer(1024, [1.5, 0.75], 4, max_channels=C, max_frames=300)
    _, mix, spec = hz.harmonize(torch.from_numpy(xs).cuda())
    assert mix is None
    pv = PhaseVocoder(1024, PITCH_SHIFT, 1.5, 4, mode=STANDARD, max_channels=C, max_frames=300)
    _, spec1 = pv.process(torch.from_numpy(xs).cuda())
    a, b = spec.cpu().numpy(), spec1.cpu().numpy()
    bins = 1024 // 2 + 1
    assert np.array_equal(a[:, :, :bins].view(np.uint32), b[:, :, :bins].view(np.uint32))


def test_harmonizer_mix_with_exact_gains(cuda):
    """Gains 2 and 0: the mix is exactly twice voice 0 (a power-of-two scale and an added
    +0 round nothing)."""
    import torch
    xs = synth(25000, 95)[None, :]
    hz = Harmonizer(512, [1.25, 2.0], 4, max_channels=1, max_frames=300)
    voices, mix, _ = hz.harmonize(torch.from_numpy(xs).cuda(), gains=[2.0, 0.0])
    v = voices.cpu().numpy()
    assert np.isfinite(v).all() and np.abs(v[0]).max() > 1e-3
    assert np.array_equal(mix.cpu().numpy(), 2.0 * v[0])


def test_harmonizer_single_voice_and_empty_input(cuda):
    import torch
    x = torch.from_numpy(synth(20000, 97)[None, :]).cuda()
    hz = Harmonizer(1024, [1.5], 4, max_channels=1, max_frames=200)
    voices, mix, _ = hz.harmonize(x, gains=[1.0])
    assert voices.shape[0] == 1
    assert np.array_equal(mix.cpu().numpy(), voices[0].cpu().numpy())
    ref = pvref.std_process(synth(20000, 97), 1024, 4, ord("p"), 1.5)
    assert rms(voices[0, 0].cpu().numpy(), ref) <= RMS_TOL
    # fewer samples than one hop: no frames, empty outputs, no error
    voices, mix, spec = hz.harmonize(x[:, :100], gains=[1.0])
    assert voices.numel() == 0 and mix.numel() == 0 and spec.shape[1] == 0
