"""The single-launch path for output-phase ratios with q = 1 (pv_fused.hip; BASELINE config 2
is pitch 2.0): the same spectrum bit for bit as the split analysis, the split path's output
bit for bit at equal run length, and the oracle's output within 1e-5 RMS — including the
whole 60 s config-2 stream."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from test_gpu_parity import RMS_TOL, rms, synth, to_dev

pytestmark = pytest.mark.gpu


def _kernels(pv, x, **kw):
    pv.profile(True)
    pv.profile_reset()
    out, spec = pv.process(x, **kw)
    prof = pv.profile_read()
    pv.profile(False)
    return out, spec, prof


def test_config2_full_stream(cuda):
    """configs[1] at full size: one 60 s stream (10 335 frames), N=1024 hop=256, pitch 2.0,
    one fused launch (+ the inter-workgroup seams), against the oracle over every sample."""
    n = 60 * 44100
    x = synth(n, 20240)
    pv = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=pv_frames(n))
    out, spec, prof = _kernels(pv, to_dev(x))
    assert prof.get("fused", (0, 0))[1] == 1 and "analysis" not in prof and "synthesis" not in prof
    frames = pv.num_frames(n)
    assert frames == 10335
    g = out.cpu().numpy()[0]
    ref = pvref.std_process(x, 1024, 4, ord("p"), 2.0)
    assert g.shape == ref.shape and np.isfinite(g).all()
    assert rms(g, ref) <= RMS_TOL
    # the spectrum it returns is the contract's analysis: phases bit-exact
    _, ph = pvref.std_analysis(x, 1024, 256, frames)
    s = spec.cpu().numpy()[0, :frames, :513]
    assert np.array_equal(s[..., 1].view(np.uint32), ph.view(np.uint32))


def pv_frames(n, hop=256):
    return max(1, -(-(n - hop) // hop))


@pytest.mark.parametrize("N,hop_div,effect,scale", [
    (1024, 4, PITCH_SHIFT, 2.0),   # config 2 (DT = 2)
    (1024, 4, TIME_SHIFT, 2.0),    # q = 1 stretch: out hop 512 (DT = 4)
    (512, 4, PITCH_SHIFT, 2.0),    # L = 256, out hop 128 (DT = 1)
    (256, 2, PITCH_SHIFT, 3.0),    # L = 128, hop 128, pitch 3
    (1024, 8, PITCH_SHIFT, 2.0),   # hop 128 (DT = 1)
])
def test_fused_equals_split_path(cuda, monkeypatch, N, hop_div, effect, scale):
    """Fused vs PV_FUSED=0 (analysis + synthesis launches) on 3 channels: spectra identical;
    outputs identical when both use the same run length, within 1e-6 otherwise (the seams
    move); both within 1e-5 RMS of the oracle."""
    C, n = 3, 70000
    xs = np.stack([synth(n, 300 + c) for c in range(C)])
    xd = to_dev(xs)
    frames = pv_frames(n, N // hop_div)
    monkeypatch.setenv("PV_FUSED", "0")
    ps = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
    out_s, spec_s, prof_s = _kernels(ps, xd)
    assert "fused" not in prof_s
    monkeypatch.delenv("PV_FUSED")
    pf = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
    out_f, spec_f, prof_f = _kernels(pf, xd)
    assert prof_f.get("fused", (0, 0))[1] == 1
    assert np.array_equal(spec_f.cpu().numpy().view(np.uint32)[:, :frames, :N // 2 + 1],
                          spec_s.cpu().numpy().view(np.uint32)[:, :frames, :N // 2 + 1])
    gf, gs = out_f.cpu().numpy(), out_s.cpu().numpy()
    assert np.abs(gf - gs).max() <= 1e-6
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord(effect), scale)
    for c in range(C):
        assert rms(gf[c], ref[c]) <= RMS_TOL, f"ch{c}"
    # same run length as the split path: bit for bit — for pitch 2 at N >= 512 through the
    # single launch's MODE 3 gather (PV_FUSED_HALF=0); its default half-size resynthesis
    # (MODE 4) is the same sum with other roundings: within 1e-6
    monkeypatch.setenv("PV_FUSED_FRAMES", str(ps.frames_per_run))
    half = effect == PITCH_SHIFT and scale == 2.0 and N >= 512
    pe = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
    out_e, _, _ = _kernels(pe, xd)
    if half:
        assert np.abs(out_e.cpu().numpy() - gs).max() <= 1e-6
        monkeypatch.setenv("PV_FUSED_HALF", "0")  # read by pv_create: a new handle
        pe = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
        out_e, _, _ = _kernels(pe, xd)
    assert np.array_equal(out_e.cpu().numpy().view(np.uint32), gs.view(np.uint32))


@pytest.mark.parametrize("n", [700, 1000, 1023, 1024, 1300, 5000])
def test_fused_short_and_ragged(cuda, n):
    """Inputs shorter than a frame, ending inside a frame, and few-run streams."""
    x = synth(n, 11)
    pv = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=64)
    frames = pv.num_frames(n)
    if frames == 0:
        return
    out, _ = pv.process(to_dev(x))
    ref = pvref.std_process(x, 1024, 4, ord("p"), 2.0)
    g = out.cpu().numpy()[0]
    assert g.shape == ref.shape and rms(g, ref) <= RMS_TOL


def test_fused_odd_output_stride_and_offset_input(cuda):
    """Unaligned input (odd float offset: scalar loads) and an odd output row stride
    (scalar stores): same result as the aligned call, nothing written past the rows."""
    import torch
    C, n = 2, 30001
    xs = np.stack([synth(n, 70 + c) for c in range(C)])
    pv = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_channels=C, max_frames=200)
    frames = pv.num_frames(n)
    olen = pv.output_length(frames)
    xbig = torch.zeros(C, n + 1, device="cuda")
    xbig[:, 1:] = to_dev(xs)
    xo = xbig[:, 1:]
    big = torch.full((C, olen + 1 if olen % 2 == 0 else olen + 2), 7.0, device="cuda")
    out = big[:, :olen]
    assert out.stride(0) % 2 == 1
    spec = pv.alloc_spec(C, frames)
    pv.process(xo, spec=spec, out=out)
    dense, _ = pv.process(to_dev(xs))
    assert torch.equal(out, dense)
    assert torch.all(big[:, olen:] == 7.0)


@pytest.mark.parametrize("N,hop_div,effect,scale", [
    (1024, 4, PITCH_SHIFT, 2.0),   # config 2: bins 257 .. 512 unread (a half-read pair)
    (256, 2, PITCH_SHIFT, 3.0),    # L = 128: only bins 0 .. 42 read (one register)
    (512, 4, PITCH_SHIFT, 2.0),    # L = 256
    (1024, 4, TIME_SHIFT, 2.0),    # stretch: every bin read
])
def test_fused_without_spectrum_output(cuda, N, hop_div, effect, scale):
    """pv_process with spec = NULL on the single launch (SURVEY §8(d) fused mode: the rows
    are consumed on chip, and for pitch > 1 the bins no output bin reads are not analysed):
    the same output bits as with the spectrum written (the split path's form is
    tests/test_gpu_parity.py test_split_path_without_spectrum_output)."""
    import torch
    from pvamd import _lib
    x = synth(44100 * 3, 31)
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_frames=1200)
    assert pv.single_launch
    out1, spec = pv.process(to_dev(x))
    out2, none = pv.process(to_dev(x), spectrum=False)
    assert none is None and spec is not None
    assert torch.equal(out1, out2)
    ref = pvref.std_process(x, N, hop_div, ord(effect), scale)
    assert rms(out2.cpu().numpy()[0], ref) <= RMS_TOL
    assert _lib.lib() is not None


@pytest.mark.parametrize("seconds", [60.0, 20.0, 37.3])
def test_fused_balanced_runs(cuda, monkeypatch, seconds):
    """One long stream whose workgroups do not fill whole rounds of the CUs takes the
    balanced single launch (some runs one frame longer, exactly `rounds` workgroups per CU):
    every sample against the oracle, and within 1e-6 of the uniform-run launch
    (PV_FUSED_BALANCE=0) — only the run seams' rounding moves."""
    import torch
    n = int(seconds * 44100)
    x = synth(n, 20241)
    pv = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=pv_frames(n))
    out, _ = pv.process(to_dev(x), spectrum=False)
    g = out.cpu().numpy()[0]
    ref = pvref.std_process(x, 1024, 4, ord("p"), 2.0)
    assert g.shape == ref.shape and np.isfinite(g).all()
    assert rms(g, ref) <= RMS_TOL
    monkeypatch.setenv("PV_FUSED_BALANCE", "0")  # read by pv_create: a new handle
    pv = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=pv_frames(n))
    out0, _ = pv.process(to_dev(x), spectrum=False)
    assert float((out0 - out).abs().max()) <= 1e-6
    again, _ = pv.process(to_dev(x), spectrum=False)  # deterministic
    assert torch.equal(again, out0)


def test_fused_balanced_runs_same_bits_alone_or_batched(cuda):
    """The balanced run split is decided from the frame count alone: a stream long
    enough to take it gives the same output bits processed alone and as either channel of a
    two-channel batch."""
    import torch
    n = int(37.3 * 44100)
    x0, x1 = synth(n, 20241), synth(n, 20242)
    pv1 = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=pv_frames(n))
    alone0, _ = pv1.process(to_dev(x0), spectrum=False)
    alone1, _ = pv1.process(to_dev(x1), spectrum=False)
    pv2 = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_channels=2, max_frames=pv_frames(n))
    both, _ = pv2.process(to_dev(np.stack([x0, x1])), spectrum=False)
    assert torch.equal(both[0], alone0[0]) and torch.equal(both[1], alone1[0])
