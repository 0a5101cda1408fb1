"""The single-launch chained path for output-phase ratios p/2^e > 1 (pv_chain.hip, opt-in
with PV_CHAIN=1; BASELINE config 3 is time stretch 0.5, q = 2): the split path's spectrum and output bit for bit at
equal run length, the oracle's output within 1e-5 RMS, repeated launches on one handle (the
run-group records are tagged per launch), ragged / short inputs, unaligned input (falls
back to the split path), and no timed-out hand-off (pv_check_device)."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from test_gpu_parity import RMS_TOL, rms, synth, to_dev

pytestmark = pytest.mark.gpu


def pv_frames(n, hop):
    return max(1, -(-(n - hop) // hop))


def _run(pv, x, **kw):
    pv.profile(True)
    pv.profile_reset()
    out, spec = pv.process(x, **kw)
    prof = pv.profile_read()
    pv.profile(False)
    pv.check_device()
    return out, spec, prof


CASES = [
    (1024, 4, TIME_SHIFT, 0.5),    # config 3: L = 512, hop 256 (D = 2), out hop 128 (DT = 1)
    (1024, 4, PITCH_SHIFT, 1.5),   # config 4's ratio at N = 1024: out hop 256 (DT = 2)
    (1024, 8, PITCH_SHIFT, 1.5),   # hop 128 (D = 1), out hop 128 (DT = 1)
    (512, 2, TIME_SHIFT, 0.5),     # L = 256, hop 256 (D = 2), out hop 128 (DT = 1)
    (512, 4, PITCH_SHIFT, 1.25),   # L = 256, hop 128 (D = 1), q = 4
    (1024, 4, PITCH_SHIFT, 0.75),  # ratio < 1: several sources per bin, q = 4
    (512, 4, TIME_SHIFT, 1.5),     # out hop 192: outside the chained kernels -> split path
]


@pytest.mark.parametrize("N,hop_div,effect,scale", CASES)
def test_chain_equals_split_path(cuda, monkeypatch, N, hop_div, effect, scale):
    """Chained vs PV_CHAIN=0 at the same run length: spectra and outputs bit-identical
    (exact integer carries, same per-frame operations, same seam sums); both within 1e-5
    RMS of the oracle."""
    C, n = 3, 90000
    hop = N // hop_div
    xs = np.stack([synth(n, 500 + c) for c in range(C)])
    xd = to_dev(xs)
    frames = pv_frames(n, hop)
    monkeypatch.setenv("PV_CHAIN", "1")
    monkeypatch.setenv("PV_CHAIN_FRAMES", "16")
    pc = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
    out_c, spec_c, prof_c = _run(pc, xd)
    monkeypatch.setenv("PV_CHAIN", "0")
    monkeypatch.setenv("PV_RUN_FRAMES", str(pc.single_launch_frames if pc.single_launch == 2 else pc.frames_per_run))
    ps = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
    out_s, spec_s, prof_s = _run(ps, xd)
    assert ps.single_launch == 0 and "chain" not in prof_s
    if pc.single_launch == 2:
        assert prof_c.get("chain", (0, 0))[1] == 1
        assert "analysis" not in prof_c and "synthesis" not in prof_c and "carry" not in prof_c
        assert pc.single_launch_frames == ps.frames_per_run == 16
    else:  # geometry outside the chained kernel's instantiations: the split path
        assert "chain" not in prof_c
    B = N // 2 + 1
    assert np.array_equal(spec_c.cpu().numpy().view(np.uint32)[:, :frames, :B],
                          spec_s.cpu().numpy().view(np.uint32)[:, :frames, :B])
    gc, gs = out_c.cpu().numpy(), out_s.cpu().numpy()
    assert np.array_equal(gc.view(np.uint32), gs.view(np.uint32))
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord(effect), scale)
    for c in range(C):
        assert rms(gc[c], ref[c]) <= RMS_TOL, f"ch{c}"


def test_chain_config3_slice_vs_oracle_and_repeat(cuda, monkeypatch):
    """Config 3's geometry on 24 channels x 10 s (1722 frames = 108 runs of 16 per
    channel, 27 run groups chained): every channel within 1e-5 RMS of the oracle, the
    spectrum's phases bit-exact, and three launches on one handle bit-identical (stale
    run-group records of an earlier launch are never taken)."""
    monkeypatch.setenv("PV_CHAIN", "1")
    monkeypatch.setenv("PV_CHAIN_FRAMES", "16")
    C, n = 24, 441000
    xs = np.stack([synth(n, 20240 + c) for c in range(C)])
    xd = to_dev(xs)
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_channels=C, max_frames=pv_frames(n, 256))
    assert pv.single_launch == 2
    out, spec, prof = _run(pv, xd)
    assert prof.get("chain", (0, 0))[1] == 1
    frames = pv.num_frames(n)
    assert frames == 1722
    g = out.cpu().numpy()
    assert np.isfinite(g).all()
    ref, _ = pvref.std_process_batch(xs, 1024, 4, ord("t"), 0.5)
    for c in range(C):
        assert rms(g[c], ref[c]) <= RMS_TOL, f"ch{c}"
    for c in (0, C - 1):
        _, ph = pvref.std_analysis(xs[c], 1024, 256, frames)
        assert np.array_equal(spec[c, :frames, :513, 1].cpu().numpy().view(np.uint32), ph.view(np.uint32))
    for _ in range(2):
        again, _, _ = _run(pv, xd)
        assert np.array_equal(again.cpu().numpy().view(np.uint32), g.view(np.uint32))


def test_chain_fewer_channels_after_more(cuda, monkeypatch):
    """A handle reused with fewer channels and frames than its capacity (the ticket ->
    (run group, channel) map follows the call, not the capacity)."""
    monkeypatch.setenv("PV_CHAIN", "1")
    C, n = 6, 60000
    xs = np.stack([synth(n, 900 + c) for c in range(C)])
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_channels=C, max_frames=pv_frames(n, 256))
    _run(pv, to_dev(xs))
    m = 25000
    sub = np.ascontiguousarray(xs[:2, :m])
    out, _, _ = _run(pv, to_dev(sub))
    ref, _ = pvref.std_process_batch(sub, 1024, 4, ord("t"), 0.5)
    g = out.cpu().numpy()
    for c in range(2):
        assert rms(g[c], ref[c]) <= RMS_TOL


@pytest.mark.parametrize("n", [700, 1000, 1023, 1024, 1300, 5000, 17000])
def test_chain_short_and_ragged(cuda, monkeypatch, n):
    """Inputs shorter than a frame, ending inside a frame, one partial run group."""
    monkeypatch.setenv("PV_CHAIN", "1")
    x = synth(n, 13)
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=128)
    frames = pv.num_frames(n)
    if frames == 0:
        return
    out, _, _ = _run(pv, to_dev(x))
    ref = pvref.std_process(x, 1024, 4, ord("t"), 0.5)
    g = out.cpu().numpy()[0]
    assert g.shape == ref.shape and rms(g, ref) <= RMS_TOL


def test_chain_unaligned_input_takes_split_path(cuda, monkeypatch):
    """An input view at an odd float offset cannot take the vector loads of the chained
    analysis: pv_process runs the split path instead, with the same result."""
    monkeypatch.setenv("PV_CHAIN", "1")
    import torch
    C, n = 2, 40001
    xs = np.stack([synth(n, 80 + c) for c in range(C)])
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_channels=C, max_frames=200)
    xbig = torch.zeros(C, n + 1, device="cuda")
    xbig[:, 1:] = to_dev(xs)
    out, _, prof = _run(pv, xbig[:, 1:], n_samples=n)
    assert "chain" not in prof and prof.get("analysis", (0, 0))[1] == 1
    ref, _ = pvref.std_process_batch(xs, 1024, 4, ord("t"), 0.5)
    for c in range(C):
        assert rms(out[c].cpu().numpy(), ref[c]) <= RMS_TOL
