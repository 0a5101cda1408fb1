"""GPU parity of the HIP path (through the C-ABI) against the CPU oracle."""
import numpy as np
import pytest

import pvref
from pvamd import PhaseVocoder, REF_COMPAT, STANDARD, TIME_SHIFT, PITCH_SHIFT

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5  # BASELINE.json north_star: <= 1e-5 RMS per sample vs the CPU reference


def synth(n, seed, sr=44100, tones=3):
    """configs 2-4 generator: 3 sines f~U[55,4000] Hz, a=0.1, + U(+-1e-3) noise."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sr
    x = np.zeros(n)
    for _ in range(tones):
        f = rng.uniform(55, 4000)
        ph = rng.uniform(0, 2 * np.pi)
        x += 0.1 * np.sin(2 * np.pi * f * t + ph)
    x += rng.uniform(-1e-3, 1e-3, n)
    return x.astype(np.float32)


def to_dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


# (the analysis's frame-loop forms: 1024/4, 512/4, 1024/2, 512/2 the register rotation in
# groups of 4 / 4 / 2 / 2 frames; 1024/8 and 256/4 the mirrored pairs without it; 2048/* the
# L = 1024 per-bin split)
@pytest.mark.parametrize("N,hop_div", [(1024, 4), (2048, 4), (512, 4), (256, 4), (1024, 2), (2048, 8),
                                       (512, 2), (1024, 8)])
def test_std_analysis_bit_exact(cuda, N, hop_div):
    x = synth(20 * N, 7)
    pv = PhaseVocoder(N, TIME_SHIFT, 1.0, hop_div, mode=STANDARD, max_frames=1000)
    spec = pv.analysis(to_dev(x)).cpu().numpy()[0]
    frames = pv.num_frames(len(x))
    mag, ph = pvref.std_analysis(x, N, N // hop_div, frames)
    g_mag, g_ph = spec[:frames, :N // 2 + 1, 0], spec[:frames, :N // 2 + 1, 1]
    assert np.array_equal(g_ph.view(np.uint32), ph.view(np.uint32)), \
        f"phase mismatch: {np.sum(g_ph != ph)} bins, max {np.abs(g_ph - ph).max()}"
    # magnitudes use the hardware square root (<= 1 ulp): at most one
    # unit in the last place from the correctly rounded oracle
    ulp = np.abs(g_mag.view(np.int32).astype(np.int64) - mag.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1, f"mag: {np.sum(ulp > 1)} bins off by more than 1 ulp (max {ulp.max()})"


@pytest.mark.parametrize("effect,scale", [(TIME_SHIFT, 0.5), (TIME_SHIFT, 1.0), (PITCH_SHIFT, 2.0),
                                          (PITCH_SHIFT, 1.5), (PITCH_SHIFT, 0.75), (TIME_SHIFT, 1.5)])
def test_std_process_parity(cuda, effect, scale):
    N, hop_div = 1024, 4
    x = synth(3 * 44100 // 2, 20240)
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_frames=1000)
    out, _ = pv.process(to_dev(x))
    g = out.cpu().numpy()[0]
    ref = pvref.std_process(x, N, hop_div, ord(effect), scale)
    assert g.shape == ref.shape
    err = rms(g, ref)
    assert err <= RMS_TOL, f"rms {err}"


def test_std_process_multichannel(cuda):
    N, hop_div, C = 1024, 4, 5
    xs = np.stack([synth(30000, 20240 + c) for c in range(C)])
    pv = PhaseVocoder(N, TIME_SHIFT, 0.5, hop_div, mode=STANDARD, max_channels=C, max_frames=200)
    out, _ = pv.process(to_dev(xs))
    g = out.cpu().numpy()
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord("t"), 0.5)
    for c in range(C):
        assert rms(g[c], ref[c]) <= RMS_TOL


@pytest.mark.parametrize("N,hop_div,effect,scale,packed", [
    (2048, 4, PITCH_SHIFT, 1.5, True),    # config 4 (packed rows, as bench.py): bins 684 ..
    (2048, 4, PITCH_SHIFT, 1.5, False),   # 1024 unread (2 of 8 pairs and bin L skipped)
    (2048, 8, PITCH_SHIFT, 3.0, False),   # bins above 341 unread
    (2048, 4, PITCH_SHIFT, 0.75, False),  # pitch < 1: every bin read
    (2048, 4, TIME_SHIFT, 0.5, False),    # stretch at L = 1024
    (1024, 4, TIME_SHIFT, 0.5, True),     # config 3 (L = 512: no skip in the kernel)
    (1024, 4, PITCH_SHIFT, 1.5, False),
])
def test_split_path_without_spectrum_output(cuda, N, hop_div, effect, scale, packed):
    """pv_process(spec = NULL) on the split path: the rows go through the handle's own
    buffer and, for pitch > 1, the bins no output bin reads are not analysed — the output is
    the same bits as with a caller-owned spectrum, before and after, on 3 channels; a
    spectrum requested afterwards is complete (every bin, bit-exact phases)."""
    import torch
    C, n = 3, 60000
    xs = np.stack([synth(n, 410 + c) for c in range(C)])
    xd = to_dev(xs)
    frames = pv_frames(n, N // hop_div)
    from pvamd import _lib
    lay = _lib.PV_SPEC_PACKED if packed else _lib.PV_SPEC_NATURAL
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames + 5,
                      spec_layout=lay)
    assert not pv.single_launch
    out1, spec1 = pv.process(xd)
    out2, none = pv.process(xd, spectrum=False)
    assert none is None
    assert torch.equal(out1, out2)
    out3, spec3 = pv.process(xd)
    assert torch.equal(out3, out1) and torch.equal(spec3, spec1)
    if not packed:
        _, ph = pvref.std_analysis(xs[1], N, N // hop_div, frames)
        g = spec3.cpu().numpy()[1, :frames, :N // 2 + 1, 1]
        assert np.array_equal(g.view(np.uint32), ph.view(np.uint32))
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord(effect), scale)
    g2 = out2.cpu().numpy()
    for c in range(C):
        assert g2[c].shape == ref[c].shape and rms(g2[c], ref[c]) <= RMS_TOL, f"ch{c}"


def pv_frames(n, hop):
    return max(1, -(-(n - hop) // hop))


def test_split_equals_fused(cuda):
    N, hop_div = 1024, 4
    x = synth(40000, 3)
    pv = PhaseVocoder(N, PITCH_SHIFT, 1.5, hop_div, mode=STANDARD, max_frames=400)
    out1, spec1 = pv.process(to_dev(x))
    spec2 = pv.analysis(to_dev(x))
    out2 = pv.resynthesis(spec2)
    assert np.array_equal(spec1.cpu().numpy(), spec2.cpu().numpy())
    assert np.array_equal(out1.cpu().numpy(), out2.cpu().numpy())


@pytest.mark.parametrize("N,hop_div", [(1024, 4), (256, 2), (512, 4), (2048, 4)])
def test_ref_compat_parity(cuda, N, hop_div):
    x = synth(30000, 11)
    pv = PhaseVocoder(N, TIME_SHIFT, 1.0, hop_div, mode=REF_COMPAT, max_frames=1000)
    out, spec = pv.process(to_dev(x))
    g = out.cpu().numpy()[0]
    ref = pvref.compat_process(x, N, hop_div)
    assert g.shape == ref.shape
    err = rms(g, ref)
    assert err <= RMS_TOL, f"rms {err}"


@pytest.mark.parametrize("N,hop_div,scale", [(1024, 4, 0.5), (1024, 4, 1.5), (512, 4, 0.75), (2048, 4, 2.0),
                                          (256, 2, 0.5)])
def test_ref_compat_time_scale_parity(cuda, N, hop_div, scale):
    """REF_COMPAT with a time scale: the overlap-add at outHopSize = (int)(scale * hop)
    (phaseVocoder.h:74 -> phaseVocoder.cpp:68; kernel.cu:354 keeps the spectrum unscaled),
    against the oracle's running accumulator at that hop."""
    x = synth(30000, 12)
    pv = PhaseVocoder(N, TIME_SHIFT, scale, hop_div, mode=REF_COMPAT, max_frames=1000)
    hs = pv.outHopSize
    assert hs == int(np.float32(scale) * np.float32(N // hop_div))
    out, _ = pv.process(to_dev(x))
    g = out.cpu().numpy()[0]
    ref = pvref.compat_process(x, N, hop_div, out_hop=hs)
    assert g.shape == ref.shape
    assert rms(g, ref) <= RMS_TOL


def test_ref_compat_spectrum(cuda):
    N = 1024
    x = synth(N, 5)
    pv = PhaseVocoder(N, TIME_SHIFT, 1.0, 4, mode=REF_COMPAT, max_frames=4)
    spec = pv.analysis(to_dev(x), frames=1, n_samples=N).cpu().numpy()[0, 0]
    ref = pvref.compat_analysis_frame(x, N)
    mag_ref = ref.real
    assert np.max(np.abs(spec[:2 * N, 0] - mag_ref)) <= 1e-5 * np.max(mag_ref)
    # phase contract of atanf(Im/Re) (kernel.cu:101-109) under fp32 FFT rounding: a bin's
    # complex value carries an absolute error of a few ulp of the frame's largest bin, so its
    # angle is good to ~ k eps max|X| / |X_k| (conditioning), plus atanf's own ulps; the
    # comparison is modulo pi (atan(y/x) jumps by pi where Re changes sign)
    m = mag_ref > 0
    d = np.abs(spec[:2 * N, 1][m].astype(np.float64) - ref.imag[m])
    d = np.minimum(d, np.pi - d)
    tol = 32 * np.finfo(np.float32).eps * mag_ref.max() / mag_ref[m] + 4e-7
    assert np.all(d <= tol), f"worst excess {np.max(d / tol):.2f}x of the bound"
    big = mag_ref > 1e-3 * mag_ref.max()
    assert np.max(np.minimum(np.abs(spec[:2 * N, 1][big] - ref.imag[big]),
                             np.pi - np.abs(spec[:2 * N, 1][big] - ref.imag[big]))) < 2e-4


def test_table_blob_roundtrip_and_validation(cuda):
    """The init-time broadcast payload: export -> import into another
    handle of the same configuration keeps outputs bit-identical; a blob built for a
    different configuration is rejected."""
    import torch
    from pvamd import PVError
    x = synth(20000, 9)
    a = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=100)
    b = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=100)
    blob = a.export_tables()
    assert blob.numel() > 1024 * 4
    b.import_tables(blob)
    assert torch.equal(b.export_tables(), blob)
    oa, _ = a.process(to_dev(x))
    ob, _ = b.process(to_dev(x))
    assert torch.equal(oa, ob)
    c = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=100)
    with pytest.raises(PVError):
        c.import_tables(blob)


def test_edge_cases_empty_short_and_silence(cuda):
    import torch
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=100)
    # n <= hop: no frames (main.cpp:231 loop never runs)
    assert pv.num_frames(200) == 0
    out, spec = pv.process(torch.zeros(200, device="cuda"))
    assert out.numel() == 0 and spec.numel() == 0
    # n < N: frames read zeros past the end
    x = synth(700, 4)
    out, _ = pv.process(to_dev(x))
    ref = pvref.std_process(x, 1024, 4, ord("t"), 0.5)
    assert out.shape[1] == ref.shape[0] and rms(out.cpu().numpy()[0], ref) <= RMS_TOL
    # digital silence then signal (autotune.wav starts with 1124 zeros): zero bins have
    # phase 0 by definition, so the unwrap state stays in step with the oracle
    x = np.concatenate([np.zeros(5000, np.float32), synth(20000, 5)])
    out, spec = pv.process(to_dev(x))
    ref = pvref.std_process(x, 1024, 4, ord("t"), 0.5)
    assert rms(out.cpu().numpy()[0], ref) <= RMS_TOL
    assert torch.all(spec[0, 0, :513, 1] == 0)


def test_ragged_channel_strides_and_determinism(cuda):
    """channels with a row stride larger than n; two runs must be bit-identical."""
    import torch
    C, n, ld = 3, 15000, 16384
    xs = np.zeros((C, ld), np.float32)
    for c in range(C):
        xs[c, :n] = synth(n, 100 + c)
    dev = to_dev(xs)
    pv = PhaseVocoder(1024, PITCH_SHIFT, 1.5, 4, mode=STANDARD, max_channels=C, max_frames=100)
    o1, _ = pv.process(dev, n_samples=n)
    o2, _ = pv.process(dev, n_samples=n)
    assert torch.equal(o1, o2)
    for c in range(C):
        ref = pvref.std_process(xs[c, :n], 1024, 4, ord("p"), 1.5)
        assert rms(o1[c].cpu().numpy(), ref) <= RMS_TOL


@pytest.mark.parametrize("N,hop_div,effect,scale", [
    (256, 2, TIME_SHIFT, 1.0),     # L=128, out hop 128: register overlap-add
    (512, 4, TIME_SHIFT, 1.0),     # L=256, out hop 128
    (512, 4, PITCH_SHIFT, 1.25),   # L=256, out hop 128, pitch map
    (2048, 4, TIME_SHIFT, 1.0),    # L=1024, out hop 512
    (2048, 4, PITCH_SHIFT, 0.8),   # L=1024, pitch
    (256, 4, TIME_SHIFT, 1.0),     # out hop 64: LDS ring overlap-add
    (1024, 4, TIME_SHIFT, 0.75),   # out hop 192: LDS ring overlap-add
    (2048, 8, TIME_SHIFT, 1.0),    # L=1024, out hop 256
    # pitch >= 1 takes the MODE 3 kernels (one source per bin, byte-offset map, zero slot)
    (2048, 4, PITCH_SHIFT, 1.0),   # L=1024: every bin its own source
    (2048, 4, PITCH_SHIFT, 2.0),   # L=1024, q = 1: odd bins sourceless (zero slot); single launch
    (2048, 8, PITCH_SHIFT, 1.25),  # L=1024, out hop 256 (DT = 2)
    (1024, 4, PITCH_SHIFT, 1.0),   # L=512
    (1024, 3, PITCH_SHIFT, 1.5),   # L=512, hop 341: LDS ring overlap-add (DT = 0)
    # output-phase ratios whose denominator q is not a power of two (hop not one): the
    # generic modular path (M mod q, (t + 1) mod q), which the power-of-two kernels skip
    (1024, 3, TIME_SHIFT, 0.5),    # hop 341, out hop 170: q = 341
    (512, 3, TIME_SHIFT, 1.37),    # hop 170, out hop 232: q = 85, stretch > 1
    (2048, 6, TIME_SHIFT, 0.8),    # L=1024, hop 341, out hop 272: q = 341
    (256, 3, TIME_SHIFT, 1.5),     # L=128, hop 85, out hop 127: q = 85
    (1024, 4, TIME_SHIFT, 0.25),   # out hop 64: q = 4, LDS ring
])
def test_std_process_parity_geometries(cuda, N, hop_div, effect, scale):
    """Both overlap-add paths (registers when the out hop is a multiple of 128 and
    L <= 1024, LDS ring otherwise) across FFT sizes."""
    x = synth(40000, 31)
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_frames=2000)
    out, _ = pv.process(to_dev(x))
    ref = pvref.std_process(x, N, hop_div, ord(effect), scale)
    assert out.shape[1] == ref.shape[0]
    assert rms(out.cpu().numpy()[0], ref) <= RMS_TOL


@pytest.mark.parametrize("C", [1, 32])
def test_long_streams_segmented_carry(cuda, C):
    """Long streams with few channels take the segmented unwrap-count scans (k_carry with
    16 run segments per 64 bins at C = 1, 4 at C = 32): integer, so the split cannot change
    a bit; checked end to end against the oracle (stretch 0.5 needs the carries, q = 2)."""
    N, hop_div, n = 1024, 4, 780000  # ~3050 frames per channel
    xs = np.stack([synth(n, 900 + c) for c in range(C)])
    pv = PhaseVocoder(N, TIME_SHIFT, 0.5, hop_div, mode=STANDARD, max_channels=C, max_frames=3100)
    nruns = -(-pv.num_frames(n) // pv.frames_per_run)
    assert nruns >= 64  # the segmented scans only run for >= 64 runs
    out, _ = pv.process(to_dev(xs))
    g = out.cpu().numpy()
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord("t"), 0.5)
    for c in range(C):
        assert rms(g[c], ref[c]) <= RMS_TOL, f"C={C} ch{c}"


@pytest.mark.parametrize("mode", [STANDARD, REF_COMPAT])
def test_odd_output_stride(cuda, mode):
    """out rows at an odd float stride: the vectorised stores must fall back to scalar."""
    import torch
    C, N = 3, 1024
    xs = np.stack([synth(25000, 60 + c) for c in range(C)])
    pv = PhaseVocoder(N, TIME_SHIFT, 0.5 if mode == STANDARD else 1.0, 4, mode=mode,
                      max_channels=C, max_frames=200)
    frames = pv.num_frames(xs.shape[1])
    olen = pv.output_length(frames)
    big = torch.full((C, olen + 1 if olen % 2 == 0 else olen + 2), 7.0, device="cuda")
    out = big[:, :olen]
    assert out.stride(0) % 2 == 1
    spec = pv.alloc_spec(C, frames)
    pv.process(to_dev(xs), spec=spec, out=out)
    dense, _ = pv.process(to_dev(xs))
    assert torch.equal(out, dense)
    assert torch.all(big[:, olen:] == 7.0)  # nothing written past the row


@pytest.mark.parametrize("F", [8, 16, 32, 42, 48, 64, 72, 88])
@pytest.mark.parametrize("effect,scale", [(TIME_SHIFT, 0.5), (PITCH_SHIFT, 1.5)])
def test_run_length_geometries(cuda, monkeypatch, F, effect, scale):
    """Run lengths the handle can pick (8, 16, 32 for small batches; a multiple of 8 in
    48 .. 96 for large ones at L <= 512 — 88 for config 3) and any even PV_RUN_FRAMES override
    (42: F = 2 mod 4) give the oracle's output; run boundaries only move the seams
    (<= 1e-6 between runs)."""
    N, hop_div, C = 1024, 4, 3
    xs = np.stack([synth(110250, 20240 + c) for c in range(C)])
    monkeypatch.setenv("PV_RUN_FRAMES", str(F))
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=440)
    assert pv.frames_per_run == F
    out, _ = pv.process(to_dev(xs))
    g = out.cpu().numpy()
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord(effect), scale)
    for c in range(C):
        assert rms(g[c], ref[c]) <= RMS_TOL, f"F={F} ch{c}"
    monkeypatch.setenv("PV_RUN_FRAMES", "16")
    pv16 = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=440)
    out16, _ = pv16.process(to_dev(xs))
    assert np.abs(out16.cpu().numpy() - g).max() <= 1e-6


@pytest.mark.parametrize("n", [1000, 900, 769, 1023])
def test_short_input_between_n_minus_hop_and_n(cuda, n):
    """N - hop < n < N: the one frame is partly past the end and must read
    zeros there (deviation 1), not the samples that follow in memory — with C = 2 and
    ldx == n those are the next channel's, with C = 1 a sentinel tail placed after n."""
    import torch
    N, hop_div = 1024, 4
    assert N - N // hop_div < n < N
    xs = np.stack([synth(n, 70), synth(n, 71) + 0.5]).astype(np.float32)
    pv = PhaseVocoder(N, TIME_SHIFT, 0.5, hop_div, mode=STANDARD, max_channels=2, max_frames=8)
    frames = pv.num_frames(n)
    assert frames >= 1                                       # every frame reaches past n
    out, spec = pv.process(to_dev(xs))                       # ldx == n
    for c in range(2):
        ref = pvref.std_process(xs[c], N, hop_div, ord("t"), 0.5)
        assert rms(out[c].cpu().numpy(), ref) <= RMS_TOL, f"channel {c}"
        mag, ph = pvref.std_analysis(xs[c], N, N // hop_div, frames)
        assert np.array_equal(spec[c, :frames, :N // 2 + 1, 1].cpu().numpy().view(np.uint32), ph.view(np.uint32))
    buf = torch.full((N + 64,), 1e3, device="cuda")
    buf[:n] = to_dev(xs[0])
    one = PhaseVocoder(N, TIME_SHIFT, 0.5, hop_div, mode=STANDARD, max_frames=8)
    o1, _ = one.process(buf[:n])
    assert torch.equal(o1[0], out[0])


@pytest.mark.parametrize("effect,scale", [(TIME_SHIFT, 0.5), (PITCH_SHIFT, 1.5)])
def test_nonfinite_burst_recovers(cuda, effect, scale):
    """Contract v4: a burst of NaN and Inf input samples makes the frames that contain it
    non-finite, but every phase stays finite (atan2's clamped ratio), so no unwrap decision
    corrupts the run sums and carries: the output after the burst's last frame is finite and
    matches the oracle (which restates the same clamp), and the phases are bit-exact."""
    N, hop_div = 1024, 4
    hop = N // hop_div
    x = synth(60000, 99)
    x[20000:20010] = np.nan
    x[20100] = np.inf
    x[20200] = -np.inf
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_frames=400)
    out, spec = pv.process(to_dev(x))
    frames = pv.num_frames(len(x))
    _, ph = pvref.std_analysis(x, N, hop, frames)
    g_ph = spec[0, :frames, :N // 2 + 1, 1].cpu().numpy()
    assert np.all(np.isfinite(g_ph)) and np.all(np.isfinite(ph))
    # equal phases everywhere; bit-identical outside the frames that hold a non-finite
    # sample (there every bin is NaN + i NaN and its phase +-0 by the NaN's sign bit, which
    # the platforms set differently — a zero sign no decision or output depends on)
    assert np.array_equal(g_ph, ph)
    bad = np.zeros(frames, bool)
    for t in range(frames):
        bad[t] = not np.all(np.isfinite(x[t * hop:t * hop + N]))
    assert bad.sum() > 0
    assert np.array_equal(g_ph[~bad].view(np.uint32), ph[~bad].view(np.uint32))
    assert np.all(np.abs(g_ph[bad]) == 0.0)
    g = out.cpu().numpy()[0]
    ref = pvref.std_process(x, N, hop_div, ord(effect), scale)
    assert g.shape == ref.shape
    # output samples of frames that start after the burst's last sample
    last_bad = (20200 // hop) + 1
    hs = pv.outHopSize
    start = (last_bad + 1) * hs + N
    assert np.all(np.isfinite(g[start:])) and np.all(np.isfinite(ref[start:]))
    assert rms(g[start:], ref[start:]) <= RMS_TOL
    # and before the burst too
    first_bad = 20000 // hop - N // hop
    assert rms(g[:max(first_bad, 0) * hs], ref[:max(first_bad, 0) * hs]) <= RMS_TOL


def test_spec_null_rows_reserved_for_graph_capture(cuda):
    """pv_process(spec = NULL) on the split path allocates the handle's own rows at its first
    call: under a stream capture that first call is refused (no allocation is
    captured), after pv_reserve_spectrum the same call captures, and the graph's replay gives
    the uncaptured call's bits."""
    import ctypes
    import torch
    from pvamd import _lib
    x = synth(30000, 5)
    xd = to_dev(x)
    mk = lambda: PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=200)
    ref_pv = mk()
    assert not ref_pv.single_launch
    ref, _ = ref_pv.process(xd, spectrum=False)  # first call outside a capture: allocates
    pv = mk()
    frames = pv.num_frames(len(x))
    out = pv.alloc_out(1, frames)
    L = _lib.lib()
    s = torch.cuda.Stream()
    torch.cuda.synchronize()

    def call():
        return L.pv_process(pv._h, xd.data_ptr(), xd.numel(), len(x), 1, frames, None, 0, out.data_ptr(),
                            out.stride(0), ctypes.c_void_p(s.cuda_stream))

    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        g.capture_begin()
        st = call()
        g.capture_end()
    assert st == _lib.PV_ERR_ARG and b"pv_reserve_spectrum" in L.pv_last_error()
    pv.reserve_spectrum()
    pv.reserve_spectrum()  # idempotent
    out.zero_()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        g2.capture_begin()
        st = call()
        g2.capture_end()
    assert st == _lib.PV_OK
    g2.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_reserve_spectrum_on_single_launch_is_a_no_op(cuda):
    """A single-launch handle (q = 1: pitch 2.0) keeps a spec = NULL spectrum on chip, so
    pv_reserve_spectrum allocates nothing and a capture of its pv_process needs no reserve."""
    pv = PhaseVocoder(1024, PITCH_SHIFT, 2.0, 4, mode=STANDARD, max_frames=200)
    assert pv.single_launch
    pv.reserve_spectrum()
    x = to_dev(synth(30000, 6))
    out, spec = pv.process(x, spectrum=False)
    assert spec is None
    ref = pvref.std_process(synth(30000, 6), 1024, 4, ord("p"), 2.0)
    assert rms(out.cpu().numpy()[0], ref) <= RMS_TOL


def test_capacity_limits_are_enforced_and_reachable(cuda):
    """A call may use exactly the handle's max_channels x max_frames (every kernel grid and
    workspace sized for it) and is refused beyond either, before any launch."""
    import torch
    from pvamd import _lib
    N, hop = 1024, 256
    C, F = 3, 40
    n = (F + 1) * hop  # exactly F frames (main.cpp:231)
    pv = PhaseVocoder(N, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_channels=C, max_frames=F)
    assert pv.num_frames(n) == F
    xs = np.stack([synth(n, 40 + c) for c in range(C)])
    out, _ = pv.process(torch.from_numpy(xs).cuda())
    ref, _ = pvref.std_process_batch(xs, N, 4, ord("t"), 0.5)
    for c in range(C):
        assert rms(out.cpu().numpy()[c], ref[c]) <= RMS_TOL
    with pytest.raises(_lib.PVError, match="capacity"):
        pv.process(torch.from_numpy(np.stack([synth(n + hop, 1)] * C)).cuda())  # F + 1 frames
    with pytest.raises(_lib.PVError, match="capacity"):
        pv.process(torch.from_numpy(np.stack([synth(n, 1)] * (C + 1))).cuda())  # C + 1 channels
    # the handle still works after the refusals
    out2, _ = pv.process(torch.from_numpy(xs).cuda())
    assert torch.equal(out, out2)


def test_two_handles_on_two_streams_are_independent(cuda):
    """include/pv.h: different handles share nothing — two handles driven concurrently on two
    streams give the same bits as each alone."""
    import torch
    xs = np.stack([synth(50000, 60 + c) for c in range(2)])
    xd = torch.from_numpy(xs).cuda()
    a = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_channels=2, max_frames=300)
    b = PhaseVocoder(2048, PITCH_SHIFT, 1.5, 4, mode=STANDARD, max_channels=2, max_frames=300)
    ra, _ = a.process(xd)
    rb, _ = b.process(xd)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for _ in range(3):
        oa, ob = a.alloc_out(2, a.num_frames(50000)), b.alloc_out(2, b.num_frames(50000))
        a.process(xd, out=oa, spectrum=False, stream=s1.cuda_stream)
        b.process(xd, out=ob, spectrum=False, stream=s2.cuda_stream)
        outs.append((oa, ob))
    torch.cuda.synchronize()
    for oa, ob in outs:
        assert torch.equal(oa, ra) and torch.equal(ob, rb)
