"""GPU parity of the real-time ring-buffer mode (pv_rt_*, BASELINE config 5) through the
C-ABI: a stream pushed callback by callback must equal the CPU oracle's offline pipeline
over the same stream prefixed with N - hop zeros (include/pv.h), its analysed phases must
be bit-identical to the oracle's, and the hipGraph callback must equal the plain push."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder, RealTimeVocoder

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5  # BASELINE.json north_star: <= 1e-5 RMS per sample vs the CPU reference


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


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def oracle_stream(x, N, hop_div, effect, scale, K):
    hop = N // hop_div
    xp = np.concatenate([np.zeros(N - hop, np.float32), x[:K * hop]])
    return xp, pvref.std_process(xp, N, hop_div, ord(effect), scale, frames=K)


@pytest.mark.parametrize("N,hop_div,effect,scale,per_push", [
    (256, 4, PITCH_SHIFT, 1.5, 1),     # config 5 geometry: 64-sample callbacks
    (256, 4, TIME_SHIFT, 0.5, 3),
    (1024, 4, TIME_SHIFT, 0.5, 2),
    (512, 4, TIME_SHIFT, 1.5, 1),      # out hop 192 (not a multiple of 64)
    (2048, 4, PITCH_SHIFT, 2.0, 4),    # L = 1024 instantiation
    (1024, 2, PITCH_SHIFT, 0.75, 5),
    (1024, 3, TIME_SHIFT, 0.5, 2),     # hop 341, out hop 170: q = 341 (generic modular path)
    (512, 3, TIME_SHIFT, 1.37, 1),     # hop 170, out hop 232: q = 85
])
def test_rt_stream_matches_oracle(cuda, N, hop_div, effect, scale, per_push):
    import torch
    hop = N // hop_div
    K = 60 if N <= 512 else 24
    K -= K % per_push
    x = synth(K * hop, 4242)
    rt = RealTimeVocoder(N, effect, scale, hop_div, channels=1)
    hs = rt.outHopSize
    spec = torch.zeros((1, per_push, rt.spec_stride, 2), dtype=torch.float32, device="cuda")
    outs, phases = [], []
    xd = dev(x)
    for j in range(K // per_push):
        o = rt.push(xd[j * per_push * hop:(j + 1) * per_push * hop], spec=spec)
        outs.append(o.cpu().numpy()[0])
        phases.append(spec.cpu().numpy()[0, :, :N // 2 + 1, 1].copy())
    g = np.concatenate(outs)
    assert g.shape == (K * hs,)
    xp, ref = oracle_stream(x, N, hop_div, effect, scale, K)
    err = rms(g, ref[:K * hs])
    assert err <= RMS_TOL, f"rms {err}"
    _, ph = pvref.std_analysis(xp, N, hop, K)
    gph = np.concatenate(phases)
    assert np.array_equal(gph.view(np.uint32), ph.view(np.uint32)), \
        f"phase mismatch in {np.sum(gph != ph)} bins"


def test_rt_many_channels_and_batch_equivalence(cuda):
    """256 channels (config 5 width): every channel equals the GPU batched pv_process of
    its zero-prefixed stream, and the oracle."""
    N, hop_div, C, K = 256, 4, 256, 40
    hop = N // hop_div
    xs = np.stack([synth(K * hop, 100 + c) for c in range(C)])
    rt = RealTimeVocoder(N, PITCH_SHIFT, 1.5, hop_div, channels=C)
    xd = dev(xs)
    g = np.concatenate([rt.push(xd[:, j * hop:(j + 1) * hop].contiguous()).cpu().numpy()
                        for j in range(K)], axis=1)
    xp = np.concatenate([np.zeros((C, N - hop), np.float32), xs], axis=1)
    pv = PhaseVocoder(N, PITCH_SHIFT, 1.5, hop_div, mode=STANDARD, max_channels=C, max_frames=K)
    out, _ = pv.process(dev(xp), frames=K)
    b = out.cpu().numpy()[:, :K * hop]
    assert np.max(np.abs(g - b)) <= 1e-6
    for c in (0, 77, 255):
        _, ref = oracle_stream(xs[c], N, hop_div, PITCH_SHIFT, 1.5, K)
        assert rms(g[c], ref[:K * hop]) <= RMS_TOL


@pytest.mark.parametrize("launch", ["direct", "graph"])
def test_rt_graph_callback_equals_push_and_reset(cuda, monkeypatch, launch):
    """The synchronous callback (direct launch by default, or the captured hipGraph replay)
    equals the plain push, and reset restarts the stream."""
    monkeypatch.setenv("PV_RT_LAUNCH", launch)
    N, hop_div, C, K = 256, 4, 8, 30
    hop = N // hop_div
    xs = np.stack([synth(K * hop, 900 + c) for c in range(C)])
    a = RealTimeVocoder(N, PITCH_SHIFT, 2.0, hop_div, channels=C)
    b = RealTimeVocoder(N, PITCH_SHIFT, 2.0, hop_div, channels=C)
    b.capture(1)
    xd = dev(xs)
    pa, pb = [], []
    for j in range(K):
        pa.append(a.push(xd[:, j * hop:(j + 1) * hop].contiguous()).cpu().numpy())
        pb.append(b.callback(xs[:, j * hop:(j + 1) * hop]).copy())
    ga, gb = np.concatenate(pa, axis=1), np.concatenate(pb, axis=1)
    assert np.array_equal(ga, gb)
    # reset restarts the stream: the first callbacks repeat exactly
    import torch
    torch.cuda.synchronize()
    b.reset()
    torch.cuda.synchronize()
    again = [b.callback(xs[:, j * hop:(j + 1) * hop]).copy() for j in range(5)]
    assert np.array_equal(np.concatenate(again, axis=1), gb[:, :5 * hop])


def test_rt_rejects_ref_compat_and_bad_sizes(cuda):
    from pvamd import PVError
    from pvamd import _lib
    import ctypes
    cfg = _lib.config(1024, 4, ord("t"), 1.0, _lib.PV_MODE_REF_COMPAT, 1, 1, 0)
    h = ctypes.c_void_p()
    assert _lib.lib().pv_rt_create(ctypes.byref(cfg), 1, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
    with pytest.raises(PVError):
        RealTimeVocoder(1000, PITCH_SHIFT, 1.0, 4)
