"""Seeded random configurations against the oracle: FFT size, hop divisor, effect, scale,
channel count and length drawn from the ranges the handle accepts, each through pv_process
(whichever path the handle picks: single launch or split, register or LDS-ring overlap-add,
power-of-two or generic output-phase denominator) and, for STANDARD, the bit-exact
analysis.  A fixed seed list, so a failure names a reproducible case."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, REF_COMPAT, STANDARD, TIME_SHIFT, PhaseVocoder
from test_gpu_parity import RMS_TOL, rms, synth

pytestmark = pytest.mark.gpu


def draw(seed):
    rng = np.random.default_rng(seed)
    N = int(rng.choice([256, 512, 1024, 2048]))
    hop_div = int(rng.choice([2, 3, 4, 4, 4, 8]))
    compat = rng.random() < 0.2
    if compat:
        effect, scale = TIME_SHIFT, float(rng.choice([1.0, 0.5, 1.5]))
    elif rng.random() < 0.5:
        effect, scale = PITCH_SHIFT, float(rng.choice([0.5, 0.75, 1.0, 1.25, 1.5, 2.0, 3.0]))
    else:
        effect, scale = TIME_SHIFT, float(rng.choice([0.25, 0.5, 0.75, 1.0, 1.37, 1.5, 2.0]))
    C = int(rng.integers(1, 4))
    n = int(rng.integers(N // 2, 12 * N))
    return N, hop_div, compat, effect, scale, C, n


@pytest.mark.parametrize("seed", list(range(64)))
def test_random_configuration_matches_oracle(cuda, seed):
    import torch
    N, hop_div, compat, effect, scale, C, n = draw(1000 + seed)
    hop = N // hop_div
    if effect == TIME_SHIFT and int(np.float32(scale) * np.float32(hop)) > N:
        pytest.skip("out hop > N is refused by pv_create")
    xs = np.stack([synth(n, 5000 + 17 * seed + c) for c in range(C)])
    mode = REF_COMPAT if compat else STANDARD
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=mode, max_channels=C, max_frames=max(1, n // hop + 2))
    out, spec = pv.process(torch.from_numpy(xs).cuda())
    g = out.cpu().numpy()
    frames = pv.num_frames(n)
    for c in range(C):
        if compat:
            ref = pvref.compat_process(xs[c], N, hop_div, out_hop=pv.outHopSize)
        else:
            ref = pvref.std_process(xs[c], N, hop_div, ord(effect), scale)
        assert g[c].shape == ref.shape, (seed, N, hop_div, effect, scale)
        assert np.isfinite(g[c]).all()
        assert rms(g[c], ref) <= RMS_TOL, (seed, N, hop_div, effect, scale, C, n)
    if not compat and frames > 0:
        s = pv.unpack_spec(spec).cpu().numpy()
        _, ph = pvref.std_analysis(xs[0], N, hop, frames)
        assert np.array_equal(s[0, :frames, :, 1].view(np.uint32), ph.view(np.uint32)), seed


@pytest.mark.parametrize("seed", list(range(16)))
def test_random_configuration_in_segments(cuda, seed):
    """The same draws (STANDARD) as 2-5 consecutive frame segments (pv_segment_*): the
    assembled output equals the whole stream's up to the seams' summation order."""
    import torch
    from test_gpu_segments import run_segments
    N, hop_div, compat, effect, scale, C, n = draw(3000 + seed)
    hop = N // hop_div
    if compat or (effect == TIME_SHIFT and int(np.float32(scale) * np.float32(hop)) > N):
        pytest.skip("STANDARD draws only")
    xs = np.stack([synth(n, 7000 + 13 * seed + c) for c in range(C)])
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=max(1, n // hop + 2))
    xd = torch.from_numpy(xs).cuda()
    whole, _ = pv.process(xd)
    nseg = 2 + seed % 4
    got = run_segments(pv, xd, nseg)
    assert got.shape == whole.shape
    assert np.max(np.abs(got.cpu().numpy() - whole.cpu().numpy())) <= 1e-6, (seed, N, hop_div, effect, scale)


@pytest.mark.parametrize("seed", list(range(16)))
def test_random_real_time_configuration(cuda, seed):
    """Real-time mode (pv_rt_*) on random draws: the stream pushed in random-size blocks of
    whole hops equals the oracle's offline pipeline over the zero-prefixed stream."""
    from pvamd import RealTimeVocoder
    from test_gpu_rt import dev, oracle_stream
    rng = np.random.default_rng(9000 + seed)
    N = int(rng.choice([256, 512, 1024, 2048]))
    hop_div = int(rng.choice([2, 4, 4, 8]))
    if rng.random() < 0.5:
        effect, scale = PITCH_SHIFT, float(rng.choice([0.75, 1.0, 1.5, 2.0]))
    else:
        effect, scale = TIME_SHIFT, float(rng.choice([0.5, 0.75, 1.0, 1.5]))
    hop = N // hop_div
    K = int(rng.integers(6, 40))
    x = synth(K * hop, 9500 + seed)
    rt = RealTimeVocoder(N, effect, scale, hop_div, channels=1)
    hs = rt.outHopSize
    xd = dev(x)
    outs, j = [], 0
    while j < K:
        m = int(min(K - j, rng.integers(1, 5)))
        outs.append(rt.push(xd[j * hop:(j + m) * hop]).cpu().numpy()[0])
        j += m
    g = np.concatenate(outs)
    assert g.shape == (K * hs,)
    _, ref = oracle_stream(x, N, hop_div, effect, scale, K)
    assert rms(g, ref[:K * hs]) <= RMS_TOL, (seed, N, hop_div, effect, scale, K)
