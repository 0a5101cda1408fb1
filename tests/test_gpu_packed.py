"""The PV_SPEC_PACKED spectrum row layout (include/pv.h): rows of exactly N/2 float2 with
bins 0 and N/2 (both real) folded into slot 0 as sign-coded magnitudes, so every row store
is whole 64-byte segments.  It changes where two bins are stored, nothing else: the
unpacked rows equal the natural layout's bit for bit, and every output equals the natural
layout's bit for bit, on every kernel geometry that writes or reads rows (shifted-register
and plain analysis, per-lane and LDS unwrap constants, register and LDS overlap-add, the
q = 1 single launch, pv_resynthesis's run sums, L = 128 .. 1024)."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from pvamd import _lib
from test_gpu_parity import RMS_TOL, rms, synth, to_dev

pytestmark = pytest.mark.gpu

GEOMS = [  # (N, hop_div, effect, scale)
    (1024, 4, TIME_SHIFT, 0.5),    # config 3: shifted-register analysis, per-lane constants
    (2048, 4, PITCH_SHIFT, 1.5),   # config 4: L = 1024
    (1024, 4, PITCH_SHIFT, 2.0),   # config 2: the q = 1 single launch (pv_fused.hip)
    (256, 4, PITCH_SHIFT, 1.5),    # config 5's geometry, L = 128
    (512, 2, TIME_SHIFT, 1.5),     # hop 256 = 128 D, out hop 384: LDS-ring overlap-add
    (1024, 8, TIME_SHIFT, 0.75),   # hop 128: 64 % hop_div = 0
    (1024, 3, TIME_SHIFT, 1.0),    # hop 341: plain analysis, e_k from LDS (EKL)
]


def _pair(N, hop_div, effect, scale, C, frames):
    kw = dict(mode=STANDARD, max_channels=C, max_frames=frames)
    nat = PhaseVocoder(N, effect, scale, hop_div, **kw)
    pk = PhaseVocoder(N, effect, scale, hop_div, spec_layout=_lib.PV_SPEC_PACKED, **kw)
    assert pk.spec_layout == _lib.PV_SPEC_PACKED and nat.spec_layout == _lib.PV_SPEC_NATURAL
    assert pk.spec_bins == pk.spec_stride == N // 2 and nat.spec_bins == N // 2 + 1
    return nat, pk


@pytest.mark.parametrize("N,hop_div,effect,scale", GEOMS)
def test_packed_process_bit_identical(cuda, N, hop_div, effect, scale):
    C, n = 3, 50000 + 777
    xs = np.stack([synth(n, 900 + c) for c in range(C)])
    nat, pk = _pair(N, hop_div, effect, scale, C, n // (N // hop_div) + 2)
    xd = to_dev(xs)
    out_n, spec_n = nat.process(xd)
    out_p, spec_p = pk.process(xd)
    fr = nat.num_frames(n)
    a = nat.unpack_spec(spec_n)[:, :fr].cpu().numpy()
    b = pk.unpack_spec(spec_p)[:, :fr].cpu().numpy()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "unpacked rows differ"
    assert np.array_equal(out_n.cpu().numpy().view(np.uint32), out_p.cpu().numpy().view(np.uint32))
    # and the phases of bins 0 and N/2 are exactly +0 or pi (what the sign bit encodes)
    ph = b[..., [0, N // 2], 1]
    assert np.all((ph.view(np.uint32) == 0) | (ph == np.float32(np.pi)))
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord(effect), scale)
    g = out_p.cpu().numpy()
    for c in range(C):
        assert rms(g[c][:ref.shape[1]], ref[c]) <= RMS_TOL


@pytest.mark.parametrize("N,hop_div,effect,scale", [GEOMS[0], GEOMS[1], GEOMS[4]])
def test_packed_split_entry_points(cuda, N, hop_div, effect, scale):
    """pv_analysis then pv_resynthesis (the run sums re-read the packed phases of bins 0
    and N/2 from slot 0) equals the natural layout's output."""
    n = 40000
    x = synth(n, 5)
    nat, pk = _pair(N, hop_div, effect, scale, 1, n // (N // hop_div) + 2)
    xd = to_dev(x)
    outs = []
    for pv in (nat, pk):
        spec = pv.analysis(xd)
        outs.append(pv.resynthesis(spec).cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    # bit-exact phases against the oracle's contract analysis through the unpacking
    fr = pk.num_frames(n)
    _, ph = pvref.std_analysis(x, N, N // hop_div, fr)
    got = pk.unpack_spec(pk.analysis(xd)).cpu().numpy()[0, :fr, :, 1]
    assert np.array_equal(got.view(np.uint32), ph.view(np.uint32))


def test_packed_rejected_where_unsupported(cuda):
    from pvamd import REF_COMPAT, RealTimeVocoder  # noqa: F401
    with pytest.raises(_lib.PVError):
        PhaseVocoder(1024, TIME_SHIFT, 1.0, 4, mode=REF_COMPAT, spec_layout=_lib.PV_SPEC_PACKED)
    L = _lib.lib()
    import ctypes
    h = ctypes.c_void_p()
    cfg = _lib.config(256, 4, ord("p"), 1.5, _lib.PV_MODE_STANDARD, 4, 1, 0, spec_layout=_lib.PV_SPEC_PACKED)
    assert L.pv_rt_create(ctypes.byref(cfg), 4, ctypes.byref(h)) == _lib.PV_ERR_UNSUPPORTED
