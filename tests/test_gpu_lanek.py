"""Per-lane unwrap constants in the split synthesis (pv_syn_run.hpp LANEK, pv_info
lane_constants): when e_k and (p j_k) mod q repeat every 64 bins (64 a multiple of N / hop,
q of 64 hop / N — BASELINE configs 3 and 4) the synthesis keeps them in two registers
instead of reading two LDS tables per bin and frame.  The output must be bit-identical to
the table path (PV_SYN_LANEK=0) and within 1e-5 RMS of the oracle."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from test_gpu_parity import RMS_TOL, rms, synth, to_dev

pytestmark = pytest.mark.gpu


def pv_frames(n, hop):
    return max(1, -(-(n - hop) // hop))


CASES = [  # (N, hop_div, effect, scale, lane constants expected)
    (1024, 4, TIME_SHIFT, 0.5, 1),     # config 3: q = 2
    (2048, 4, PITCH_SHIFT, 1.5, 1),    # config 4: q = 2, L = 1024 (gains + split twiddles in registers)
    (2048, 4, TIME_SHIFT, 0.25, 1),    # L = 1024, out hop 128 (DT = 1), q = 4
    (2048, 16, PITCH_SHIFT, 1.5, 1),   # L = 1024, hop 128 (DT = 1), q = 2
    (1024, 4, PITCH_SHIFT, 1.25, 1),   # q = 4 divides 64 / 4
    (512, 4, PITCH_SHIFT, 0.75, 1),    # L = 256, hop 128, q = 4 divides 16
    (512, 8, PITCH_SHIFT, 0.75, 0),    # out hop 64: the LDS-ring synthesis reads the tables
    (1024, 4, PITCH_SHIFT, 1.03125, 0),  # q = 32 does not divide 16: the tables
    (1024, 4, PITCH_SHIFT, 2.0, 0),    # q = 1: the single-launch path (no split synthesis)
]


@pytest.mark.parametrize("N,hop_div,effect,scale,expect", CASES)
def test_lane_constants_equal_tables(cuda, monkeypatch, N, hop_div, effect, scale, expect):
    C, n = 2, 70000
    hop = N // hop_div
    xs = np.stack([synth(n, 321 + c) for c in range(C)])
    xd = to_dev(xs)
    frames = pv_frames(n, hop)
    outs = {}
    for v in ("1", "0"):
        monkeypatch.setenv("PV_SYN_LANEK", v)
        pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_channels=C, max_frames=frames)
        if v == "1":
            assert pv.single_launch == 1 or pv.lane_constants == expect
        else:
            assert pv.lane_constants == 0
        out, _ = pv.process(xd)
        outs[v] = out.cpu().numpy()
    assert np.array_equal(outs["1"].view(np.uint32), outs["0"].view(np.uint32))
    ref, _ = pvref.std_process_batch(xs, N, hop_div, ord(effect), scale)
    for c in range(C):
        assert rms(outs["1"][c], ref[c]) <= RMS_TOL, f"ch{c}"
