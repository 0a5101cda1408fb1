"""pv_profile_enable's sampling stride (include/pv.h): with k > 1 only every k-th
pv_process call's launches carry hipEvents, and the outputs do not depend on it."""
import numpy as np
import pytest

from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from test_gpu_parity import synth, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("effect,scale,kernels", [(TIME_SHIFT, 0.5, {"analysis", "synthesis"}),
                                                  (PITCH_SHIFT, 2.0, {"fused"})])
def test_profile_stride(cuda, effect, scale, kernels):
    n = 30000
    pv = PhaseVocoder(1024, effect, scale, 4, mode=STANDARD, max_channels=2, max_frames=n // 256 + 2)
    xd = to_dev(np.stack([synth(n, 1), synth(n, 2)]))
    ref, _ = pv.process(xd)
    ref = ref.cpu().numpy()
    for stride, calls, timed in ((1, 5, 5), (3, 7, 3), (4, 4, 1)):
        pv.profile(stride)
        pv.profile_reset()
        for _ in range(calls):
            out, _ = pv.process(xd)
        prof = pv.profile_read()
        pv.profile(False)
        for k in kernels:
            assert prof[k][1] == timed, (stride, k, prof[k])
            assert prof[k][0] > 0.0
        assert np.array_equal(out.cpu().numpy(), ref)
    with pytest.raises(Exception):
        pv.profile(-1)
