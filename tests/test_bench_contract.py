"""bench.py pieces that run without a GPU: the synthetic generator (configs 2-4 of
BASELINE.md) and the CPU-baseline leg of the JSON line (oracle timed on host cores)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_synthetic_channels_are_seeded_and_bounded():
    a = bench.synth_channels_np(3, 4096, 20240)
    b = bench.synth_channels_np(3, 4096, 20240)
    assert a.dtype == np.float32 and a.shape == (3, 4096)
    assert np.array_equal(a, b)                       # seed = 20240 + channel
    assert not np.array_equal(a[0], a[1])
    assert np.abs(a).max() <= 0.3 + 1e-3 + 1e-6        # 3 sines of 0.1 + noise 1e-3


def test_cpu_baseline_fields():
    for single in (False, True):
        cpu = bench.cpu_baseline(1024, 4, ord("t"), 0.5, 44100, target_s=0.2, single=single)
        assert set(cpu) >= {"value", "unit", "cores", "kind", "sample"}
        assert cpu["unit"] == "frames/s" and cpu["kind"] == "port"
        assert cpu["value"] > 0 and cpu["cores"] >= 1
        if single:
            assert cpu["cores"] == 1


def test_metric_matches_baseline_json():
    import json
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert bench.METRIC == base["metric"]
    assert bench.HBM_PEAK_GBS == 8000.0
