"""bench.py pieces that run without a GPU: the synthetic generator (configs 2-4 of
BASELINE.md), the CPU-baseline leg of the JSON line (oracle timed on host cores) and the
oracle check of the timed batch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_synthetic_channels_are_seeded_and_bounded():
    a = bench.synth_channels_np(3, 4096, 20240)
    b = bench.synth_channels_np(3, 4096, 20240, threads=3)   # threaded == serial
    assert a.dtype == np.float32 and a.shape == (3, 4096)
    assert np.array_equal(a, b)                       # seed = 20240 + channel
    assert not np.array_equal(a[0], a[1])
    assert np.abs(a).max() <= 0.3 + 1e-3 + 1e-6        # 3 sines of 0.1 + noise 1e-3
    # a rank's shard (seed0 = 20240 + rank*C) is the same channels of the global batch
    g = bench.synth_channels_np(4, 4096, 20240)
    assert np.array_equal(bench.synth_channels_np(2, 4096, 20242), g[2:])


def test_cpu_baseline_fields_same_channels():
    x = bench.synth_channels_np(4, 44100, 20240)
    for single in (False, True):
        cpu = bench.cpu_baseline(x, 1024, 4, ord("t"), 0.5, target_s=0.2, single=single)
        assert set(cpu) >= {"value", "unit", "cores", "kind", "sample"}
        assert cpu["unit"] == "frames/s" and cpu["kind"] == "port"
        assert cpu["value"] > 0 and cpu["cores"] >= 1
        if single:
            assert cpu["cores"] == 1
        else:
            assert cpu["cores"] == bench.cpu_share()[0]
            assert "of the GPU batch" in cpu["sample"]


def test_check_channels_spread():
    assert bench.check_channels(1) == [0]
    idx = bench.check_channels(1024)
    assert len(idx) == 16 and idx[0] == 0 and idx[-1] == 1023
    assert bench.check_channels(5) == [0, 1, 2, 3, 4]


def test_oracle_check_detects_error():
    import pvref
    x = bench.synth_channels_np(3, 8192, 20240)
    frames = pvref.num_frames(8192, 256)
    ref, _ = pvref.std_process_batch(x, 1024, 4, ord("t"), 0.5, frames, 2)
    idx = [0, 2]
    ok = bench.oracle_check(x, ref[idx].copy(), idx, 1024, 4, ord("t"), 0.5, frames, True)
    assert ok["pass"] and ok["max"] == 0.0 and ok["channels"] == idx
    bad = ref[idx].copy()
    bad[1, 100] += 1.0
    r = bench.oracle_check(x, bad, idx, 1024, 4, ord("t"), 0.5, frames, True)
    assert not r["pass"] and r["max"] > 1e-5
    assert not bench.oracle_check(x, ref[idx].copy(), idx, 1024, 4, ord("t"), 0.5, frames, False)["pass"]


def test_metric_matches_baseline_json():
    import json
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert bench.METRIC == base["metric"]
    assert bench.HBM_PEAK_GBS == 8000.0


def test_compat_oracle_batch_and_baseline():
    """The REF_COMPAT workload's checker and CPU baseline: the OpenMP batch equals the
    per-channel fp64 restatement."""
    import pvref
    x = bench.synth_channels_np(3, 20000, 20240)
    out, used = pvref.compat_process_batch(x, 1024, 4, threads=2)
    for c in range(3):
        assert np.max(np.abs(out[c] - pvref.compat_process(x[c], 1024, 4))) <= 1e-6
    frames = pvref.num_frames(20000, 256)
    chk = bench.oracle_check(x, out[[0, 2]].copy(), [0, 2], 1024, 4, ord("t"), 1.0, frames, True, compat=True)
    assert chk["pass"] and "compat" in chk["oracle"]
    cpu = bench.cpu_baseline(x, 1024, 4, ord("t"), 1.0, target_s=0.2, compat=True)
    assert cpu["value"] > 0 and "REF_COMPAT" in cpu["sample"]
