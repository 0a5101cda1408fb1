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


def test_roofline_reports_both_roofs(tmp_path):
    """the line carries the HBM and the VALU roof of the dominant kernel and
    names the regime: "hbm" / "valu" when that roof's fraction exceeds bench.BIND_FRAC,
    "power" when the workload was measured at the package power cap, otherwise "latency"
    with the ablation evidence of profiles/regime.json."""
    import json
    N, hop, hs, B, frames = 1024, 256, 128, 512, 1024 * 1722
    regime = tmp_path / "regime.json"
    regime.write_text(json.dumps({"c3": {"clock_ghz": 1.85, "clock_source": "test",
                                         "analysis": {"latency_evidence": {"memory_side_ms": 1.86}}}}))
    kw = dict(regime_path=str(regime))
    r = bench.roofline("analysis", 2.0, "c3", N, hop, hs, B, frames, False, None, **kw)
    assert r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["achieved"] - (4 * hop + 8 * B) * frames / 2e-3 / 1e9) < 1e-6
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-12
    v = r["valu"]
    assert v["peak_tflops"] == 157.3
    assert abs(v["flops_per_frame"] - (2.5 * N * 10 + N + 25 * 513)) < 1e-9
    # the two STANDARD halves sum to SURVEY's 5 N log2 N + 5 N + 40 (N/2+1) (~77 kflop)
    tot = bench.alg_flops_per_frame("analysis", N, False) + bench.alg_flops_per_frame("synthesis", N, False)
    assert abs(tot - (5 * N * 10 + 5 * N + 40 * 513)) < 1e-9 and 76e3 < tot < 78e3
    comp = bench.alg_flops_per_frame("compat_analysis", N, True) + bench.alg_flops_per_frame("synthesis", N, True)
    assert 147e3 < comp < 150e3
    assert r["bound"] in ("hbm", "valu", "latency")

    def isa_file(sha, cyc):
        p = tmp_path / "isa.json"
        p.write_text(json.dumps({"_sources_sha16": sha, "c3": {"analysis": {"valu_cycles_per_frame": cyc}}}))
        return str(p)

    sha = bench.kernel_sources_sha()
    # issue fractions at the peak and at the measured clock
    r2 = bench.roofline("analysis", 2.0, "c3", N, hop, hs, B, frames, False, None, isa_path=isa_file(sha, 1600.0), **kw)
    f = 1600.0 * frames / (1024 * 2e-3 * 2.4e9)
    assert abs(r2["valu"]["issue_frac_at_peak_clock"] - f) < 1e-12
    fm = 1600.0 * frames / (1024 * 2e-3 * 1.85e9)
    assert abs(r2["valu"]["issue_frac_at_measured_clock"] - fm) < 1e-12
    assert r2["valu"]["measured_clock_ghz"] == 1.85
    assert "STALE" not in r2["valu"]["issue_source"]
    # HBM 0.56, issue 0.73 at the measured clock: neither roof binds -> latency, with evidence
    assert r2["frac"] < bench.BIND_FRAC and fm < bench.BIND_FRAC
    assert r2["bound"] == "latency" and r2["latency_evidence"] == {"memory_side_ms": 1.86}
    # an issue fraction above the threshold binds
    r3 = bench.roofline("analysis", 2.0, "c3", N, hop, hs, B, frames, False, None, isa_path=isa_file(sha, 2400.0), **kw)
    assert r3["bound"] == "valu" and "latency_evidence" not in r3
    # so does the HBM roof
    r4 = bench.roofline("analysis", 1.2, "c3", N, hop, hs, B, frames, False, None, isa_path=isa_file(sha, 100.0), **kw)
    assert r4["frac"] > bench.BIND_FRAC and r4["bound"] == "hbm"
    # a stale estimate is reported but never decides the regime
    r5 = bench.roofline("analysis", 2.0, "c3", N, hop, hs, B, frames, False, None, isa_path=isa_file("0", 4000.0), **kw)
    assert "STALE" in r5["valu"]["issue_source"] and r5["valu"]["issue_frac_at_peak_clock"] is None
    assert r5["bound"] == "latency"
    # a workload measured at the package power cap: "power", with its evidence, below the
    # HBM roof whatever the issue fraction
    regime2 = tmp_path / "regime2.json"
    regime2.write_text(json.dumps({"c3": {"clock_ghz": 1.79, "clock_source": "test", "package_power_w": 1400,
                                          "power_cap_w": 1400,
                                          "analysis": {"latency_evidence": {"memory_side_ms": 1.86},
                                                       "power_evidence": {"clock_ghz": 1.79}}}}))
    kw2 = dict(regime_path=str(regime2))
    for cyc in (1600.0, 2400.0):
        r6 = bench.roofline("analysis", 2.0, "c3", N, hop, hs, B, frames, False, None, isa_path=isa_file(sha, cyc), **kw2)
        assert r6["bound"] == "power" and r6["power_evidence"] == {"clock_ghz": 1.79}
        assert r6["latency_evidence"] == {"memory_side_ms": 1.86}
    r7 = bench.roofline("analysis", 1.2, "c3", N, hop, hs, B, frames, False, None, isa_path=isa_file(sha, 100.0), **kw2)
    assert r7["bound"] == "hbm"


def test_committed_regime_evidence():
    """profiles/regime.json carries the measured clock and the latency evidence of the
    headline kernel, citing its sources."""
    import json
    reg = json.load(open(os.path.join(ROOT, "profiles", "regime.json")))
    ev = reg["c3"]["analysis"]["latency_evidence"]
    assert 1.5 < reg["c3"]["clock_ghz"] < 2.4 and "r06_clock_power_c3" in reg["c3"]["clock_source"]
    assert reg["c3"]["package_power_w"] >= 0.99 * reg["c3"]["power_cap_w"]
    pe = reg["c3"]["analysis"]["power_evidence"]
    for src in pe["sources"].split(", "):
        assert os.path.exists(os.path.join(ROOT, src)), src
    assert ev["memory_side_ms"] > 0 and "r04_ab_c3_ablation" in ev["sources"]
    for src in ("r04_ab_c3_ablation.txt", "r05_mix_probe.jsonl", "r05_ab_ring.json"):
        assert os.path.exists(os.path.join(ROOT, "profiles", src))


def test_path_bytes_count_hbm_bytes_only():
    """path_hbm_frac counts the bytes that go through HBM: the split path
    writes and re-reads the spectrum rows, the single launch (config 2) keeps them on chip."""
    # config 3: 1 KiB in, 512 B out, a packed 4 KiB row written and re-read
    assert bench.path_bytes_per_frame(256, 128, 512, 512, False) == 4 * 256 + 4 * 128 + 8 * 512 * 2
    # config 2 on the single launch: the samples only (4 hop_a + 4 hop_s)
    assert bench.path_bytes_per_frame(256, 256, 512, 512, True) == 2048


def test_committed_c2_regime_evidence():
    """The config-2 single launch's regime is stated with evidence: the
    clock measured on c2 steps and the latency evidence of its per-wave stamps, so the bench
    line's roofline carries both."""
    import json
    reg = json.load(open(os.path.join(ROOT, "profiles", "regime.json")))
    c2 = reg["c2"]
    assert 1.5 < c2["clock_ghz"] <= 2.4 and "stamps" in c2["clock_source"]
    ev = c2["fused"]["latency_evidence"]
    assert ev["launch_span_us"] > 0 and ev["sources"]
    for src in ev["sources"].split(", "):
        assert os.path.exists(os.path.join(ROOT, src.split(" ")[0])), src
    N, hop, hs, B, frames = 1024, 256, 256, 512, 1722
    sha = bench.kernel_sources_sha()
    r = bench.roofline("fused", 0.023, "c2", N, hop, hs, B, frames, False, None, spec_written=False)
    assert r["valu"]["measured_clock_ghz"] == c2["clock_ghz"]
    if r["bound"] == "latency":
        assert r["latency_evidence"] == ev
    del sha


def test_committed_isa_static_matches_sources():
    """profiles/isa_static.json must describe this build's kernels (regenerate it with
    scripts/isa_static.py after a kernel change)."""
    import json
    isa = json.load(open(os.path.join(ROOT, "profiles", "isa_static.json")))
    assert isa["_sources_sha16"] == bench.kernel_sources_sha()
    for wl, k in (("c3", "analysis"), ("c3", "synthesis"), ("c4", "analysis"), ("c4", "synthesis"),
                  ("compat", "compat_analysis"), ("c2", "fused"), ("rt", "rt")):
        assert isa[wl][k]["valu_cycles_per_frame"] > 0
