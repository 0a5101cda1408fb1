#!/usr/bin/env python3
"""Where the time of the config-2 single launch (k_fused, pv_fused.hip) goes: every wave
stamps s_memrealtime (100 MHz) at its start, after the table set-up barrier, after each of
its F frames, after the frame loop and at its end, in a diagnostic build only

  make -C phase-vocoder_amd/csrc -j8 variant NAME=stamps DEFS="-DPV_FUSED_STAMPS -DPV_DIAGNOSTIC_BUILD"
  PV_LIB_PATH=phase-vocoder_amd/build/variants/libpv_stamps.so python scripts/fused_stamps.py

(the product kernel executes no stamp).  Runs config 2 (one 60 s stream, N = 1024, pitch
2.0) back to back for ~1 s, then reads the stamps of the last launch and prints one JSON
line: the launch span, the dispatch ramp (wave start offsets), the per-phase durations and
the clock (s_memtime / s_memrealtime)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-vocoder_amd"))
sys.path.insert(0, ROOT)

SLOTS = 16


def pct(a, q):
    return float(np.percentile(a, q)) if a.size else None


def main():
    import torch
    from bench import synth_channels_np
    from pvamd import PhaseVocoder, STANDARD, PITCH_SHIFT, _lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 44100 * 60
    N, hop_div = 1024, 4
    x = torch.from_numpy(synth_channels_np(1, n, 20240, 1)).cuda()
    pv = PhaseVocoder(N, PITCH_SHIFT, 2.0, hop_div, mode=STANDARD, max_channels=1,
                      max_frames=n // (N // hop_div) + 2, spec_layout=_lib.PV_SPEC_PACKED)
    fr = pv.num_frames(n)
    spec, out = pv.alloc_spec(1, fr), pv.alloc_out(1, fr)
    F = pv.info.single_launch_frames
    assert F > 0, "config 2 must take the single-launch path"
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < 1.0:
        if os.environ.get("STAMPS_WRITE_SPEC") == "1":
            pv.process(x, spec=spec, out=out)
        else:  # bench.py's c2 default: the rows stay on chip
            pv.process(x, out=out, spectrum=False)
        steps += 1
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    L = _lib.lib()
    L.pv_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    nruns = -(-fr // F)
    nw = 4 * (-(-nruns // 4))
    buf = np.zeros(nw * SLOTS, np.uint64)
    _lib.check(L.pv_debug_stamps(pv._h, buf.ctypes.data, buf.size), "pv_debug_stamps")
    st = buf.reshape(nw, SLOTS).astype(np.int64)
    st = st[st[:, 0] != 0]  # the waves the launch had (a balanced launch has fewer than nruns)
    if len(sys.argv) > 2:
        np.save(sys.argv[2], st)  # raw stamps for offline analysis
    rt0, mt0, setup = st[:, 0], st[:, 1], st[:, 2]
    frames = st[:, 3:3 + min(F, 6)]
    f0_ready, wg_done = st[:, 10], st[:, 9]
    loop_end, rt1, mt1 = st[:, 11], st[:, 12], st[:, 13]
    t_min = rt0.min()
    us = 0.01  # 100 MHz ticks -> us
    ghz = (mt1 - mt0) / np.maximum(rt1 - rt0, 1) * 0.1
    hw, xcc = st[:, 14], st[:, 15]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    frame_d = np.diff(np.concatenate([setup[:, None], frames], axis=1), axis=1)
    res = {
        "launch_span_us": float((rt1.max() - t_min) * us),
        "waves": int(len(st)), "runs_uniform_F": int(nruns), "F": F, "steps": steps, "host_ms_per_step": dt * 1e3,
        "start_offset_us": {q: pct((rt0 - t_min) * us, q) for q in (0, 10, 50, 90, 100)},
        "setup_us": {q: pct((setup - rt0) * us, q) for q in (10, 50, 90, 100)},
        "frame_us": {f"frame{j}": {q: pct(frame_d[:, j] * us, q) for q in (10, 50, 90)} for j in range(frame_d.shape[1])},
        "frame0_input_wait_us": {q: pct((f0_ready - setup) * us, q) for q in (10, 50, 90, 100)},
        "wg_barrier_wait_us": {q: pct((wg_done - loop_end) * us, q) for q in (10, 50, 90, 100)},
        "seams_us": {q: pct((rt1 - wg_done) * us, q) for q in (10, 50, 90, 100)},
        "seams_us_by_wave": {w: {q: pct(((rt1 - wg_done) * us)[w::4], q) for q in (50, 90, 100)} for w in range(4)},
        "wave_total_us": {q: pct((rt1 - rt0) * us, q) for q in (10, 50, 90, 100)},
        "end_offset_us": {q: pct((rt1 - t_min) * us, q) for q in (0, 10, 50, 90, 100)},
        "clock_GHz": {q: pct(ghz, q) for q in (10, 50, 90)},
        "xcc_waves": np.bincount(xcc & 0xF, minlength=8).tolist(),
        "distinct_cu_se_xcc": int(len(set(zip(cu.tolist(), se.tolist(), (xcc & 0xF).tolist())))),
    }
    # placement: waves per SIMD, wave index -> SIMD, and whether workgroups k, k + 256,
    # k + 512 share a CU (what a placement-aware run-length pattern would rely on)
    simd = (hw >> 4) & 0x3
    sh = (hw >> 12) & 0x1
    cukey = (xcc & 0xF) * 4096 + se * 512 + sh * 256 + cu
    simdkey = cukey * 4 + simd
    _, per_simd = np.unique(simdkey, return_counts=True)
    _, per_cu = np.unique(cukey, return_counts=True)
    wave_in_wg = np.arange(len(st)) % 4
    wg = np.arange(len(st)) // 4
    res["placement"] = {
        "simds_used": int(per_simd.size), "waves_per_simd_hist": np.bincount(per_simd).tolist(),
        "cus_used": int(per_cu.size), "waves_per_cu_hist": np.bincount(per_cu).tolist(),
        "wave_index_equals_simd_frac": float(np.mean(wave_in_wg == simd)),
    }
    cu_of_wg = {}
    for i in range(len(st)):
        cu_of_wg.setdefault(int(wg[i]), set()).add(int(cukey[i]))
    pairs = [(k, k + 256) for k in range(len(cu_of_wg)) if k + 256 in cu_of_wg]
    res["placement"]["wg_k_and_k256_same_cu_frac"] = float(np.mean([cu_of_wg[a] == cu_of_wg[b] for a, b in pairs])) if pairs else None
    res["placement"]["wg_single_cu_frac"] = float(np.mean([len(v) == 1 for v in cu_of_wg.values()]))
    # time histogram of live waves (how many waves run at each microsecond of the launch)
    edges = np.arange(0, res["launch_span_us"] + 1.0, 1.0)
    live = [int(np.sum(((rt0 - t_min) * us <= e) & ((rt1 - t_min) * us > e))) for e in edges]
    res["live_waves_per_us"] = live
    print(json.dumps(res))


if __name__ == "__main__":
    main()
