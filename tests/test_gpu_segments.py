"""One long stream as consecutive frame segments (pv_segment_*, SURVEY.md §8(e)'s time
shard): each segment analysed alone, summarised, and resynthesised after the earlier
segments' summaries gives the whole stream's output — the unwrap counts are integer sums and
the boundary decisions the contract's, so only the overlap-add's summation order at the
segment seams differs (<= 1e-6) — and the oracle's (<= 1e-5 RMS)."""
import numpy as np
import pytest

import pvref
from pvamd import PITCH_SHIFT, STANDARD, TIME_SHIFT, PhaseVocoder
from pvamd.dist import assemble_segments, frame_segments
from test_gpu_parity import RMS_TOL, rms, synth, to_dev

pytestmark = pytest.mark.gpu


def run_segments(pv, x, nseg):
    import torch
    xd = to_dev(x) if not isinstance(x, torch.Tensor) else x
    xd = xd.unsqueeze(0) if xd.dim() == 1 else xd
    n = xd.shape[1]
    total = pv.num_frames(n)
    hop = pv.hopSize
    sums, blocks, firsts = [], [], []
    for f0, nf in frame_segments(total, nseg):
        if nf == 0:
            continue
        spec = pv.analysis(xd[:, f0 * hop:], frames=nf, n_samples=n - f0 * hop)
        before = torch.stack(sums).contiguous() if sums else None
        blocks.append(pv.segment_resynthesis(spec, f0, before, frames=nf))
        sums.append(pv.segment_summary(spec, nf))
        firsts.append(f0)
    return assemble_segments(blocks, firsts, pv.outHopSize, pv.output_length(total))


@pytest.mark.parametrize("N,hop_div,effect,scale,nseg", [
    (1024, 4, TIME_SHIFT, 0.5, 3),     # config 3 geometry: q = 2
    (1024, 4, PITCH_SHIFT, 1.5, 4),    # q = 2, pitch map
    (1024, 4, TIME_SHIFT, 0.75, 5),    # q = 4, LDS ring overlap-add
    (2048, 4, PITCH_SHIFT, 1.5, 2),    # config 4 geometry
    (1024, 3, TIME_SHIFT, 0.5, 3),     # q = 341 (generic modular path)
    (512, 4, PITCH_SHIFT, 2.0, 3),     # q = 1: no unwrap state at all
])
def test_segments_equal_the_whole_stream(cuda, N, hop_div, effect, scale, nseg):
    x = synth(80000, 606)
    pv = PhaseVocoder(N, effect, scale, hop_div, mode=STANDARD, max_frames=1000)
    whole, _ = pv.process(to_dev(x))
    got = run_segments(pv, x, nseg)
    g, w = got.cpu().numpy()[0], whole.cpu().numpy()[0]
    assert g.shape == w.shape
    assert np.max(np.abs(g - w)) <= 1e-6
    ref = pvref.std_process(x, N, hop_div, ord(effect), scale)
    assert rms(g, ref) <= RMS_TOL


def test_segments_multichannel_and_one_frame_segments(cuda):
    """Several channels at once, and segments of one frame each at the start (every
    boundary decision comes from the summaries)."""
    import torch
    C = 3
    xs = np.stack([synth(12000, 700 + c) for c in range(C)])
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_channels=C, max_frames=100)
    xd = torch.from_numpy(xs).cuda()
    whole, _ = pv.process(xd)
    total = pv.num_frames(xs.shape[1])
    got = run_segments(pv, xd, total)  # one frame per segment
    assert np.max(np.abs(got.cpu().numpy() - whole.cpu().numpy())) <= 1e-6


def test_segment_summary_refuses_an_empty_segment(cuda):
    import torch
    from pvamd import _lib
    pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=10)
    spec = pv.alloc_spec(1, 1)
    with pytest.raises(_lib.PVError):
        pv.segment_summary(spec, 0)
    del torch


def test_two_rank_stream_segments(cuda):
    """Two fresh rank processes (gloo; the 8-GPU node runs the same code over RCCL), one
    stream: each rank analyses and resynthesises its half after one all-gather of the
    summaries; the assembled output equals the whole stream's."""
    import json
    import os
    import subprocess
    import sys
    from test_gpu_dist import _free_port
    here = os.path.dirname(os.path.abspath(__file__))
    world, n = 2, 120000
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(here, "dist_stream_child.py"), str(n)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    res.sort(key=lambda d: d["rank"])
    assert res[0]["first"] == 0 and res[1]["first"] == res[0]["count"] > 0
    for d in res:
        assert d["finite"] and d["max_vs_whole"] <= 1e-6 and d["rms_vs_oracle"] <= RMS_TOL, d
