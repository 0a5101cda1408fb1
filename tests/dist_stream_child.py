"""One rank of tests/test_gpu_segments.py's two-rank run (a fresh child process per rank;
not collected by pytest): one long stream split into frame segments across the ranks
(pvamd.dist.process_stream_segments, gloo process group), the blocks all-gathered and
assembled on every rank, checked against the whole stream on one handle and the oracle.
Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "phase-vocoder_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import pvref
    from pvamd import STANDARD, TIME_SHIFT, PhaseVocoder
    from pvamd.dist import assemble_segments, process_stream_segments
    from test_gpu_parity import rms, synth

    n = int(sys.argv[1])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    try:
        x = synth(n, 909)
        pv = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=pv_frames(n))
        xd = torch.from_numpy(x).cuda()
        block, f0, segs = process_stream_segments(pv, xd)
        # every rank's block, padded to the longest, to every rank
        L = max(pv.output_length(c) for _, c in segs)
        mine = torch.zeros((1, L), dtype=torch.float32)
        if block is not None:
            mine[:, :block.shape[1]] = block.cpu()
        allb = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allb, mine)
        blocks = [allb[r][:, :pv.output_length(c)].numpy() for r, (_, c) in enumerate(segs) if c > 0]
        firsts = [f for f, c in segs if c > 0]
        total = pv.num_frames(n)
        got = assemble_segments(blocks, firsts, pv.outHopSize, pv.output_length(total))[0]
        whole, _ = pv.process(xd)
        w = whole.cpu().numpy()[0]
        ref = pvref.std_process(x, 1024, 4, ord("t"), 0.5)
        print(json.dumps({"rank": rank, "first": f0, "count": segs[rank][1],
                          "max_vs_whole": float(np.max(np.abs(got - w))), "rms_vs_oracle": rms(got, ref),
                          "finite": bool(np.isfinite(got).all())}), flush=True)
    finally:
        dist.destroy_process_group()


def pv_frames(n, hop=256):
    return max(1, (n - hop + hop - 1) // hop)


if __name__ == "__main__":
    main()
