"""Multi-GPU plumbing for the phase-vocoder path.

Channels are independent mono streams, so they shard contiguously across ranks with no
data-path collective.  The only collective is the init-time broadcast (RCCL over xGMI
on MI355X nodes) of the constant tables rank 0 built, as BASELINE.json north_star asks;
a final all-reduce of the per-rank step time gives the max-over-ranks timing.
"""
from __future__ import annotations


def channel_shard(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of channels for `rank`: (first, count); sizes differ by <= 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def broadcast_blob(blob, src: int = 0, group=None):
    """Broadcast a (device or CPU) uint8 tensor in place from `src`."""
    import torch.distributed as dist
    dist.broadcast(blob, src=src, group=group)
    return blob


def broadcast_tables(pv, src: int = 0, group=None, local=None):
    """Rank `src` exports its handle's tables (pv_export_tables: one device blob); every
    other rank imports them (pv_import_tables).  The receiving ranks' handles are normally
    created with `tables_external=True`: they build no tables, so what they compute with is
    exactly what arrived over the wire.  With the nccl backend (RCCL over xGMI) the device
    blob is broadcast as is; a CPU backend (gloo: the CPU multi-process tests, a rehearsal on
    one GPU) stages it through host memory.  Returns whether the received blob is
    bit-identical to this rank's own tables — `local` (a handle of the same configuration
    that built them) or, on `src`, the sent blob itself — or None when there is nothing
    local to compare with."""
    import torch
    import torch.distributed as dist
    is_src = dist.get_rank(group) == src
    nccl = dist.get_backend(group) == "nccl"
    dev = getattr(pv, "blob_device", None) or f"cuda:{pv.device}"
    if is_src:
        mine = pv.export_tables()
        blob = mine if nccl else mine.cpu()
    else:
        blob = torch.empty(pv.tables_bytes(), dtype=torch.uint8, device=dev if nccl else "cpu")
    broadcast_blob(blob, src=src, group=group)
    blob = blob.to(dev)
    if not is_src:
        pv.import_tables(blob)
    ref = pv if is_src else local
    if ref is None:
        return None
    return bool(torch.equal(blob, ref.export_tables()))


# ---------------------------------------------------------------- one stream, many ranks
# SURVEY.md §8(e), the optional time shard: a single long stream split into consecutive frame
# segments, one per rank.  The frames are independent; the only sequential quantity is the
# per-bin integer unwrap count, so each rank summarises its segment (pv_segment_summary: a
# decision total and two boundary phases per bin), the summaries are all-gathered (one
# collective of C x 3 x bins_pad int32 per rank), and each rank resynthesises its segment
# with the count of everything before it (pv_segment_resynthesis) — the same unwrap counts
# and output phases as one GPU processing the whole stream.  The overlap of neighbouring
# segments' outputs (N - out_hop samples) is added where the blocks are assembled.

def frame_segments(total_frames: int, world: int) -> list[tuple[int, int]]:
    """Consecutive frame segments (first, count) for ranks 0 .. world - 1; sizes differ by
    <= 1 and empty segments (world > total_frames) come last."""
    return [channel_shard(total_frames, world, r) for r in range(world)]


def assemble_segments(blocks, firsts, out_hop: int, out_len: int):
    """Sum each segment's overlap-add block at its stream position first * out_hop (numpy or
    torch, [C, len] each) -> the whole stream's output [C, out_len]."""
    import numpy as np
    is_np = isinstance(blocks[0], np.ndarray)
    if is_np:
        out = np.zeros((blocks[0].shape[0], out_len), blocks[0].dtype)
    else:
        import torch
        out = torch.zeros((blocks[0].shape[0], out_len), dtype=blocks[0].dtype, device=blocks[0].device)
    for b, f in zip(blocks, firsts):
        p = f * out_hop
        n = min(b.shape[1], out_len - p)
        if n > 0:
            out[:, p:p + n] += b[:, :n]
    return out


def process_stream_segments(pv, x, group=None, n_samples: int | None = None):
    """Run one stream [C, n] (on this rank's device; every rank holds it, or at least its
    own frames' samples at their stream positions) as this rank's frame segment.  Returns
    (block, first_frame, segments): this rank's overlap-add block [C, frames*outHop + N -
    outHop] (None for an empty segment) and the (first, count) list of all ranks."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    x = x.unsqueeze(0) if x.dim() == 1 else x
    C, n = x.shape
    n = n if n_samples is None else n_samples
    total = pv.num_frames(n)
    segs = frame_segments(total, world)
    f0, nf = segs[rank]
    hop = pv.hopSize
    words = pv._L.pv_segment_summary_words(pv._h)
    spec = None
    if nf > 0:
        spec = pv.analysis(x[:, f0 * hop:], frames=nf, n_samples=n - f0 * hop)
        mine = pv.segment_summary(spec, nf)
    else:
        mine = torch.zeros((C, words), dtype=torch.int32, device=x.device)
    nccl = dist.get_backend(group) == "nccl"
    send = mine if nccl else mine.cpu()
    got = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(got, send, group=group)
    if nf == 0:
        return None, f0, segs
    # the earlier non-empty segments, in stream order (empty ones come last: none precedes)
    before = [got[j] for j in range(rank) if segs[j][1] > 0]
    summaries = torch.stack(before).to(x.device).contiguous() if before else None
    block = pv.segment_resynthesis(spec, f0, summaries, frames=nf)
    return block, f0, segs
