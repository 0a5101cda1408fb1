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


def broadcast_tables(pv, src: int = 0, group=None) -> bool:
    """Rank `src` exports its handle's tables (pv_export_tables: one device blob); every
    other rank imports them (pv_import_tables).  With the nccl backend (RCCL over xGMI) the
    device blob is broadcast as is; a CPU backend (gloo: the CPU multi-process tests, a
    rehearsal on one GPU) stages it through host memory.  Returns True when this rank's own
    tables were already bit-identical to the received ones."""
    import torch
    import torch.distributed as dist
    mine = pv.export_tables()
    wire = mine if dist.get_backend(group) == "nccl" else mine.cpu()
    blob = wire.clone() if dist.get_rank(group) == src else torch.empty_like(wire)
    broadcast_blob(blob, src=src, group=group)
    blob = blob.to(mine.device)
    same = bool(torch.equal(blob, mine))
    if dist.get_rank(group) != src:
        pv.import_tables(blob)
    return same
