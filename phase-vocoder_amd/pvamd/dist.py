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
    """Rank `src` exports its handle's tables; every other rank imports them.  Returns True
    when this rank's own tables were already bit-identical to the received ones."""
    import torch
    import torch.distributed as dist
    mine = pv.export_tables()
    blob = mine.clone() if dist.get_rank(group) == src else torch.empty_like(mine)
    broadcast_blob(blob, src=src, group=group)
    same = bool(torch.equal(blob, mine))
    if dist.get_rank(group) != src:
        pv.import_tables(blob)
    return same
