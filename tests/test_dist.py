"""Multi-process (gloo, world_size 2, CPU) coverage of the sharded path: channel
partition, the init-time table broadcast and the max-over-ranks timing reduction."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pvamd.dist import broadcast_blob, broadcast_tables, channel_shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1) shards: every channel exactly once
        first, count = channel_shard(8192, world, rank)
        got = torch.tensor([first, count])
        allg = [torch.zeros(2, dtype=torch.long) for _ in range(world)]
        dist.all_gather(allg, got)
        # 2) table broadcast: rank 0's blob reaches every rank bit-exactly
        g = torch.Generator().manual_seed(1234)
        ref = torch.randint(0, 256, (12345,), dtype=torch.uint8, generator=g)
        blob = ref.clone() if rank == 0 else torch.zeros_like(ref)
        broadcast_blob(blob, src=0)
        # 3) max over ranks of the step time
        t = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        results[rank] = (sorted(tuple(x.tolist()) for x in allg), bool(torch.equal(blob, ref)), float(t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_shard_broadcast_timing(world):
    port = _free_port()
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, port, results), nprocs=world, join=True)
    for r in range(world):
        shards, same, tmax = results[r]
        assert same and tmax == float(world)
        covered = []
        for first, count in shards:
            covered.extend(range(first, first + count))
        assert covered == list(range(8192))


def test_channel_shard_uneven():
    parts = [channel_shard(10, 4, r) for r in range(4)]
    assert parts == [(0, 3), (3, 3), (6, 2), (8, 2)]
    with pytest.raises(ValueError):
        channel_shard(10, 4, 4)


class _FakeHandle:
    """Stands in for PhaseVocoder's export_tables / import_tables on CPU; external=True is a
    handle created with tables_external (no tables until an import)."""
    blob_device = "cpu"

    def __init__(self, rank, external=False):
        g = torch.Generator().manual_seed(99 if rank == 0 else 100 + rank)
        self.tables = None if external else torch.randint(0, 256, (4096,), dtype=torch.uint8, generator=g)
        self.imported = 0

    def tables_bytes(self):
        return 4096

    def export_tables(self):
        assert self.tables is not None, "tables_external handle: nothing to export"
        return self.tables.clone()

    def import_tables(self, blob):
        self.tables = blob.clone()
        self.imported += 1


def _tables_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        h = _FakeHandle(rank, external=rank != 0)
        local = _FakeHandle(0) if rank == 2 else None  # rank 2 compares with a local build
        same = broadcast_tables(h, src=0, local=local)
        results[rank] = (same, h.imported, h.tables.sum().item(), int(h.tables[:8].sum()))
    finally:
        dist.destroy_process_group()


def test_broadcast_tables_gloo():
    """broadcast_tables over gloo: rank 0 keeps its tables; the others start with none
    (tables_external) and hold exactly rank 0's after the import; a rank given a locally
    built handle reports whether the received blob equals it."""
    world, port = 3, _free_port()
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_tables_worker, args=(world, port, results), nprocs=world, join=True)
    assert results[0][0] is True and results[0][1] == 0
    for r in range(1, world):
        assert results[r][1] == 1
        assert results[r][2:] == results[0][2:]
    assert results[1][0] is None       # nothing local to compare with
    assert results[2][0] is True       # its local build (seed 99) equals rank 0's


def test_frame_segments_cover_the_stream_in_order():
    from pvamd.dist import frame_segments
    for total in (0, 1, 3, 10, 1722, 10335):
        for world in (1, 2, 3, 8):
            segs = frame_segments(total, world)
            assert len(segs) == world
            pos = 0
            for f, c in segs:
                assert f == pos and c >= 0
                pos += c
            assert pos == total
            counts = [c for _, c in segs]
            assert max(counts) - min(counts) <= 1
            # empty segments only at the end (pv_segment_summary refuses an empty one)
            assert counts == sorted(counts, reverse=True)


def test_assemble_segments_is_the_overlap_add_of_the_blocks():
    import numpy as np
    from pvamd.dist import assemble_segments, frame_segments
    rng = np.random.default_rng(5)
    N, hs, total, C = 64, 16, 37, 2
    frames = rng.standard_normal((C, total, N))
    want = np.zeros((C, total * hs + N - hs))
    for t in range(total):
        want[:, t * hs:t * hs + N] += frames[:, t]
    blocks, firsts = [], []
    for f, c in frame_segments(total, 3):
        b = np.zeros((C, c * hs + N - hs))
        for u in range(c):
            b[:, u * hs:u * hs + N] += frames[:, f + u]
        blocks.append(b)
        firsts.append(f)
    got = assemble_segments(blocks, firsts, hs, want.shape[1])
    assert np.allclose(got, want, rtol=0, atol=1e-12)


def test_segment_abi_checks_without_gpu():
    import ctypes
    from pvamd import _lib
    L = _lib.lib()
    assert L.pv_segment_summary_words(None) == 0
    assert L.pv_segment_summary(None, None, 0, 1, 1, None, None) == _lib.PV_ERR_ARG
    assert L.pv_segment_resynthesis(None, None, 0, 1, 1, 0, None, 0, None, 0, None) == _lib.PV_ERR_ARG
    assert {"pv_segment_summary", "pv_segment_resynthesis", "pv_segment_summary_words"} <= set(_lib.declared_symbols())
    del ctypes
