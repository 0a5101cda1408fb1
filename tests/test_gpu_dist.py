"""Multi-GPU readiness on one GPU: two fresh child processes, one per rank,
gloo process group (the 8-GPU node runs the same code over RCCL).  Each rank takes its
contiguous channel shard, receives rank 0's real pv_export_tables blob through
pvamd.dist.broadcast_tables (rank 1's handle is created with tables_external: it builds no
tables and refuses to compute until the broadcast delivers rank 0's, so the
import must take effect), runs pv_process on its shard and checks it against the oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_with_table_broadcast(cuda):
    world, total, n = 2, 6, 60000
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_child.py"), str(total), str(n)],
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
    covered = []
    for d in res:
        covered.extend(range(d["first"], d["first"] + d["count"]))
        assert d["finite"] and d["tables_equal"]
        assert max(d["rms"]) <= 1e-5, d
        assert d["rms_max_all_ranks"] <= 1e-5
    assert covered == list(range(total))
    # rank 0 sent its own tables; rank 1 had none (tables_external: it refused to compute
    # before the broadcast) and computed with exactly what arrived
    assert res[0]["same_before"] is True and res[1]["same_before"] is None
    assert res[1]["refused_without_tables"] is True
