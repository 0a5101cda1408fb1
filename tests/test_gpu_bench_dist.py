"""The N-rank path of bench.py rehearsed on the one GPU of a box:
`python bench.py --gpus 2` with no launcher starts its two rank processes itself, over gloo
(PV_DIST_BACKEND=gloo: two ranks cannot share one device over RCCL).  The 8-GPU node runs
the same code with the nccl (= RCCL) backend, one rank per GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu(cuda):
    env = dict(os.environ, PV_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--channels", "8",
                        "--seconds", "1", "--steps", "3", "--warmup", "1", "--no-cpu"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["dist_backend"] == "gloo"
    assert d["tables_broadcast"]["bit_identical_to_local"] is True
    chk = d["rms_vs_oracle"]
    assert chk["pass"] and chk["ranks"] == 2 and chk["all_finite"]
    # value = frames of both ranks / max-over-ranks time
    frames = d["config"]["channels_per_gpu"] * d["config"]["frames_per_channel"] * 2 * d["steps"]
    assert abs(d["value"] * d["ms_per_step"] * d["steps"] * 1e-3 - frames) <= 1e-6 * frames


@pytest.mark.gpu
def test_bench_two_ranks_config4(cuda):
    """The 8-GPU configuration itself (BASELINE.json configs[3]: N=2048, hop 512, pitch 1.5,
    the L = 1024 table blob) through launch_ranks + broadcast_tables + the max-reductions."""
    env = dict(os.environ, PV_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "c4",
                        "--channels", "8", "--seconds", "1", "--steps", "3", "--warmup", "1", "--no-cpu"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["N"] == 2048 and d["config"]["hop"] == 512
    assert d["tables_broadcast"]["bit_identical_to_local"] is True
    assert d["tables_broadcast"]["bytes"] > 0
    chk = d["rms_vs_oracle"]
    assert chk["pass"] and chk["ranks"] == 2 and chk["all_finite"]


def test_bench_rejects_gpus_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE=3" in p.stderr


@pytest.mark.gpu
def test_bench_under_torchrun_one_rank_rccl(cuda):
    """The launch form of the driver's N-GPU runs (torch.distributed.run, one rank per GPU)
    with the production backend: nccl = RCCL.  One rank is what one GPU allows; it forms
    the RCCL group, broadcasts the tables and max-reduces the timing and the check exactly
    as every rank of the 8-GPU run does."""
    import socket
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PV_DIST_BACKEND"):
        env.pop(k, None)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "1", "--channels", "8", "--seconds", "1",
                        "--steps", "3", "--warmup", "1", "--no-cpu"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["dist_backend"] == "nccl"
    assert d["tables_broadcast"]["bit_identical_to_local"] is True
    assert d["rms_vs_oracle"]["pass"] and d["rms_vs_oracle"]["ranks"] == 1
