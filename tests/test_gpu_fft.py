"""GPU parity of the standalone FFT op (pv_fft_c2c, the reference's FFT::HPFFT API,
karnel/hpfft.h:6-11) against the CPU oracle's fp64 FFT and the reference's own 50 Hz
.dat fixtures (golden DFTs, tests/golden/make_golden.py), plus the hpfft.h drop-in's
result location (hpfft.cu:169-193: `signal` when log2 N is even, else `intermediary`)."""
import os
import subprocess

import numpy as np
import pytest

import pvref
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

FFT_BENCH = os.path.join(ROOT, "phase-vocoder_amd", "build", "fft_bench")


def rel_err(g, r):
    return float(np.sqrt(np.mean(np.abs(g - r) ** 2)) / max(np.sqrt(np.mean(np.abs(r) ** 2)), 1e-30))


def tol(n):  # fp32 radix-2: error grows like log2(n) roundings of the unit roundoff
    return 2e-7 * max(np.log2(n), 1) + 1e-7


@pytest.mark.parametrize("n", [2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048])
@pytest.mark.parametrize("inverse", [False, True])
def test_fft_batched_vs_oracle(cuda, n, inverse):
    import torch
    from pvamd.fft import fft
    rng = np.random.default_rng(n + 7 * inverse)
    B = 37
    x = (rng.standard_normal((B, n)) + 1j * rng.standard_normal((B, n))).astype(np.complex64)
    g = fft(torch.from_numpy(x).cuda(), inverse=inverse).cpu().numpy()
    for b in (0, 17, B - 1):
        r = pvref.fft_c64(x[b], inverse=inverse)
        assert rel_err(g[b], r) <= tol(n), (n, b, rel_err(g[b], r))


def test_fft_in_place_and_roundtrip(cuda):
    import torch
    from pvamd.fft import fft
    rng = np.random.default_rng(3)
    for n in (16, 32, 64, 512, 2048):
        x = (rng.standard_normal((9, n)) + 1j * rng.standard_normal((9, n))).astype(np.complex64)
        d = torch.from_numpy(x).cuda()
        fft(d, out=d)                # in place
        fft(d, inverse=True, out=d)  # unnormalised inverse: n * x
        back = d.cpu().numpy() / n
        assert rel_err(back, x) <= 2 * tol(n)


@pytest.mark.parametrize("n", [16, 32, 64])
def test_fft_small_n_offset_buffers_and_ragged_batch(cuda, n):
    """n <= 64 on buffers only 8-byte aligned (one complex element past a 16-byte boundary)
    and batches that leave a workgroup partly empty (k_fft_t8: 256 / (n / 8) transforms per
    workgroup): every transform against the oracle, nothing written past the batch."""
    import torch
    from pvamd.fft import fft
    rng = np.random.default_rng(100 + n)
    for B in (1, 33, 67):
        x = (rng.standard_normal((B, n)) + 1j * rng.standard_normal((B, n))).astype(np.complex64)
        big = torch.zeros(B * n + 2, dtype=torch.complex64, device="cuda")
        big[1:1 + B * n] = torch.from_numpy(x.reshape(-1)).cuda()
        src = big[1:1 + B * n].view(B, n)
        outb = torch.full((B * n + 2,), 7.0 + 0j, dtype=torch.complex64, device="cuda")
        dst = outb[1:1 + B * n].view(B, n)
        fft(src, out=dst)
        g = dst.cpu().numpy()
        for b in range(B):
            assert rel_err(g[b], pvref.fft_c64(x[b])) <= tol(n), (n, B, b)
        assert complex(outb[0].item()) == 7.0 + 0j and complex(outb[-1].item()) == 7.0 + 0j


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_fft_register_path_partial_blocks(cuda, n):
    """n <= 16 on 16-byte aligned buffers (k_fft_reg; n = 4 .. 16 stage the block's 256
    transforms through LDS): batches that end inside a 256-transform block, out of place and
    in place, every transform against the oracle, nothing written past the batch."""
    import torch
    from pvamd.fft import fft
    rng = np.random.default_rng(200 + n)
    for B in (1, 255, 257, 300):
        x = (rng.standard_normal((B, n)) + 1j * rng.standard_normal((B, n))).astype(np.complex64)
        r = np.stack([pvref.fft_c64(x[b]) for b in range(B)])
        src = torch.from_numpy(x).cuda()
        outb = torch.full((B + 1, n), 7.0 + 0j, dtype=torch.complex64, device="cuda")
        fft(src, out=outb[:B])
        g = outb.cpu().numpy()
        for b in range(B):
            assert rel_err(g[b], r[b]) <= tol(n), (n, B, b)
        assert np.all(g[B] == 7.0 + 0j)
        fft(src, out=src)  # in place
        assert np.array_equal(src.cpu().numpy(), g[:B])


@pytest.mark.parametrize("name", ["50Hz", "50Hz+500Hz", "500Hz+505Hz+12000Hz"])
def test_fft_reference_dat_fixtures(cuda, name):
    """The reference's FFT benchmark inputs (src/<tone>/*.dat), first 512 samples."""
    import torch
    from pvamd.fft import fft
    v = np.load(os.path.join(GOLDEN, f"dat_{name}.npy"))[:512].astype(np.complex64)
    ref = np.load(os.path.join(GOLDEN, f"dft_{name}_512.npy"))
    g = fft(torch.from_numpy(v).cuda()).cpu().numpy()
    assert rel_err(g, ref) <= tol(512)


@pytest.mark.parametrize("n", [32, 64, 256, 512, 1024])
@pytest.mark.parametrize("inverse", [0, 1])
def test_hpfft_dropin_result_location(cuda, tmp_path, n, inverse):
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    fin, fout = str(tmp_path / "in.c64"), str(tmp_path / "out.c64")
    x.tofile(fin)
    r = subprocess.run([FFT_BENCH, "check", fin, str(n), fout, str(inverse)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    g = np.fromfile(fout, np.complex64)
    assert rel_err(g, pvref.fft_c64(x, inverse=bool(inverse))) <= tol(n)


def test_fft_rejects_bad_sizes(cuda):
    import torch
    from pvamd import PVError
    from pvamd.fft import fft
    for n in (1, 3, 4096):
        with pytest.raises(PVError):
            fft(torch.zeros((2, n), dtype=torch.complex64, device="cuda"))
