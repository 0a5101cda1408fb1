"""GPU tests of the drop-in surface: the C++ driver pv_main (main.cpp's offline loop on
the phaseVocoder.h drop-in), the Python mirror's per-frame reference methods, and the
OVERLAPTEST identity path — each checked against the CPU oracle."""
import os
import struct
import subprocess

import numpy as np
import pytest

import pvref
from conftest import GOLDEN, ROOT
from pvamd import REF_COMPAT, STANDARD, TIME_SHIFT, PhaseVocoder, wav

pytestmark = pytest.mark.gpu

PV_MAIN = os.path.join(ROOT, "phase-vocoder_amd", "build", "pv_main")


def write_pcm16(path, x):
    """x = int16/32768 values (exact): write them back bit-exactly as mono 16-bit PCM."""
    ints = np.round(np.asarray(x, np.float64) * 32768.0).astype("<i2")
    body = ints.tobytes()
    hdr = b"RIFF" + struct.pack("<i", 36 + len(body)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<ihhiihh", 16, 1, 1, 44100, 88200, 2, 16)
    hdr += b"data" + struct.pack("<i", len(body))
    open(path, "wb").write(hdr + body)


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


@pytest.fixture(scope="module")
def sine440(tmp_path_factory):
    x = np.load(os.path.join(GOLDEN, "sine440_ch0_32768.npy"))
    p = str(tmp_path_factory.mktemp("wav") / "sine440.wav")
    write_pcm16(p, x)
    return p, x


@pytest.mark.parametrize("batched", [False, True])
def test_pv_main_ref_compat_config1_geometry(cuda, sine440, tmp_path, batched):
    """config 1 geometry (N=1024, hop 256, scale 1, REF_COMPAT) through the C++ driver."""
    path, x = sine440
    out_wav, dump = str(tmp_path / "out.wav"), str(tmp_path / "out.f32")
    cmd = [PV_MAIN, path, "t", out_wav, "--N", "1024", "--hopdiv", "4", "--dump-f32", dump]
    if batched:
        cmd.append("--batched")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(dump, np.float32)
    ref = pvref.compat_process(x, 1024, 4)
    n_emit = (len(x) // 256) * 256  # main.cpp:266 emits floor(n/outHop) hops
    assert len(got) >= n_emit
    assert rms(got[:n_emit], ref[:n_emit]) <= 1e-5
    s, sr, bits = wav.load(out_wav)
    assert s.shape == (2, len(x)) and bits == 16 and sr == 44100
    assert np.array_equal(s[0], s[1])  # R duplicates L (main.cpp:288-289)
    q = np.trunc(np.clip(ref[:n_emit], -1, 1) * 32767) / 32768.0
    assert np.max(np.abs(s[0, :n_emit] - q)) <= 1.01 / 32768  # at most 1 LSB from rounding


@pytest.mark.parametrize("scale", [0.5, 1.5])
@pytest.mark.parametrize("batched", [False, True])
def test_pv_main_ref_compat_time_scale(cuda, sine440, tmp_path, scale, batched):
    """main.cpp's TIME_SHIFT loop at a time scale (REF_COMPAT): floor(n / outHop) frames of
    outHop samples (main.cpp:266-287), frames past the analysed ones resynthesise zero
    spectra; per-frame and batched drivers against the oracle's overlap-add at outHop."""
    path, x = sine440
    dump = str(tmp_path / "o.f32")
    cmd = [PV_MAIN, path, "t", str(tmp_path / "o.wav"), "--N", "1024", "--hopdiv", "4",
           "--scale", str(scale), "--dump-f32", dump]
    if batched:
        cmd.append("--batched")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(dump, np.float32)
    hs = int(np.float32(scale) * np.float32(256))
    ref = pvref.compat_process(x, 1024, 4, out_hop=hs)
    n_emit = (len(x) // hs) * hs
    # the batched driver dumps what it writes to the WAV (outLen = timeScale * n samples,
    # main.cpp's output file), the per-frame one every emitted hop
    m = min(len(got), len(ref), n_emit)
    assert m >= min(n_emit, int(np.float32(scale) * len(x)))
    assert rms(got[:m], ref[:m]) <= 1e-5
    if len(got) > len(ref):
        assert not np.any(got[len(ref):n_emit])  # past the analysed frames' overlap-add: zero spectra


def test_pv_main_standard_batched(cuda, sine440, tmp_path):
    path, x = sine440
    dump = str(tmp_path / "o.f32")
    r = subprocess.run([PV_MAIN, path, "p", str(tmp_path / "o.wav"), "--N", "1024", "--hopdiv", "4",
                        "--scale", "1.5", "--mode", "std", "--batched", "--dump-f32", dump],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(dump, np.float32)
    ref = pvref.std_process(x, 1024, 4, ord("p"), 1.5)
    assert rms(got, ref[:len(got)]) <= 1e-5


def test_python_mirror_per_frame_loop_matches_batched(cuda):
    """main.cpp's per-frame loop written with the reference method names."""
    import torch
    x = np.load(os.path.join(GOLDEN, "sine440_ch0_32768.npy"))[:8192]
    N, hd = 1024, 4
    pv = PhaseVocoder(N, TIME_SHIFT, 1.0, hd, mode=REF_COMPAT, max_frames=64)
    hop = pv.hopSize
    d_input = torch.zeros(len(x) + 2 * N, device="cuda")
    d_input[:len(x)] = torch.from_numpy(x).cuda()
    nspec = len(x) // hop + 1
    d_output = torch.zeros((nspec, pv.spec_stride, 2), device="cuda")
    for i in range(0, len(x) - hop, hop):                       # main.cpp:231
        pv.analysis_CUFFT(d_input[i:], d_output[i // hop])
    back = torch.zeros(N, device="cuda")
    final = torch.empty(N, device="cuda")
    emitted = []
    for i in range(len(x) // pv.outHopSize):                    # main.cpp:266
        pv.resynthesis_CUFFT(back, d_output[min(i, nspec - 1)], final)
        back.copy_(final)
        emitted.append(back[:pv.outHopSize].cpu().numpy().copy())
    got = np.concatenate(emitted)
    ref = pvref.compat_process(x, N, hd)
    assert rms(got, ref[:len(got)]) <= 1e-5
    out, _ = PhaseVocoder(N, TIME_SHIFT, 1.0, hd, mode=REF_COMPAT, max_frames=64).process(
        torch.from_numpy(x).cuda())
    assert rms(got, out.cpu().numpy()[0][:len(got)]) <= 1e-6


def test_overlap_test_identity(cuda):
    """OVERLAPTEST (main.cpp:156-202, kernel.cu:289-298): out = w^2 x + back[hop:]."""
    import ctypes
    import torch
    from pvamd import _lib
    from pvamd.tables import hamming_ref
    N, hop = 256, 128
    rng = np.random.default_rng(0)
    x = rng.standard_normal(N).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    w = hamming_ref(N)
    dx, db, dw = (torch.from_numpy(v).cuda() for v in (x, b, w))
    out = torch.empty(N, device="cuda")
    st = _lib.lib().pv_test_overlap_add(ctypes.c_void_p(dx.data_ptr()), ctypes.c_void_p(dw.data_ptr()),
                                        ctypes.c_void_p(db.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                        N, hop, None)
    assert st == 0
    ref = (x * w) * w
    ref[:N - hop] += b[hop:]
    assert np.allclose(out.cpu().numpy(), ref, rtol=1e-6, atol=1e-6)


# ------------------------------------------------------------ config 1 at full size
REF_440 = os.path.join(GOLDEN, "testtones_440sine.wav")  # the reference's testtones/440sine.wav


def run_main(args, timeout=300):
    r = subprocess.run([PV_MAIN] + args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def check_wav_1lsb(out_wav, ref, n_total, n_emit):
    s, sr, bits = wav.load(out_wav)
    assert s.shape == (2, n_total) and bits == 16 and sr == 44100
    assert np.array_equal(s[0], s[1])                      # R duplicates L (main.cpp:288-289)
    q = np.trunc(np.nan_to_num(np.clip(ref[:n_emit], -1, 1)) * 32767) / 32768.0
    assert np.max(np.abs(s[0, :n_emit] - q)) <= 1.01 / 32768  # within 1 LSB
    assert np.all(s[0, n_emit:] == 0)                        # never written (main.cpp:266)


@pytest.mark.parametrize("batched", [False, True])
def test_config1_full_440sine_wav(cuda, tmp_path, batched):
    """BASELINE configs[0] on the whole reference input: testtones/440sine.wav (441000
    stereo frames, data chunk 2 bytes short), N=1024 hop 256, REF_COMPAT, scale 1: all
    1722 frames of channel 0 through main.cpp's loop (per frame: PhaseVocoder ->
    CudaPhase::*_CUFFT of include/kernel.h, timed by CudaPhase::timer()) vs the oracle."""
    x = wav.load(REF_440)[0][0]
    assert len(x) == 441000
    out_wav, dump = str(tmp_path / "out.wav"), str(tmp_path / "out.f32")
    args = [REF_440, "t", out_wav, "--N", "1024", "--hopdiv", "4", "--dump-f32", dump]
    stdout = run_main(args + (["--batched"] if batched else ["--timer"]))
    ref = pvref.compat_process(x, 1024, 4)
    assert pvref.num_frames(len(x), 256) == 1722
    n_emit = (len(x) // 256) * 256                             # 1722 resynthesis frames
    got = np.fromfile(dump, np.float32)
    assert len(got) >= n_emit
    assert rms(got[:n_emit], ref[:n_emit]) <= 1e-5
    frame_rms = np.sqrt(np.mean((got[:n_emit] - ref[:n_emit]).reshape(-1, 256) ** 2, axis=1))
    assert frame_rms.max() <= 1e-5                             # every emitted hop, not only the mean
    check_wav_1lsb(out_wav, ref, len(x), n_emit)
    if not batched:
        line = [ln for ln in stdout.splitlines() if ln.startswith("CudaPhase::timer()")][0]
        assert float(line.split("analysis ")[1].split(" ms")[0]) > 0


@pytest.mark.parametrize("batched", [False, True])
def test_single_arg_constructor_hann(cuda, tmp_path, batched):
    """PhaseVocoder(int samples) (phaseVocoder.h:46-78): periodic Hann
    0.5f*(1 - cosf(2 pi i/N)), hop N/2, timeScale 1.  Per frame the window reaches the
    kernels only through CudaPhase's `win` argument (pv_set_window), so this also checks
    that kernel.h honours the caller's window (kernel.cu:301, :406)."""
    x = wav.load(REF_440)[0][0]
    out_wav, dump = str(tmp_path / "o.wav"), str(tmp_path / "o.f32")
    run_main([REF_440, "t", out_wav, "--N", "1024", "--single-arg", "--dump-f32", dump]
             + (["--batched"] if batched else []))
    ref = pvref.compat_process(x, 1024, 2, window=pvref.hann_ref(1024))
    ham = pvref.compat_process(x, 1024, 2)
    n_emit = (len(x) // 512) * 512
    got = np.fromfile(dump, np.float32)[:n_emit]
    assert rms(got, ref[:n_emit]) <= 1e-5
    assert rms(got, ham[:n_emit]) > 1e-3                       # the window really differs
    check_wav_1lsb(out_wav, ref, len(x), n_emit)


@pytest.mark.parametrize("batched", [False, True])
def test_nan_faithful_leading_silence(cuda, tmp_path, batched):
    """kernel.cu:101-109: atanf(0/0) = NaN for the all-zero bins of digital silence (as at
    the start of testtones/autotune.wav, 1124 zeros) poisons those frames' resynthesis and
    the overlap-add samples they reach; the default (deviation 4) gives phase 0 instead."""
    x = wav.load(REF_440)[0][0][:60000].copy()
    x[:3000] = 0.0                                             # frames 0..7 entirely silent
    path = str(tmp_path / "sil.wav")
    write_pcm16(path, x)
    dump, dump0 = str(tmp_path / "nan.f32"), str(tmp_path / "zero.f32")
    common = [path, "t", str(tmp_path / "o.wav"), "--N", "1024", "--hopdiv", "4"] + (["--batched"] if batched else [])
    run_main(common + ["--nan-faithful", "--dump-f32", dump])
    run_main(common + ["--dump-f32", dump0])
    n_emit = (len(x) // 256) * 256
    got = np.fromfile(dump, np.float32)[:n_emit]
    ref = pvref.compat_process(x, 1024, 4, nan_faithful=True)[:n_emit]
    assert np.isnan(ref).sum() > 1000
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert rms(got[fin], ref[fin]) <= 1e-5
    got0 = np.fromfile(dump0, np.float32)[:n_emit]
    assert np.all(np.isfinite(got0))
    assert rms(got0, pvref.compat_process(x, 1024, 4)[:n_emit]) <= 1e-5


def test_python_mirror_single_arg_and_set_window(cuda):
    import torch
    from pvamd import _lib
    x = np.load(os.path.join(GOLDEN, "sine440_ch0_32768.npy"))
    pv = PhaseVocoder.single_arg(1024, max_frames=128)
    assert (pv.hopSize, pv.outHopSize, pv.timeScale) == (512, 512, 1.0)
    assert np.array_equal(pv.imp, pvref.hann_ref(1024))
    out, _ = pv.process(torch.from_numpy(x).cuda())
    assert rms(out.cpu().numpy()[0], pvref.compat_process(x, 1024, 2, window=pvref.hann_ref(1024))) <= 1e-5
    # an arbitrary caller window (CudaPhase `win`) on a 4-argument handle
    w = (0.3 + 0.7 * np.random.default_rng(3).random(1024)).astype(np.float32)
    h = PhaseVocoder(1024, TIME_SHIFT, 1.0, 4, mode=REF_COMPAT, max_frames=128)
    h.set_window(torch.from_numpy(w).cuda())
    out, _ = h.process(torch.from_numpy(x).cuda())
    assert rms(out.cpu().numpy()[0], pvref.compat_process(x, 1024, 4, window=w)) <= 1e-5
    s = PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, max_frames=16)
    with pytest.raises(Exception):
        s.set_window(torch.from_numpy(w).cuda())
    with pytest.raises(Exception):
        PhaseVocoder(1024, TIME_SHIFT, 0.5, 4, mode=STANDARD, window=_lib.PV_WINDOW_HANN_REF)


@pytest.mark.parametrize("batched", [False, True])
def test_gpu_reproduces_reference_output_testout_wav(cuda, tmp_path, batched):
    """The reference's own output artifact: output/testout.wav = main.cpp
    (PhaseVocoder(256, 't', 1, 2)) on testtones/test.wav.  The GPU driver's 16-bit WAV is
    within 1 LSB of it at every sample, and >= 99.9 % bit-identical
    (tests/golden/make_reference_artifacts.py; the oracle pin is
    tests/test_oracle.py::test_oracle_reproduces_reference_output_testout_wav)."""
    x = np.load(os.path.join(GOLDEN, "ref_test_wav_ch0_int16.npy")).astype(np.float32) / np.float32(32768.0)
    ref_out = np.load(os.path.join(GOLDEN, "ref_testout_wav_L_int16.npy")).astype(np.int64)
    path = str(tmp_path / "test.wav")
    write_pcm16(path, x)
    out_wav = str(tmp_path / "testout.wav")
    run_main([path, "t", out_wav] + (["--batched"] if batched else []))   # main.cpp:84 defaults
    s, sr, bits = wav.load(out_wav)
    assert s.shape == (2, 441000) and bits == 16
    got = np.round(s[0].astype(np.float64) * 32768).astype(np.int64)
    d = got - ref_out
    assert np.abs(d).max() <= 1
    assert np.mean(d == 0) >= 0.999
    assert np.array_equal(s[0], s[1])


@pytest.mark.parametrize("args,N,hop_div,effect,scale", [
    ([], 256, 2, "t", 1.0),                                                  # main.cpp:84 geometry
    (["--N", "1024", "--hopdiv", "4", "--scale", "0.5", "--mode", "std"], 1024, 4, "t", 0.5),
    (["--single-arg", "--N", "512"], 512, 2, "t", 1.0),                     # PhaseVocoder(int)
])
def test_pv_main_rt_callback_stream(cuda, sine440, tmp_path, args, N, hop_div, effect, scale):
    """main.cpp's RT block (main.cpp:45-59) on the drop-in: the RtAudio-shaped callback
    memcpys each nSamps-sample buffer into curr_input and calls analysis()
    (phaseVocoder.h:131-132); the buffers' emitted samples are the oracle's pipeline over the
    stream prefixed with N - hop zeros (the real-time contract, include/pv.h)."""
    path, x = sine440
    x = x[:60000]
    p2 = str(tmp_path / "in.wav")
    write_pcm16(p2, x)
    dump = str(tmp_path / "rt.f32")
    r = subprocess.run([PV_MAIN, p2, effect, str(tmp_path / "rt.wav"), "--rt", "--dump-f32", dump] + args,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(dump, np.float32)
    hop = N // hop_div
    hs = int(scale * hop)
    K = (len(x) // N) * (N // hop)  # frames of the whole buffers pushed
    assert got.shape == (K * hs,)
    xp = np.concatenate([np.zeros(N - hop, np.float32), x[:K * hop]])
    ref = pvref.std_process(xp, N, hop_div, ord(effect), scale, frames=K)
    assert rms(got, ref[:K * hs]) <= 1e-5


KH_CHECK = os.path.join(ROOT, "phase-vocoder_amd", "build", "kernel_h_check")


@pytest.mark.parametrize("N", [256, 1024])
def test_pv_analysis_rt_on_caller_stream(cuda, tmp_path, N):
    """CudaPhase::pv_analysis_RT (karnel/kernel.h:16, kernel.cu:219-260) through the drop-in
    kernel.h: one frame windowed by cudaWindow_HanRT's inline periodic Hann (= the oracle's
    hann_ref), shifted, padded to 2N, 2N FFT, {mag, atanf(Im/Re)} of all 2N bins — against
    the oracle with that window; enqueued on the caller's stream (it waits behind a busy
    kernel there) and the declared 6-argument overload gives the same bits."""
    import json
    rng = np.random.default_rng(7)
    t = np.arange(N) / 44100.0
    x = (0.3 * np.sin(2 * np.pi * 440.0 * t) + 0.05 * rng.standard_normal(N)).astype(np.float32)
    fin, fout = str(tmp_path / "in.f32"), str(tmp_path / "out.f32")
    x.tofile(fin)
    r = subprocess.run([KH_CHECK, str(N), fin, fout], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["pending_while_stream_busy"] and res["overloads_equal"], res
    spec = np.fromfile(fout, np.float32).reshape(2 * N, 2)
    ref = pvref.compat_analysis_frame(x, N, window=pvref.hann_ref(N))
    mag_ref = ref.real
    assert np.max(np.abs(spec[:, 0] - mag_ref)) <= 1e-5 * np.max(mag_ref)
    m = mag_ref > 0
    d = np.abs(spec[:, 1][m].astype(np.float64) - ref.imag[m])
    d = np.minimum(d, np.pi - d)  # atan(Im/Re) is taken modulo pi (kernel.cu:108)
    tol = 32 * np.finfo(np.float32).eps * mag_ref.max() / mag_ref[m] + 4e-7
    assert np.all(d <= tol), f"worst excess {np.max(d / tol):.2f}x of the bound"
    # and it is not the Hamming of pv_analysis_CUFFT
    ham = pvref.compat_analysis_frame(x, N)
    assert np.max(np.abs(spec[:, 0] - ham.real)) > 1e-3 * np.max(mag_ref)
