"""ctypes binding of the CPU oracle (oracle/pvref.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product (phase-vocoder_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libpvref.so")
_lib = None

TIME_SHIFT = ord("t")
PITCH_SHIFT = ord("p")

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c_long, c_int, c_float = ctypes.c_long, ctypes.c_int, ctypes.c_float
        L.pvr_hann_periodic.argtypes = [c_int, _f32p]
        L.pvr_hamming_ref.argtypes = [c_int, _f32p]
        L.pvr_hann_ref.argtypes = [c_int, _f32p]
        L.pvr_fft_twiddles.argtypes = [c_int, _f32p]
        L.pvr_split_twiddles.argtypes = [c_int, _f32p]
        L.pvr_expected_advance.argtypes = [c_int, c_int, _f32p, _i32p]
        L.pvr_atan2f.argtypes = [c_float, c_float]
        L.pvr_atan2f.restype = c_float
        L.pvr_fft_c32.argtypes = [_f32p, _f32p, c_int, _f32p, c_int]
        L.pvr_rfft_c32.argtypes = [_f32p, c_int, _f32p, _f32p, _f32p, _f32p]
        L.pvr_fft_v3_applies.argtypes = [c_int]
        L.pvr_fft_v3_applies.restype = c_int
        L.pvr_fft_v3_table_size.argtypes = [c_int]
        L.pvr_fft_v3_table_size.restype = c_int
        L.pvr_fft_v3_table.argtypes = [c_int, _f32p]
        L.pvr_fft_c32_v3.argtypes = [_f32p, _f32p, c_int, _f32p, c_int]
        L.pvr_rfft_win_c32.argtypes = [_f32p, _f32p, c_int, _f32p, _f32p, _f32p, _f32p]
        L.pvr_contract_version.restype = c_int
        L.pvr_unwrap_count.argtypes = [c_float, c_float, c_float]
        L.pvr_unwrap_count.restype = c_int
        L.pvr_num_frames.argtypes = [c_long, c_int]
        L.pvr_num_frames.restype = c_int
        L.pvr_out_hop.argtypes = [c_int, c_int, c_int, c_float]
        L.pvr_out_hop.restype = c_int
        L.pvr_std_analysis.argtypes = [_f32p, c_long, c_int, c_int, c_int, _f32p]
        L.pvr_std_process.argtypes = [_f32p, c_long, c_int, c_int, c_int, c_float, c_int, _f64p]
        L.pvr_std_process.restype = c_int
        L.pvr_compat_analysis_frame.argtypes = [_f32p, c_int, _f32p, _f64p, c_int]
        L.pvr_compat_resynth_frame.argtypes = [_f64p, c_int, _f32p, _f64p]
        L.pvr_compat_process.argtypes = [_f32p, c_long, c_int, c_int, c_int, _f64p]
        L.pvr_compat_process.restype = c_int
        L.pvr_compat_process_ex.argtypes = [_f32p, c_long, c_int, c_int, c_int, ctypes.c_void_p, c_int, _f64p]
        L.pvr_compat_process_ex.restype = c_int
        L.pvr_compat_process_hs.argtypes = [_f32p, c_long, c_int, c_int, c_int, c_int, ctypes.c_void_p, c_int, _f64p]
        L.pvr_compat_process_hs.restype = c_int
        L.pvr_fft_c64.argtypes = [_f64p, c_int, c_int]
        L.pvr_std_process_batch.argtypes = [_f32p, c_long, c_long, c_int, c_int, c_int, c_int,
                                            c_float, c_int, _f32p, c_long, c_int]
        L.pvr_std_process_batch.restype = c_int
        L.pvr_port_std_process_batch.argtypes = L.pvr_std_process_batch.argtypes
        L.pvr_port_std_process_batch.restype = c_int
        L.pvr_compat_process_batch.argtypes = [_f32p, c_long, c_long, c_int, c_int, c_int, c_int,
                                               _f32p, c_long, c_int]
        L.pvr_compat_process_batch.restype = c_int
        L.pvr_port_compat_process_batch.argtypes = L.pvr_compat_process_batch.argtypes
        L.pvr_port_compat_process_batch.restype = c_int
        _lib = L
    return _lib


def contract_version():
    """version of the fp32 analysis contract this oracle restates (pvref.h)"""
    return int(lib().pvr_contract_version())


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# ---------------------------------------------------------------- tables
def hann_periodic(N):
    w = np.empty(N, np.float32)
    lib().pvr_hann_periodic(N, w)
    return w


def hann_ref(N):
    """PhaseVocoder(int samples) window (phaseVocoder.h:64-66)."""
    w = np.empty(N, np.float32)
    lib().pvr_hann_ref(N, w)
    return w


def hamming_ref(N):
    w = np.empty(N, np.float32)
    lib().pvr_hamming_ref(N, w)
    return w


def fft_twiddles(L):
    tw = np.empty(L, np.float32)  # L/2 complex
    lib().pvr_fft_twiddles(L, tw)
    return tw


def split_twiddles(N):
    tws = np.empty(2 * (N // 2 + 1), np.float32)
    lib().pvr_split_twiddles(N, tws)
    return tws


def expected_advance(N, hop):
    e = np.empty(N // 2 + 1, np.float32)
    j = np.empty(N // 2 + 1, np.int32)
    lib().pvr_expected_advance(N, hop, e, j)
    return e, j


# ---------------------------------------------------------------- primitives
def atan2f(y, x):
    return np.float32(lib().pvr_atan2f(float(y), float(x)))


def fft_c32(z, inverse=False):
    """Contract radix-2 Stockham FFT of a complex64 vector (length power of 2)."""
    z = np.ascontiguousarray(z, dtype=np.complex64)
    L = z.shape[0]
    buf = z.view(np.float32).copy()
    tmp = np.empty_like(buf)
    lib().pvr_fft_c32(buf, tmp, L, fft_twiddles(L), 1 if inverse else 0)
    return buf.view(np.complex64)


def fft_v3_applies(L):
    return bool(lib().pvr_fft_v3_applies(int(L)))


def fft_v3_table(L):
    """contract v3 pass table (pvref.c pvr_fft_v3_table): float32 pairs"""
    t = np.empty(2 * max(1, lib().pvr_fft_v3_table_size(L)), np.float32)
    lib().pvr_fft_v3_table(L, t)
    return t


def analysis_fft_table(L):
    """the table the contract's analysis FFT of L points uses"""
    return fft_v3_table(L) if fft_v3_applies(L) else fft_twiddles(L)


def fft_c32_v3(z, inverse=False):
    """Contract v3 FFT (L in [128, 512], pvref.c pvr_fft_c32_v3)."""
    z = np.ascontiguousarray(z, dtype=np.complex64)
    L = z.shape[0]
    assert fft_v3_applies(L)
    buf = z.view(np.float32).copy()
    tmp = np.empty_like(buf)
    lib().pvr_fft_c32_v3(buf, tmp, L, fft_v3_table(L), 1 if inverse else 0)
    return buf.view(np.complex64)


def rfft_c32(xw):
    """the contract's real FFT of windowed samples (v3 FFT for N/2 <= 512, no window fold)"""
    xw = _c32(xw)
    N = xw.shape[0]
    X = np.empty(2 * (N // 2 + 1), np.float32)
    work = np.empty(2 * N, np.float32)
    lib().pvr_rfft_c32(xw, N, analysis_fft_table(N // 2), split_twiddles(N), X, work)
    return X.view(np.complex64)


def rfft_win_c32(x, w):
    """the contract's analysis transform of raw samples x with window w (x * w, then
    rfft_c32)"""
    x, w = _c32(x), _c32(w)
    N = x.shape[0]
    X = np.empty(2 * (N // 2 + 1), np.float32)
    work = np.empty(2 * N, np.float32)
    lib().pvr_rfft_win_c32(x, w, N, analysis_fft_table(N // 2), split_twiddles(N), X, work)
    return X.view(np.complex64)


def unwrap_count(phi, phi_prev, e):
    return lib().pvr_unwrap_count(float(phi), float(phi_prev), float(e))


def num_frames(n, hop):
    return lib().pvr_num_frames(int(n), int(hop))


def out_hop(N, hop_div, effect, scale):
    return lib().pvr_out_hop(N, hop_div, effect, float(scale))


def fft_c64(z, inverse=False):
    a = np.ascontiguousarray(z, dtype=np.complex128).copy()
    lib().pvr_fft_c64(a.view(np.float64), a.shape[0], 1 if inverse else 0)
    return a


# ---------------------------------------------------------------- pipelines
def std_analysis(x, N, hop, frames=None):
    """fp32 contract analysis -> complex64-shaped array [frames, N/2+1] of (mag + i*phase)."""
    x = _c32(x)
    if frames is None:
        frames = num_frames(x.shape[0], hop)
    spec = np.empty(frames * (N // 2 + 1) * 2, np.float32)
    lib().pvr_std_analysis(x, x.shape[0], N, hop, frames, spec)
    s = spec.reshape(frames, N // 2 + 1, 2)
    return s[..., 0].copy(), s[..., 1].copy()


def std_process(x, N, hop_div, effect, scale, frames=None):
    x = _c32(x)
    hop = N // hop_div
    if frames is None:
        frames = num_frames(x.shape[0], hop)
    hs = out_hop(N, hop_div, effect, scale)
    out = np.zeros(frames * hs + (N - hs), np.float64)
    lib().pvr_std_process(x, x.shape[0], N, hop_div, effect, float(scale), frames, out)
    return out


def std_process_batch(x, N, hop_div, effect, scale, frames=None, threads=0):
    """x: [C, n] float32. Returns (out [C, len] float32, threads_used)."""
    x = _c32(x)
    C, n = x.shape
    hop = N // hop_div
    if frames is None:
        frames = num_frames(n, hop)
    hs = out_hop(N, hop_div, effect, scale)
    olen = frames * hs + (N - hs)
    out = np.zeros((C, olen), np.float32)
    used = lib().pvr_std_process_batch(x, n, n, C, N, hop_div, effect, float(scale), frames,
                                       out, olen, int(threads))
    return out, used


def port_std_process_batch(x, N, hop_div, effect, scale, frames=None, threads=0):
    """The fp32 CPU port (oracle/pvport.c): x [C, n] float32 -> (out [C, len] float32,
    threads used).  bench.py's cpu_baseline; pinned to std_process_batch by the tests."""
    x = _c32(x)
    C, n = x.shape
    hop = N // hop_div
    if frames is None:
        frames = num_frames(n, hop)
    hs = out_hop(N, hop_div, effect, scale)
    olen = frames * hs + (N - hs)
    out = np.zeros((C, olen), np.float32)
    used = lib().pvr_port_std_process_batch(x, n, n, C, N, hop_div, effect, float(scale), frames,
                                            out, olen, int(threads))
    return out, used


def compat_process_batch(x, N, hop_div, frames=None, threads=0):
    """REF_COMPAT per channel (x: [C, n] float32, OpenMP over channels).
    Returns (out [C, len] float32, threads_used)."""
    x = _c32(x)
    C, n = x.shape
    hop = N // hop_div
    if frames is None:
        frames = num_frames(n, hop)
    olen = frames * hop + (N - hop)
    out = np.zeros((C, olen), np.float32)
    used = lib().pvr_compat_process_batch(x, n, n, C, N, hop_div, frames, out, olen, int(threads))
    return out, used


def port_compat_process_batch(x, N, hop_div, frames=None, threads=0):
    """The fp32 CPU port of REF_COMPAT (oracle/pvport.c): x [C, n] float32 -> (out [C, len]
    float32, threads used).  The compat line's cpu_baseline; pinned to compat_process_batch
    (the fp64 restatement) by the tests."""
    x = _c32(x)
    C, n = x.shape
    hop = N // hop_div
    if frames is None:
        frames = num_frames(n, hop)
    olen = frames * hop + (N - hop)
    out = np.zeros((C, olen), np.float32)
    used = lib().pvr_port_compat_process_batch(x, n, n, C, N, hop_div, frames, out, olen, int(threads))
    return out, used


def compat_analysis_frame(frame, N, nan_faithful=False, window=None):
    """kernel.cu:299-348 on one frame; window: float32[N] (None = the Hamming of the
    4-argument constructor; hann_ref(N) = cudaWindow_HanRT of pv_analysis_RT)."""
    b = np.empty(4 * N, np.float64)
    w = hamming_ref(N) if window is None else _c32(window)
    lib().pvr_compat_analysis_frame(_c32(frame), N, w, b, 1 if nan_faithful else 0)
    return b.view(np.complex128)  # (mag + i*phase) per bin, 2N bins


def compat_process(x, N, hop_div, frames=None, window=None, nan_faithful=False, out_hop=None):
    """REF_COMPAT whole-signal path; window: float32[N] (None = the Hamming of the
    4-argument constructor); out_hop: the overlap-add hop of a time scale, (int)(scale * hop)
    (None = hop)."""
    x = _c32(x)
    hop = N // hop_div
    hs = hop if out_hop is None else int(out_hop)
    if frames is None:
        frames = num_frames(x.shape[0], hop)
    out = np.zeros(frames * hs + (N - hs), np.float64)
    w = None if window is None else _c32(window)
    lib().pvr_compat_process_hs(x, x.shape[0], N, hop_div, hs, frames,
                                None if w is None else w.ctypes.data, 1 if nan_faithful else 0, out)
    return out
