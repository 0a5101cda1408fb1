"""Host copies of the handle's window tables (same double->float recipes as pv_api.cpp)."""
from __future__ import annotations

import numpy as np

PV_WINDOW_DEFAULT, PV_WINDOW_HAMMING_REF, PV_WINDOW_HANN_REF = 0, 1, 2


def hann_periodic(N: int) -> np.ndarray:
    n = np.arange(N, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * np.pi * n / N)).astype(np.float32)


def _cosf(arg: np.ndarray) -> np.ndarray:
    # the C library's cosf, as libpv's pv_create (and the reference's host code) calls it
    import ctypes
    import ctypes.util
    m = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
    m.cosf.argtypes = [ctypes.c_float]
    m.cosf.restype = ctypes.c_float
    return np.array([m.cosf(float(a)) for a in np.asarray(arg, np.float32)], np.float32)


def hann_ref(N: int) -> np.ndarray:
    # phaseVocoder.h:64-66 (PhaseVocoder(int samples)): 0.5f * (1.f - cosf(2.f*M_PI*i/samples)),
    # the argument evaluated in double and rounded to float for cosf
    arg = (2.0 * np.pi * np.arange(N, dtype=np.float64) / N).astype(np.float32)
    return (np.float32(0.5) * (np.float32(1.0) - _cosf(arg))).astype(np.float32)


def hamming_ref(N: int) -> np.ndarray:
    # phaseVocoder.h:85-89: float omega; imp[i] = 0.54f - 0.46f*cos(omega*i) in float
    omega = np.float32(2.0 * np.pi / (N - 1))
    arg = (omega * np.arange(N, dtype=np.float32)).astype(np.float32)
    return (np.float32(0.54) - np.float32(0.46) * _cosf(arg)).astype(np.float32)


def analysis_window(N: int, mode: str, window: int = PV_WINDOW_DEFAULT) -> np.ndarray:
    if mode != "ref_compat":
        return hann_periodic(N)
    return hann_ref(N) if window == PV_WINDOW_HANN_REF else hamming_ref(N)
