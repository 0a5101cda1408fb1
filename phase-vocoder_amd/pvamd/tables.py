"""Host copies of the handle's window tables (same double->float recipes as pv_api.cpp)."""
from __future__ import annotations

import numpy as np


def hann_periodic(N: int) -> np.ndarray:
    n = np.arange(N, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * np.pi * n / N)).astype(np.float32)


def hamming_ref(N: int) -> np.ndarray:
    # phaseVocoder.h:85-89: float omega; imp[i] = 0.54f - 0.46f*cos(omega*i) in float
    omega = np.float32(2.0 * np.pi / (N - 1))
    arg = (omega * np.arange(N, dtype=np.float32)).astype(np.float32)
    return (np.float32(0.54) - np.float32(0.46) * np.cos(arg).astype(np.float32)).astype(np.float32)


def analysis_window(N: int, mode: str) -> np.ndarray:
    return hamming_ref(N) if mode == "ref_compat" else hann_periodic(N)
