"""Standalone batched FFT op over libpv's pv_fft_c2c (include/pv.h): the reference's
FFT::HPFFT::computeGPUFFT / computeGPUIFFT (karnel/hpfft.h:6-11, hpfft.cu:145-203),
radix-2 Stockham, unnormalised in both directions."""
from __future__ import annotations

import ctypes

from . import _lib
from .vocoder import _ptr, _torch


def fft(x, inverse: bool = False, out=None, stream=None):
    """x: complex64 CUDA tensor [..., n] (n a power of two in [2, 2048]) -> same shape."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.complex64 and x.is_contiguous()
    n = x.shape[-1]
    batch = x.numel() // n if n else 0
    if out is None:
        out = torch.empty_like(x)
    s = ctypes.c_void_p(int(stream) if stream is not None
                        else torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(_lib.lib().pv_fft_c2c(_ptr(x), _ptr(out), int(n), int(batch), 1 if inverse else 0, s),
               "pv_fft_c2c")
    return out


def ifft(x, out=None, stream=None):
    return fft(x, inverse=True, out=out, stream=stream)
