"""Harmoniser over libpv's pv_harmon* (include/pv.h): K pitch-shifted voices of one input
from a single analysis — the "multiple pitch shifts on a single input" the reference
plans (README.md:50) — optionally mixed with per-voice gains."""
from __future__ import annotations

import ctypes

from . import _lib
from .vocoder import _ptr, _torch


class Harmonizer:
    def __init__(self, samples: int, ratios, hop: int = 4, *, max_channels: int = 1,
                 max_frames: int = 4096, device: int = 0):
        self.ratios = [float(r) for r in ratios]
        K = len(self.ratios)
        cfg = _lib.config(samples, hop, _lib.PV_PITCH_SHIFT, 1.0, _lib.PV_MODE_STANDARD, max_channels,
                          max_frames, device)
        arr = (ctypes.c_float * K)(*self.ratios)
        h = ctypes.c_void_p()
        self._L = _lib.lib()
        _lib.check(self._L.pv_harmonizer_create(ctypes.byref(cfg), arr, K, ctypes.byref(h)),
                   "pv_harmonizer_create")
        self._h = h
        self.device = int(device)
        self.nSamps = int(samples)
        self.hopSize = int(samples) // int(hop)
        self.spec_stride = ((self.nSamps // 2 + 1) + 7) & ~7

    def close(self):
        if getattr(self, "_h", None):
            self._L.pv_harmonizer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def num_frames(self, n: int) -> int:
        return _lib.frame_count(n, self.hopSize)

    def output_length(self, frames: int) -> int:
        return frames * self.hopSize + (self.nSamps - self.hopSize) if frames > 0 else 0

    def harmonize(self, x, gains=None, frames: int | None = None, stream=None):
        """x [C, n] CUDA float32 -> (voices [K, C, olen], mix [C, olen] or None, spec)."""
        torch = _torch()
        x = x.unsqueeze(0) if x.dim() == 1 else x
        C, n = x.shape
        frames = self.num_frames(n) if frames is None else frames
        K = len(self.ratios)
        olen = self.output_length(frames)
        dev = x.device
        spec = torch.zeros((C, frames, self.spec_stride, 2), dtype=torch.float32, device=dev)
        voices = torch.empty((K, C, olen), dtype=torch.float32, device=dev)
        mix, g = None, None
        if gains is not None:
            mix = torch.empty((C, olen), dtype=torch.float32, device=dev)
            g = (ctypes.c_float * K)(*[float(v) for v in gains])
        s = ctypes.c_void_p(int(stream) if stream is not None
                            else torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(self._L.pv_harmonize(self._h, _ptr(x), x.stride(0), n, C, frames, _ptr(spec),
                                        spec.stride(0) // 2, _ptr(voices), voices.stride(1),
                                        voices.stride(0), g, _ptr(mix),
                                        0 if mix is None else mix.stride(0), s), "pv_harmonize")
        return voices, mix, spec
