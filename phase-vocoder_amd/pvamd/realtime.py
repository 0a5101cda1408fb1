"""Real-time ring-buffer mode over libpv's pv_rt_* (include/pv.h), BASELINE config 5.

The reference sketches this path only: an RtAudio `callback` (src/main.cpp:45-59) copies
each input buffer into `PhaseVocoder::curr_input` and runs a per-callback `analysis()`
that looks back at `prev_input` / `prev_mag_phase` / `prev_output`
(src/phaseVocoder.h:16-31, README.md:46-50).  `RealTimeVocoder` keeps that shape: state
lives on the device between callbacks, one callback is one hipGraph replay
(`capture` + `callback`), or one `push` on a caller's stream.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .vocoder import PITCH_SHIFT, TIME_SHIFT, _ptr, _torch  # noqa: F401


class RealTimeVocoder:
    def __init__(self, samples: int, effect: str = PITCH_SHIFT, scaleFactor: float = 1.0,
                 hop: int = 4, *, channels: int = 1, device: int = 0):
        eff = effect if isinstance(effect, int) else ord(effect)
        cfg = _lib.config(samples, hop, eff, scaleFactor, _lib.PV_MODE_STANDARD, channels, 1, device)
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(self._L.pv_rt_create(ctypes.byref(cfg), int(channels), ctypes.byref(h)), "pv_rt_create")
        self._h = h
        self.device = int(device)
        self.channels = int(channels)
        self.nSamps = int(samples)
        self.hopSize = int(samples) // int(hop)
        self.outHopSize = int(float(scaleFactor) * self.hopSize) if chr(eff) == TIME_SHIFT else self.hopSize
        self.spec_bins = self.nSamps // 2 + 1
        self.spec_stride = (self.spec_bins + 7) & ~7
        self._graph_frames = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.pv_rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, stream=None):
        if stream is not None:
            return ctypes.c_void_p(int(stream))
        torch = _torch()
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, stream=None):
        _lib.check(self._L.pv_rt_reset(self._h, self._stream(stream)), "pv_rt_reset")

    def push(self, x, out=None, spec=None, stream=None):
        """x: [C, nframes*hop] CUDA float32 -> out [C, nframes*outHop] (device, async)."""
        torch = _torch()
        x = x.unsqueeze(0) if x.dim() == 1 else x
        C, n = x.shape
        assert C == self.channels and n % self.hopSize == 0 and x.stride(-1) == 1
        nf = n // self.hopSize
        if out is None:
            out = torch.empty((C, nf * self.outHopSize), dtype=torch.float32, device=x.device)
        lds = 0 if spec is None else spec.stride(0) // 2
        _lib.check(self._L.pv_rt_push(self._h, _ptr(x), x.stride(0), nf, _ptr(out), out.stride(0),
                                      _ptr(spec), lds, self._stream(stream)), "pv_rt_push")
        return out

    # ---------------------------------------------------------- captured callback
    def capture(self, nframes: int = 1):
        _lib.check(self._L.pv_rt_capture(self._h, int(nframes)), "pv_rt_capture")
        self._graph_frames = int(nframes)
        fi = ctypes.POINTER(ctypes.c_float)()
        fo = ctypes.POINTER(ctypes.c_float)()
        _lib.check(self._L.pv_rt_host_buffers(self._h, ctypes.byref(fi), ctypes.byref(fo)),
                   "pv_rt_host_buffers")
        ni, no = nframes * self.hopSize, nframes * self.outHopSize
        # zero-copy numpy views of the pinned callback buffers
        self.host_in = np.ctypeslib.as_array(fi, shape=(self.channels, ni))
        self.host_out = np.ctypeslib.as_array(fo, shape=(self.channels, no))

    def callback(self, x: np.ndarray | None = None) -> np.ndarray:
        """One synchronous callback: x (host [C, nframes*hop], or None when host_in was
        filled in place) -> host_out view [C, nframes*outHop]."""
        src = None
        if x is not None:
            x = np.ascontiguousarray(x, dtype=np.float32)
            src = x.ctypes.data_as(ctypes.c_void_p)
        _lib.check(self._L.pv_rt_callback(self._h, src, None), "pv_rt_callback")
        return self.host_out
