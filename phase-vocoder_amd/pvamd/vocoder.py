"""Python mirror of the reference's `PhaseVocoder` / `CudaPhase` surface over libpv.

Same names, argument meaning and (optionally) the print-and-exit error behaviour of the
reference, so parity tests read like src/main.cpp:
  PhaseVocoder(samples, effect, scaleFactor, hop)      src/phaseVocoder.h:79-116
  .nSamps .hopSize .outHopSize .timeScale .imp          src/phaseVocoder.h:16-31
  .analysis_CUFFT(input, output, fft, intermediary)     src/phaseVocoder.cpp:25-33
  .resynthesis_CUFFT(backFrame, frontFrame, output)     src/phaseVocoder.cpp:60-76
plus the batched entry points the MI355X design is built around (analysis / resynthesis /
process over channels x frames).  Tensors are torch CUDA tensors (device memory and the
current stream are the only things torch provides here).
"""
from __future__ import annotations

import ctypes
import sys

import numpy as np

from . import _lib
from ._lib import PV_MODE_REF_COMPAT, PV_MODE_STANDARD, PVError

TIME_SHIFT = "t"  # phaseVocoder.h:6
PITCH_SHIFT = "p"  # phaseVocoder.h:7
REF_COMPAT = "ref_compat"
STANDARD = "standard"


def _torch():
    import torch  # plumbing only: device memory + streams

    return torch


def _ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


class PhaseVocoder:
    """`class PhaseVocoder` (src/phaseVocoder.h:9-139) on the MI355X HIP path."""

    def __init__(self, samples: int, effect: str = TIME_SHIFT, scaleFactor: float = 1.0,
                 hop: int = 2, *, mode: str = REF_COMPAT, max_channels: int = 1,
                 max_frames: int = 4096, device: int = 0, exit_on_error: bool = False,
                 window: int = _lib.PV_WINDOW_DEFAULT, nan_faithful: bool = False,
                 spec_layout: int = _lib.PV_SPEC_NATURAL, tables_external: bool = False):
        """window: PV_WINDOW_DEFAULT (the mode's), PV_WINDOW_HAMMING_REF or
        PV_WINDOW_HANN_REF (the 1-argument constructor's, phaseVocoder.h:64-66; see
        `single_arg`); nan_faithful: REF_COMPAT atanf(0/0) = NaN (kernel.cu:101-109);
        spec_layout: PV_SPEC_NATURAL or PV_SPEC_PACKED (STANDARD: bin N/2 folded into slot 0,
        see `unpack_spec`); tables_external: build no tables — `import_tables` (or
        pvamd.dist.broadcast_tables) must load them before any compute call."""
        self.exit_on_error = exit_on_error
        eff = effect if isinstance(effect, int) else ord(effect)
        m = PV_MODE_REF_COMPAT if mode == REF_COMPAT else PV_MODE_STANDARD
        cfg = _lib.config(samples, hop, eff, scaleFactor, m, max_channels, max_frames, device, window,
                          1 if nan_faithful else 0, spec_layout, 1 if tables_external else 0)
        self.window = int(window)
        h = ctypes.c_void_p()
        self._L = _lib.lib()
        self._call(self._L.pv_create(ctypes.byref(cfg), ctypes.byref(h)), "pv_create")
        self._h = h
        info = _lib.new_info()
        self._call(self._L.pv_get_info(self._h, ctypes.byref(info)), "pv_get_info")
        self.info = info
        self.device = int(device)
        self.mode = mode
        self.effect = chr(eff)
        # field names of phaseVocoder.h
        self.nSamps = info.n_samps
        self.N = info.n_samps
        self.hopSize = info.hop
        self.outHopSize = info.out_hop
        self.timeScale = float(scaleFactor) if self.effect == TIME_SHIFT else 1.0
        self.spec_bins = info.spec_bins
        self.spec_stride = info.spec_stride
        self.frames_per_run = info.frames_per_run
        # 0 split path, 1 single q = 1 launch (pv_fused.hip)
        self.single_launch = info.single_launch
        self.single_launch_frames = info.single_launch_frames
        self.lane_constants = info.lane_constants
        self.spec_layout = info.spec_layout

    @classmethod
    def single_arg(cls, samples: int, **kw):
        """`PhaseVocoder(int samples)` (src/phaseVocoder.h:46-78): hop = samples/2,
        timeScale 1, periodic Hann window 0.5f*(1 - cosf(2 pi i/N))."""
        return cls(samples, TIME_SHIFT, 1.0, 2, mode=REF_COMPAT,
                   window=_lib.PV_WINDOW_HANN_REF, **kw)

    def set_window(self, win, stream=None):
        """REF_COMPAT: use the caller's window (CUDA float32 tensor of nSamps) for the
        analysis and the resynthesis, as CudaPhase::*_CUFFT's `win` (kernel.cu:301, :406)."""
        assert win.is_cuda and win.numel() == self.nSamps and win.is_contiguous()
        self._call(self._L.pv_set_window(self._h, _ptr(win), self._stream(stream)), "pv_set_window")

    # -------------------------------------------------------------- plumbing
    def _call(self, status, what):
        if status != _lib.PV_OK:
            if self.exit_on_error:  # the reference's checkCUDAError_ (io.cpp:115-124)
                L = _lib.lib()
                print(f"Cuda error: {what}: {L.pv_last_error().decode()}.", file=sys.stderr)
                sys.exit(1)
            _lib.check(status, what)

    def _stream(self, stream=None):
        if stream is not None:
            return ctypes.c_void_p(int(stream))
        torch = _torch()
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "_h", None):
            self._L.pv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def imp(self) -> np.ndarray:
        """Analysis window (phaseVocoder.h:16 `imp`), host copy."""
        from .tables import analysis_window
        return analysis_window(self.nSamps, self.mode, self.window)

    # -------------------------------------------------------------- geometry
    def num_frames(self, n_samples: int) -> int:
        return _lib.frame_count(n_samples, self.hopSize)

    def output_length(self, frames: int) -> int:
        return int(self._L.pv_output_length(self._h, int(frames)))

    def alloc_spec(self, channels: int, frames: int):
        torch = _torch()
        return torch.zeros((channels, frames, self.spec_stride, 2), dtype=torch.float32,
                           device=f"cuda:{self.device}")

    def unpack_spec(self, spec):
        """Spectrum rows of this handle -> natural {mag, phase} bins 0 .. N/2, as a
        [..., N/2 + 1, 2] float32 tensor (a copy).  PV_SPEC_PACKED rows carry bins 0 and N/2
        in slot 0 as sign-coded magnitudes (include/pv.h pv_unpack_bins): exact."""
        torch = _torch()
        B = self.nSamps // 2 + 1
        if self.spec_layout != _lib.PV_SPEC_PACKED:
            return spec[..., :B, :].clone()
        L = self.nSamps // 2
        out = torch.empty(spec.shape[:-2] + (B, 2), dtype=spec.dtype, device=spec.device)
        out[..., 1:L, :] = spec[..., 1:L, :]
        s0 = spec[..., 0, :]
        pi = torch.tensor(float(np.float32(np.pi)), dtype=spec.dtype, device=spec.device)
        zero = torch.zeros((), dtype=spec.dtype, device=spec.device)
        for dst, src in ((0, s0[..., 0]), (L, s0[..., 1])):
            out[..., dst, 0] = src.abs()
            out[..., dst, 1] = torch.where(torch.signbit(src), pi, zero)
        return out

    def alloc_out(self, channels: int, frames: int):
        torch = _torch()
        return torch.empty((channels, self.output_length(frames)), dtype=torch.float32,
                           device=f"cuda:{self.device}")

    # -------------------------------------------------------------- batched API
    @staticmethod
    def _as2d(x):
        return x.unsqueeze(0) if x.dim() == 1 else x

    def analysis(self, x, frames: int | None = None, n_samples: int | None = None, spec=None,
                 stream=None):
        """x: [C, n] (or [n]) float32 CUDA -> spec [C, frames, spec_stride, 2]."""
        x = self._as2d(x)
        assert x.is_cuda and x.dtype.is_floating_point and x.stride(-1) == 1
        C, n = x.shape
        n_samples = n if n_samples is None else n_samples
        frames = self.num_frames(n_samples) if frames is None else frames
        if spec is None:
            spec = self.alloc_spec(C, frames)
        self._call(self._L.pv_analysis(self._h, _ptr(x), x.stride(0), n_samples, C, frames,
                                       _ptr(spec), spec.stride(0) // 2, self._stream(stream)),
                   "pv_analysis")
        return spec

    def resynthesis(self, spec, frames: int | None = None, out=None, ola_in=None, stream=None):
        """spec [C, frames, spec_stride, 2] -> out [C, frames*outHop + N - outHop]."""
        C = spec.shape[0]
        frames = spec.shape[1] if frames is None else frames
        if out is None:
            out = self.alloc_out(C, frames)
        ld_ola = 0 if ola_in is None else self._as2d(ola_in).stride(0)
        self._call(self._L.pv_resynthesis(self._h, _ptr(spec), spec.stride(0) // 2, C, frames,
                                          _ptr(ola_in), ld_ola, _ptr(out), out.stride(0),
                                          self._stream(stream)), "pv_resynthesis")
        return out

    # -------------------------------------------------------------- stream segments
    def segment_summary(self, spec, frames: int | None = None, stream=None):
        """pv_segment_summary: spec [C, frames, spec_stride, 2] of one segment of a longer
        stream -> summary [C, words] int32 (device)."""
        torch = _torch()
        C = spec.shape[0]
        frames = spec.shape[1] if frames is None else frames
        words = self._L.pv_segment_summary_words(self._h)
        summary = torch.empty((C, words), dtype=torch.int32, device=spec.device)
        self._call(self._L.pv_segment_summary(self._h, _ptr(spec), spec.stride(0) // 2, C, frames,
                                              _ptr(summary), self._stream(stream)), "pv_segment_summary")
        return summary

    def segment_resynthesis(self, spec, frame0: int, summaries=None, frames: int | None = None, out=None,
                            stream=None):
        """pv_segment_resynthesis: the segment starting at stream frame `frame0`, after the
        earlier segments' summaries [s, C, words] (None or empty for the first segment) ->
        its own overlap-add [C, frames*outHop + N - outHop]."""
        C = spec.shape[0]
        frames = spec.shape[1] if frames is None else frames
        if out is None:
            out = self.alloc_out(C, frames)
        seg = 0 if summaries is None else int(summaries.shape[0])
        if seg:
            assert summaries.is_contiguous() and summaries.dtype == _torch().int32
        self._call(self._L.pv_segment_resynthesis(self._h, _ptr(spec), spec.stride(0) // 2, C, frames,
                                                  int(frame0), _ptr(summaries) if seg else None, seg,
                                                  _ptr(out), out.stride(0), self._stream(stream)),
                   "pv_segment_resynthesis")
        return out

    def process(self, x, frames: int | None = None, n_samples: int | None = None, spec=None,
                out=None, stream=None, spectrum: bool = True):
        """analysis -> processing -> resynthesis; returns (out, spec).  spectrum=False: the
        caller gets no spectrum (spec is None) — the single launch keeps the rows on chip, the
        split path uses the handle's own buffer; for pitch > 1 the bins no output bin reads
        are then not analysed (same output bits)."""
        x = self._as2d(x)
        C, n = x.shape
        n_samples = n if n_samples is None else n_samples
        frames = self.num_frames(n_samples) if frames is None else frames
        if not spectrum and spec is not None:
            raise ValueError("spectrum=False with a spec buffer")
        if spectrum and spec is None:
            spec = self.alloc_spec(C, frames)
        if out is None:
            out = self.alloc_out(C, frames)
        self._call(self._L.pv_process(self._h, _ptr(x), x.stride(0), n_samples, C, frames,
                                      _ptr(spec) if spec is not None else None,
                                      spec.stride(0) // 2 if spec is not None else 0, _ptr(out),
                                      out.stride(0), self._stream(stream)), "pv_process")
        return out, spec

    def reserve_spectrum(self):
        """Allocate (once, zeroed) the handle's own spectrum rows that process(spectrum=False)
        uses on the split path, so that such calls can be captured into a graph."""
        self._call(self._L.pv_reserve_spectrum(self._h), "pv_reserve_spectrum")

    # -------------------------------------------------------------- reference per-frame API
    def analysis_CUFFT(self, input, output, fft=None, intermediary=None):
        """PhaseVocoder::analysis_CUFFT (phaseVocoder.cpp:25-33): one frame of nSamps
        samples starting at `input` -> `output` (2N float2 in REF_COMPAT).  `fft` and
        `intermediary` are accepted for signature parity and unused (as in the reference
        the cuFFT path never touches `fft`; the window product stays on chip here)."""
        self._call(self._L.pv_analysis(self._h, _ptr(input), self.nSamps, self.nSamps, 1, 1,
                                       _ptr(output), self.spec_stride, self._stream()),
                   "analysis_CUFFT")

    def resynthesis_CUFFT(self, backFrame, frontFrame, output):
        """PhaseVocoder::resynthesis_CUFFT (phaseVocoder.cpp:60-76): output[0..N) =
        frame(frontFrame) + backFrame[outHop..N) shifted to the front (cudaOverlapAdd,
        kernel.cu:111-119)."""
        ola = backFrame[self.outHopSize:]
        self._call(self._L.pv_resynthesis(self._h, _ptr(frontFrame), self.spec_stride, 1, 1,
                                          _ptr(ola), self.nSamps, _ptr(output), self.nSamps,
                                          self._stream()), "resynthesis_CUFFT")

    # -------------------------------------------------------------- shared tables
    def tables_bytes(self) -> int:
        """Size of this handle's table blob (pv_export_tables with no destination)."""
        n = ctypes.c_size_t()
        self._call(self._L.pv_export_tables(self._h, None, 0, ctypes.byref(n), None), "pv_export_tables")
        return int(n.value)

    def export_tables(self):
        """Constant tables as one uint8 CUDA tensor (header + windows + twiddles + ...)."""
        torch = _torch()
        n = ctypes.c_size_t()
        self._call(self._L.pv_export_tables(self._h, None, 0, ctypes.byref(n), None), "pv_export_tables")
        blob = torch.zeros(n.value, dtype=torch.uint8, device=f"cuda:{self.device}")
        self._call(self._L.pv_export_tables(self._h, _ptr(blob), n.value, ctypes.byref(n),
                                            self._stream()), "pv_export_tables")
        return blob

    def import_tables(self, blob):
        self._call(self._L.pv_import_tables(self._h, _ptr(blob), blob.numel(), self._stream()),
                   "pv_import_tables")

    # -------------------------------------------------------------- profiling (bench.py)
    def profile(self, enable=True):
        """enable: False/0 off, True/1 every launch, k > 1 every k-th call's launches."""
        k = int(enable) if not isinstance(enable, bool) else (1 if enable else 0)
        self._call(self._L.pv_profile_enable(self._h, k), "pv_profile_enable")

    def profile_read(self) -> dict:
        cap = 8
        names = (ctypes.c_char_p * cap)()
        ms = (ctypes.c_double * cap)()
        cnt = (ctypes.c_int * cap)()
        n = self._L.pv_profile_read(self._h, names, ms, cnt, cap)
        return {names[i].decode(): (ms[i], cnt[i]) for i in range(n)}

    def profile_reset(self):
        self._L.pv_profile_reset(self._h)
