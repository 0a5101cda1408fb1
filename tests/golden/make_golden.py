#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the build container,
where /root/reference exists; the GPU box never reads /root/reference).

Independence: everything here is plain numpy (pocketfft, fp64) written from the
reference's source semantics, NOT from oracle/pvref.c, so the CPU tests can pin the
oracle against it (the reference itself cannot be built - nvcc/cuFFT
absent - and has no tests of its own; cuFFT's contract is the DFT).

Inputs are the reference's own fixtures:
  testtones/440sine.wav  (config 1), testtones/1000sine.wav, src/50Hz/*.dat,
  src/50Hz+500Hz/*.dat, src/500Hz+505Hz+12000Hz/*.dat,
and output/1000hzout.wav (a reference output artifact of a sibling revision; only its
spectral signature is used).
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np

REF = os.environ.get("PV_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def wav_pcm16(path, max_frames=None):
    """Minimal independent 16-bit PCM reader (AudioFile.h:418-530 semantics: first "data"
    chunk, x/32768, missing trailing bytes -> 0)."""
    data = open(path, "rb").read()
    f = data.find(b"fmt")
    d = data.find(b"data")
    ch = struct.unpack_from("<h", data, f + 10)[0]
    bits = struct.unpack_from("<h", data, f + 22)[0]
    assert bits == 16
    size = struct.unpack_from("<i", data, d + 4)[0]
    n = size // (2 * ch)
    raw = data[d + 8:d + 8 + n * 2 * ch]
    raw = raw + bytes(n * 2 * ch - len(raw))
    v = np.frombuffer(raw, "<i2").reshape(n, ch).T.astype(np.float64) / 32768.0
    if max_frames:
        v = v[:, :max_frames]
    return v.astype(np.float32), n


def read_dat(path):
    return np.array([float(t) for t in open(path).read().split()], dtype=np.float32)


def hamming_ref(N):
    omega = np.float32(2.0 * np.pi / (N - 1))
    arg = (omega * np.arange(N, dtype=np.float32)).astype(np.float32)
    return (np.float32(0.54) - np.float32(0.46) * np.cos(arg.astype(np.float64)).astype(np.float32)).astype(np.float32)


def compat_frame_spectrum(frame, N, win):
    """kernel.cu:299-348 in fp64: window, zero-phase shift + pad to 2N, FFT 2N,
    (|X|, atan(Im/Re)) with x=y=0 -> 0 (defined deviation)."""
    t = frame.astype(np.float64) * win.astype(np.float64)
    b = np.zeros(2 * N, np.complex128)
    b[:N // 2] = t[N // 2:]
    b[N // 2 + N:] = t[:N // 2]
    X = np.fft.fft(b)
    mag = np.abs(X)
    with np.errstate(divide="ignore", invalid="ignore"):
        ph = np.arctan(X.imag / X.real)
    ph = np.where((X.real == 0) & (X.imag == 0), 0.0, ph)
    return mag, ph


def compat_frame_resynth(mag, ph, N, win):
    """kernel.cu:352-432 in fp64: x'=m cos(phi), y'=x' sin(phi); C2R N on bins 0..N/2
    (numpy irfft = cuFFT C2R / N); swap halves; window."""
    xr = mag[:N // 2 + 1] * np.cos(ph[:N // 2 + 1])
    yi = xr * np.sin(ph[:N // 2 + 1])
    y = np.fft.irfft(xr + 1j * yi, N)
    y = np.roll(y, N // 2)
    return y * win.astype(np.float64)


def compat_process(x, N, hop_div):
    hop = N // hop_div
    n = len(x)
    A = max(0, -(-(n - hop) // hop))
    win = hamming_ref(N)
    out = np.zeros(A * hop + N - hop)
    xp = np.concatenate([x, np.zeros(N, np.float32)])
    for i in range(A):
        mag, ph = compat_frame_spectrum(xp[i * hop:i * hop + N], N, win)
        out[i * hop:i * hop + N] += compat_frame_resynth(mag, ph, N, win)
    return out


def peak_freqs(y, sr, k=3, nfft=None):
    nfft = nfft or (1 << int(np.floor(np.log2(len(y)))))
    seg = y[:nfft] * np.hanning(nfft)
    S = np.abs(np.fft.rfft(seg))
    f = np.fft.rfftfreq(nfft, 1 / sr)
    peaks = []
    for i in np.argsort(S)[::-1]:
        if all(abs(f[i] - p) > 50 for p in peaks):
            peaks.append(float(f[i]))
        if len(peaks) == k:
            break
    return peaks


def main():
    meta = {"generator": "tests/golden/make_golden.py (numpy %s, pocketfft fp64)" % np.__version__}

    # config 1 input: 440sine.wav channel 0 excerpt (int16/32768)
    s440, n440 = wav_pcm16(os.path.join(REF, "testtones/440sine.wav"))
    meta["440sine_samples_per_channel"] = int(n440)
    x = s440[0, :32768].copy()
    np.save(os.path.join(OUT, "sine440_ch0_32768.npy"), x)
    for N, hd in ((1024, 4), (256, 2)):
        y = compat_process(x, N, hd)
        np.save(os.path.join(OUT, f"compat_sine440_N{N}_hd{hd}.npy"), y.astype(np.float32))

    # .dat tones through A4-A7 (REF_COMPAT spectra of the first frame, N=256)
    dats = {"50Hz": "src/50Hz/2048smp@44100.dat", "50Hz+500Hz": "src/50Hz+500Hz/512smp@44100.dat",
            "500Hz+505Hz+12000Hz": "src/500Hz+505Hz+12000Hz/2048smp@44100.dat"}
    for name, rel in dats.items():
        v = read_dat(os.path.join(REF, rel))
        np.save(os.path.join(OUT, f"dat_{name}.npy"), v)
        mag, ph = compat_frame_spectrum(v[:256], 256, hamming_ref(256))
        np.save(os.path.join(OUT, f"compat_spec_{name}_N256.npy"), np.stack([mag, ph]).astype(np.float64))
        # plain DFT known-answer of the raw tone (cuFFT C2C contract)
        np.save(os.path.join(OUT, f"dft_{name}_512.npy"), np.fft.fft(v[:512].astype(np.float64)))

    # 1000 Hz: reference output artifact signature (sibling revision) + input excerpt
    s1k, _ = wav_pcm16(os.path.join(REF, "testtones/1000sine.wav"), 44100)
    np.save(os.path.join(OUT, "sine1000_ch0_44100.npy"), s1k[0].copy())
    o1k, _ = wav_pcm16(os.path.join(REF, "output/1000hzout.wav"))
    meta["1000hzout_peaks_hz"] = peak_freqs(o1k[0, 44100:44100 + 65536].astype(np.float64), 44100)
    y = compat_process(s1k[0], 256, 2)
    meta["compat_1000sine_N256_hd2_peaks_hz"] = peak_freqs(y[4096:4096 + 32768], 44100)

    with open(os.path.join(OUT, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
