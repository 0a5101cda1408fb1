#!/usr/bin/env python3
"""Extract the reference's own output artifacts (and the inputs that produced them) into
small fixtures under tests/golden/ (run in the build container, where /root/reference
exists; the GPU box never reads /root/reference).  Data only: int16 sample arrays and
spectral features, no reference source.

  output/testout.wav      = main.cpp (PhaseVocoder(256, 't', 1, 2): N=256, hop 128,
                            REF_COMPAT, channel 0 only, R = L, 16-bit) run on
                            testtones/test.wav.  Identified by a search over the test
                            tones x N x hop divisor: correlation 1.0 with
                            the oracle, every sample within 1 LSB.  Stored: test.wav ch0
                            (the only channel main.cpp resynthesises) and testout.wav L.
  output/1000hzout.wav,   from testtones/1000sine.wav by a sibling revision of the code
  firsout.wav,            (sample correlation with the oracle <= 0.65, L != R at the head):
  outhop-2inhop-10.wav    only their spectral features are stored — the strongest peaks
                            and the energy in 1/3-octave bands of one 32768-sample segment.
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np

REF = os.environ.get("PV_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
SEG = (4096, 4096 + 32768)


def pcm16_ints(path):
    """16-bit PCM samples as int16 [channels, n] (first "data" chunk; missing bytes -> 0)."""
    data = open(path, "rb").read()
    f, d = data.find(b"fmt"), data.find(b"data")
    ch = struct.unpack_from("<h", data, f + 10)[0]
    assert struct.unpack_from("<h", data, f + 22)[0] == 16
    n = struct.unpack_from("<i", data, d + 4)[0] // (2 * ch)
    raw = data[d + 8:d + 8 + n * 2 * ch]
    raw = raw + bytes(n * 2 * ch - len(raw))
    return np.frombuffer(raw, "<i2").reshape(n, ch).T.copy()


def features(y, sr=44100, k=8):
    """Strongest k spectral peaks (>= 30 Hz apart) and 1/3-octave band energy fractions of
    y[SEG] under a Hann window."""
    seg = np.asarray(y[SEG[0]:SEG[1]], np.float64)
    S = np.abs(np.fft.rfft(seg * np.hanning(len(seg)))) ** 2
    f = np.fft.rfftfreq(len(seg), 1 / sr)
    peaks = []
    for i in np.argsort(S)[::-1]:
        if all(abs(f[i] - p) > 30 for p in peaks):
            peaks.append(float(f[i]))
        if len(peaks) == k:
            break
    edges = 100.0 * 2.0 ** (np.arange(0, 22) / 3.0)  # 100 Hz .. ~13 kHz
    bands = [float(S[(f >= lo) & (f < hi)].sum()) for lo, hi in zip(edges[:-1], edges[1:])]
    tot = float(S.sum())
    return {"peaks_hz": peaks, "band_edges_hz": edges.tolist(), "band_frac": [b / tot for b in bands],
            "rms": float(np.sqrt(np.mean(seg ** 2)))}


def main():
    x = pcm16_ints(os.path.join(REF, "testtones", "test.wav"))
    o = pcm16_ints(os.path.join(REF, "output", "testout.wav"))
    assert np.array_equal(o[0], o[1])
    np.save(os.path.join(OUT, "ref_test_wav_ch0_int16.npy"), x[0])
    np.save(os.path.join(OUT, "ref_testout_wav_L_int16.npy"), o[0])
    meta = {"generator": "tests/golden/make_reference_artifacts.py",
            "testout": {"input": "testtones/test.wav ch0", "N": 256, "hop_div": 2, "scale": 1.0,
                        "frames": 441000, "emitted": (441000 // 128) * 128},
            "sibling_artifacts": {}}
    for name in ("1000hzout", "firsout", "outhop-2inhop-10"):
        a = pcm16_ints(os.path.join(REF, "output", name + ".wav"))[0].astype(np.float64) / 32768.0
        meta["sibling_artifacts"][name] = features(a)
    json.dump(meta, open(os.path.join(OUT, "ref_artifacts.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
