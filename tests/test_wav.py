"""AudioFile WAV semantics (src/AudioFile.h) of pvamd.wav — host plumbing for config 1."""
import struct

import numpy as np
import pytest

from pvamd import wav


def pcm(samples_i, ch, bits, rate=44100, fmt=1, truncate=0):
    body = samples_i
    hdr = b"RIFF" + struct.pack("<i", 36 + len(body)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<ihhiihh", 16, fmt, ch, rate, rate * ch * bits // 8, ch * bits // 8, bits)
    hdr += b"data" + struct.pack("<i", len(body))
    data = hdr + body
    return data[:len(data) - truncate] if truncate else data


def test_decode_16bit_stereo():
    v = np.array([[0, 16384], [-32768, 32767]], "<i2")  # frames x channels
    s, sr, bits = wav.decode(pcm(v.tobytes(), 2, 16))
    assert sr == 44100 and bits == 16
    assert np.array_equal(s, np.array([[0, -1.0], [0.5, 32767 / 32768]], np.float32))


def test_decode_8bit_and_24bit():
    s, _, _ = wav.decode(pcm(bytes([0, 128, 255]), 1, 8))
    assert np.allclose(s[0], [-1.0, 0.0, 127 / 128])
    raw = bytes([0xff, 0xff, 0x7f, 0x00, 0x00, 0x80])  # +8388607, -8388608
    s, _, _ = wav.decode(pcm(raw, 1, 24))
    assert np.allclose(s[0], [8388607 / 8388608, -1.0])


def test_reject_float_and_decode_32bit_pcm_empty():
    with pytest.raises(wav.WavError):
        wav.decode(pcm(b"\0" * 8, 1, 32, fmt=3))  # MAT_ZO_FLOAT.wav / test_float.wav
    s, _, _ = wav.decode(pcm(b"\0" * 8, 1, 32))
    assert s.shape == (1, 0)


def test_short_data_chunk_reads_zeros():
    # 440sine.wav is 2 bytes short: the last R sample is missing (defined deviation)
    v = np.array([[100, 200], [300, 400]], "<i2")
    s, _, _ = wav.decode(pcm(v.tobytes(), 2, 16, truncate=2))
    assert s[0, 1] == np.float32(300 / 32768) and s[1, 1] == 0.0


def test_encode16_truncates_and_clamps():
    x = np.array([[0.5, -0.5, 2.0, -2.0, 1e-5]])
    data = wav.encode16(x)
    body = np.frombuffer(data[44:], "<i2")
    assert list(body) == [16383, -16383, 32767, -32767, 0]
    s, _, _ = wav.decode(data)
    assert s.shape == (1, 5)


def test_encode16_nan_is_zero():
    body = np.frombuffer(wav.encode16(np.array([[np.nan, 0.25]]))[44:], "<i2")
    assert list(body) == [0, 8191]


def test_reference_440sine_fixture():
    """tests/golden/testtones_440sine.wav = the reference's testtones/440sine.wav (config 1
    input): 441000 frames per the header, the data chunk 2 bytes short (last R missing)."""
    import os
    from conftest import GOLDEN
    data = open(os.path.join(GOLDEN, "testtones_440sine.wav"), "rb").read()
    s, sr, bits = wav.decode(data)
    assert s.shape == (2, 441000) and sr == 44100 and bits == 16
    assert len(data) == 44 + 441000 * 4 - 2 and s[1, -1] == 0.0
    assert np.array_equal(s[0, :32768], np.load(os.path.join(GOLDEN, "sine440_ch0_32768.npy")))
