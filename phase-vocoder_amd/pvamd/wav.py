"""WAV decode/encode with the reference's AudioFile semantics (src/AudioFile.h).

Host-side plumbing for config 1 (testtones/440sine.wav); not on the GPU hot path.
  decode  AudioFile.h:418-530  first "data" / "fmt" substring search (getIndexOfString
          :1010-1028), PCM only (audioFormat != 1 rejected :455-459), 1-2 channels,
          8-bit (x-128)/128 (:1068-1072), 16-bit x/32768 (:1038-1042),
          24-bit x/8388608 (:506-514), 32-bit PCM decodes to no samples (:515-519).
  encode  AudioFile.h:703-785  16-bit int16(clamp(s,-1,1)*32767) truncating (:1045-1049).
Defined deviation: a data chunk shorter than its header claims (440sine.wav is 2 bytes
short) decodes the missing bytes as 0 instead of reading past the buffer.
"""
from __future__ import annotations

import struct

import numpy as np


class WavError(ValueError):
    pass


def _find(data: bytes, s: bytes) -> int:
    # AudioFile::getIndexOfString scans i < size - len (so a match ending at EOF is missed)
    i = data.find(s, 0, max(0, len(data) - 1))
    return i


def decode(data: bytes):
    """Return (samples [channels, n] float32, sample_rate, bit_depth)."""
    if len(data) < 12 or data[0:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise WavError("this doesn't seem to be a valid .WAV file")
    d = _find(data, b"data")
    f = _find(data, b"fmt")
    if d < 0 or f < 0:
        raise WavError("this doesn't seem to be a valid .WAV file")
    audio_format, channels = struct.unpack_from("<hh", data, f + 8)
    sample_rate, bytes_per_sec = struct.unpack_from("<ii", data, f + 12)
    block, bit_depth = struct.unpack_from("<hh", data, f + 20)
    if audio_format != 1:
        raise WavError("compressed / non-PCM .WAV (audioFormat != 1) is not supported")
    if channels < 1 or channels > 2:
        raise WavError("neither mono nor stereo")
    bps = bit_depth // 8
    if bytes_per_sec != (channels * sample_rate * bit_depth) // 8 or block != channels * bps:
        raise WavError("the header data in this WAV file seems to be inconsistent")
    if bit_depth not in (8, 16, 24, 32):
        raise WavError("unsupported bit depth")
    (chunk,) = struct.unpack_from("<i", data, d + 4)
    n = chunk // (channels * bit_depth // 8)
    start = d + 8
    need = n * block
    raw = data[start:start + need]
    if len(raw) < need:
        raw = raw + bytes(need - len(raw))
    if bit_depth == 32:
        return np.zeros((channels, 0), np.float32), sample_rate, bit_depth
    if bit_depth == 16:
        v = np.frombuffer(raw, dtype="<i2").reshape(n, channels).T
        out = v.astype(np.float32) / np.float32(32768.0)
    elif bit_depth == 8:
        v = np.frombuffer(raw, dtype=np.uint8).reshape(n, channels).T
        out = (v.astype(np.int32) - 128).astype(np.float32) / np.float32(128.0)
    else:  # 24-bit
        b = np.frombuffer(raw, dtype=np.uint8).reshape(n, channels, 3)
        v = (b[..., 2].astype(np.int32) << 16) | (b[..., 1].astype(np.int32) << 8) | b[..., 0]
        v = np.where(v & 0x800000, v | ~0xFFFFFF, v)
        out = v.T.astype(np.float32) / np.float32(8388608.0)
    return np.ascontiguousarray(out, dtype=np.float32), sample_rate, bit_depth


def load(path: str):
    with open(path, "rb") as fh:
        return decode(fh.read())


def encode16(samples: np.ndarray, sample_rate: int = 44100) -> bytes:
    """samples [channels, n] -> 16-bit PCM WAV bytes (AudioFile::saveToWaveFile)."""
    s = np.atleast_2d(np.asarray(samples, dtype=np.float64))
    ch, n = s.shape
    # NaN (REF_COMPAT nan_faithful output) -> 0: the reference's undefined int16 cast of NaN
    # gives 0 on x86 (cvttsd2si -> 0x80000000, low 16 bits)
    ints = np.trunc(np.nan_to_num(np.clip(s, -1.0, 1.0), nan=0.0) * 32767.0).astype("<i2")
    body = ints.T.reshape(-1).tobytes()
    hdr = b"RIFF" + struct.pack("<i", 4 + 24 + 8 + len(body)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<ihhiihh", 16, 1, ch, sample_rate, ch * sample_rate * 2, ch * 2, 16)
    hdr += b"data" + struct.pack("<i", len(body))
    return hdr + body


def save16(path: str, samples: np.ndarray, sample_rate: int = 44100) -> None:
    with open(path, "wb") as fh:
        fh.write(encode16(samples, sample_rate))
