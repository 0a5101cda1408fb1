// wav.hpp — WAV decode/encode with the reference's AudioFile semantics (src/AudioFile.h):
// decode AudioFile.h:418-530 (first "data"/"fmt" match, PCM only, 1-2 channels,
// 8-bit (x-128)/128, 16-bit x/32768, 24-bit x/8388608, 32-bit PCM -> no samples);
// encode AudioFile.h:703-785 (16-bit int16(clamp(s,-1,1)*32767), truncating).
// Defined deviation: a data chunk shorter than its header claims decodes the missing
// bytes as 0 (440sine.wav is 2 bytes short; the reference reads past its buffer).
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

namespace pvwav {

struct Audio {
    int sample_rate = 44100;
    int bit_depth = 16;
    std::vector<std::vector<float>> samples;  // [channel][n]
};

inline int find(const std::vector<uint8_t>& d, const char* s) {
    const size_t n = std::strlen(s);
    for (size_t i = 0; i + n < d.size(); ++i)  // AudioFile::getIndexOfString: i < size - len
        if (std::memcmp(&d[i], s, n) == 0) return (int)i;
    return -1;
}
inline int32_t i32(const std::vector<uint8_t>& d, size_t o) {
    uint32_t v = 0;
    for (int b = 3; b >= 0; --b) v = (v << 8) | (o + b < d.size() ? d[o + b] : 0);
    return (int32_t)v;
}
inline int16_t i16(const std::vector<uint8_t>& d, size_t o) {
    uint16_t v = (uint16_t)((o + 1 < d.size() ? d[o + 1] : 0) << 8 | (o < d.size() ? d[o] : 0));
    return (int16_t)v;
}

inline bool load(const std::string& path, Audio& a, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) { err = "File doesn't exist or otherwise can't load file"; return false; }
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (d.size() < 12 || std::memcmp(&d[0], "RIFF", 4) || std::memcmp(&d[8], "WAVE", 4)) {
        err = "this doesn't seem to be a valid .WAV file"; return false;
    }
    const int di = find(d, "data"), fi = find(d, "fmt");
    if (di < 0 || fi < 0) { err = "this doesn't seem to be a valid .WAV file"; return false; }
    const int fmt = i16(d, fi + 8), ch = i16(d, fi + 10);
    a.sample_rate = i32(d, fi + 12);
    const int bps = i32(d, fi + 16), block = i16(d, fi + 20);
    a.bit_depth = i16(d, fi + 22);
    if (fmt != 1) { err = "compressed / non-PCM .WAV is not supported"; return false; }
    if (ch < 1 || ch > 2) { err = "neither mono nor stereo"; return false; }
    if (bps != ch * a.sample_rate * a.bit_depth / 8 || block != ch * (a.bit_depth / 8)) {
        err = "the header data in this WAV file seems to be inconsistent"; return false;
    }
    if (a.bit_depth != 8 && a.bit_depth != 16 && a.bit_depth != 24 && a.bit_depth != 32) {
        err = "unsupported bit depth"; return false;
    }
    const int n = i32(d, di + 4) / (ch * a.bit_depth / 8);
    const size_t start = di + 8;
    a.samples.assign(ch, {});
    if (a.bit_depth == 32) return true;  // AudioFile.h:515-519 decodes nothing
    for (int c = 0; c < ch; ++c) a.samples[c].resize(n);
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < ch; ++c) {
            const size_t o = start + (size_t)block * i + (size_t)c * (a.bit_depth / 8);
            float v;
            if (a.bit_depth == 16) v = (float)i16(d, o) / 32768.0f;
            else if (a.bit_depth == 8) v = (float)((int)(o < d.size() ? d[o] : 0) - 128) / 128.0f;
            else {
                int32_t s = ((o + 2 < d.size() ? d[o + 2] : 0) << 16) | ((o + 1 < d.size() ? d[o + 1] : 0) << 8) |
                            (o < d.size() ? d[o] : 0);
                if (s & 0x800000) s |= ~0xFFFFFF;
                v = (float)s / 8388608.0f;
            }
            a.samples[c][i] = v;
        }
    return true;
}

inline bool save16(const std::string& path, const std::vector<std::vector<float>>& s, int rate) {
    const int ch = (int)s.size();
    const int n = ch ? (int)s[0].size() : 0;
    std::vector<uint8_t> d;
    auto put = [&](const void* p, size_t k) {
        d.insert(d.end(), (const uint8_t*)p, (const uint8_t*)p + k);
    };
    const int32_t data = n * ch * 2, riff = 4 + 24 + 8 + data, sixteen = 16, bps = rate * ch * 2;
    const int16_t one = 1, chs = (int16_t)ch, block = (int16_t)(ch * 2), bits = 16;
    put("RIFF", 4); put(&riff, 4); put("WAVE", 4); put("fmt ", 4); put(&sixteen, 4); put(&one, 2);
    put(&chs, 2); put(&rate, 4); put(&bps, 4); put(&block, 2); put(&bits, 2); put("data", 4);
    put(&data, 4);
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < ch; ++c) {
            float v = s[c][i];
            v = v > 1.f ? 1.f : (v < -1.f ? -1.f : v);
            // AudioFile.h:1045-1049; NaN (REF_COMPAT nan_faithful) -> 0, what the reference's
            // undefined (int16_t)(NaN) gives on x86 (cvttsd2si 0x80000000, low 16 bits)
            const int16_t q = (v != v) ? (int16_t)0 : (int16_t)(v * 32767.);
            put(&q, 2);
        }
    std::ofstream f(path, std::ios::binary);
    f.write((const char*)d.data(), (std::streamsize)d.size());
    return f.good();
}

}  // namespace pvwav
