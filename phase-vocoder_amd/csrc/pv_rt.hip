// pv_rt.hip — real-time ring-buffer mode (BASELINE config 5).
//
// The reference only sketches this path: an RtAudio callback copies each input buffer
// into `curr_input` and calls a per-callback `PhaseVocoder::analysis()` that looks back
// at `prev_input` / `prev_mag_phase` / `prev_output` (src/main.cpp:45-59,
// src/phaseVocoder.h:16-31, README.md:46-50, karnel/kernel.cu:219-250 pv_analysis_RT).
// Here one callback is ONE launch over all channels: a wave per channel carries the
// stream state from callback to callback in HBM —
//   hist[c][N - hop]   the input samples the next frame still needs (the ring buffer)
//   phprev[c][B]       phase of the previous frame (unwrap reference)
//   M[c][B]            running unwrap count M(t)
//   ola[c][N - hs]     overlap-add accumulator of positions not yet emitted
//   tcount[c]          frames processed so far
// and per pushed frame runs analysis -> processing -> resynthesis -> overlap-add,
// emitting out_hop final samples.  The per-frame arithmetic is the batched path's
// (pv_frame.hpp), so the stream equals pv_process() over the stream prefixed with
// N - hop zeros, frame for frame (tests/test_gpu_rt.py).
#include "pv_frame.hpp"
#include "pv_kernels.h"

namespace pv {

// W waves (channels) per workgroup.  LDS: tables + per wave {FFT tile, input window
// buffer, overlap accumulator}.
template <int L>
struct RtGeo {
    static constexpr int N = 2 * L;
    static constexpr int B = L + 1;
    static constexpr int W = (L <= 512) ? 4 : 2;
    static constexpr int TILE = Geo<L>::TILE;
    // float offsets
    static constexpr int O_TW = 0;                          // L float2
    static constexpr int O_TWS = O_TW + 2 * L;              // L+1 float2 (+1 pad)
    static constexpr int O_TILE = O_TWS + 2 * (L + 2);      // W x TILE float2
    static constexpr int O_WIN = O_TILE + 2 * W * TILE;     // N
    static constexpr int O_GAIN = O_WIN + N;                // N
    static constexpr int O_EK = O_GAIN + N;                 // B (+3)
    static constexpr int O_JK = O_EK + (B + 3);             // B (+3)
    static constexpr int O_SRC = O_JK + (B + 3);            // 2B (+2), {first, count} pairs
    static constexpr int O_BUF = O_SRC + (2 * B + 2);       // W x N input window
    static_assert(O_SRC % 2 == 0, "pitch map pairs are read as 8-byte words");
    static constexpr int O_OLA = O_BUF + W * N;             // W x N overlap accumulator
    static constexpr int FLOATS = O_OLA + W * N;
    static constexpr size_t BYTES = sizeof(float) * FLOATS;
};

template <int L, int MODE, bool QPOW2>
__global__ __launch_bounds__(256) void k_rt(RtParams p) {
    using G_ = Geo<L>;
    using R_ = RtGeo<L>;
    constexpr int E = G_::E;
    constexpr int N = R_::N;
    constexpr int B = R_::B;
    constexpr int W = R_::W;
    constexpr int SPW = N / 64;
    extern __shared__ __attribute__((aligned(16))) float rsm[];
    float2* twl = reinterpret_cast<float2*>(rsm + R_::O_TW);
    float2* twsl = reinterpret_cast<float2*>(rsm + R_::O_TWS);
    float* winl = rsm + R_::O_WIN;
    float* gainl = rsm + R_::O_GAIN;
    float* ekl = rsm + R_::O_EK;
    unsigned* jkl = reinterpret_cast<unsigned*>(rsm + R_::O_JK);
    int* srcl = reinterpret_cast<int*>(rsm + R_::O_SRC);

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < L; i += 64 * W) twl[i] = p.tw[i];
    for (int i = tid; i < B; i += 64 * W) {
        twsl[i] = p.tws[i];
        ekl[i] = p.ek[i];
        jkl[i] = p.jk_mod[i];
        if (MODE == 2) { srcl[2 * i] = p.src_first[i]; srcl[2 * i + 1] = p.src_cnt[i]; }
    }
    for (int i = tid; i < N; i += 64 * W) { winl[i] = p.win[i]; gainl[i] = p.gain[i]; }
    __syncthreads();

    const int c = blockIdx.x * W + w;
    if (c >= p.channels) return;
    float2* tile = reinterpret_cast<float2*>(rsm + R_::O_TILE) + w * R_::TILE;
    float* buf = rsm + R_::O_BUF + w * N;
    float* olab = rsm + R_::O_OLA + w * N;
    const int hop = p.hop, hs = p.hs;
    const int keep = N - hop;  // history samples carried to the next frame
    const int tl = N - hs;     // overlap samples carried to the next frame

    float* hist = p.hist + (long long)c * N;
    float* olag = p.ola + (long long)c * N;
    for (int j = lane; j < keep; j += 64) buf[j] = hist[j];
    for (int j = lane; j < N; j += 64) olab[j] = (j < tl) ? olag[j] : 0.0f;
    int M[E + 1];
    float phprev[E + 1];
    {
        const int* Mg = p.M + (long long)c * p.bins_pad;
        const float* Pg = p.phprev + (long long)c * p.bins_pad;
        PV_FOR_BINS(E, lane, { M[i] = Mg[k]; phprev[i] = Pg[k]; })
    }
    unsigned t = p.tcount[c];
    const PhaseMap pmap{p.rho * kInv2Pi, (unsigned)p.q, (unsigned)p.p_mod, p.q_pow2, p.inv_q,
                        (float)p.p_mod * p.inv_q, p.rho < 1.0f ? 1 : 0};
    const SynLds stb{twl, twsl, ekl, jkl, srcl};
    const float* inc = p.in + (long long)c * p.ldi;
    float* outc = p.out + (long long)c * p.ldo;

    for (int f = 0; f < p.nframes; ++f, ++t) {
        for (int j = lane; j < hop; j += 64) buf[keep + j] = inc[(long long)f * hop + j];
        wave_lds_sync();
        // ---- analysis (same operations as k_std_analysis)
        float2 z[E];
        {
            const float2* b2 = reinterpret_cast<const float2*>(buf) + lane;
            const float2* w2 = reinterpret_cast<const float2*>(winl) + lane;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const float2 xv = lds_ld(&b2[64 * q]);
                const float2 wv = lds_ld(&w2[64 * q]);
                z[q].x = xv.x * wv.x;
                z[q].y = xv.y * wv.y;
            }
        }
        fft_run<L, false, false>(z, tile, twl, tw0, lane);  // the split reads the last pass's registers
        float2 sv[E + 1];
        float2* srow = (p.spec != nullptr)
                           ? p.spec + (long long)c * p.ld_spec + (long long)f * p.spec_stride
                           : nullptr;
        constexpr int CH = 3;
        static_for<0, (E + CH) / CH>([&](auto ic) {
            constexpr int i0 = decltype(ic)::value * CH;
            float2 X[CH];
            split_chunk_bp<L, CH, false, i0>(z, twsl, lane, X);
#pragma unroll
            for (int c2 = 0; c2 < CH; ++c2) {
                const int i = i0 + c2;
                if (i > E) break;
                const float ph = atan2_pv(X[c2].y, X[c2].x);
                const float mag = __builtin_amdgcn_sqrtf(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
                sv[i] = make_float2(mag, ph);
                if (srow != nullptr && (i < E || lane == 0)) srow[(i == E) ? L : lane + 64 * i] = sv[i];
            }
        });
        wave_lds_sync();
        // ---- processing + resynthesis: time samples to tile (natural order)
        const unsigned q32 = (unsigned)p.q;  // <= 2^24 (QPOW2) or <= 32768
        const unsigned tq = QPOW2 ? ((t + 1u) & (q32 - 1u)) : ((t + 1u) % q32);
        float ekr[E + 1];       // unused (KREG = false)
        unsigned jkr[E + 1];
        synth_frame<L, MODE, true, QPOW2>(sv, true, tq, M, phprev, pmap, stb, tw0, tile, lane, z, ekr, jkr);
        // ---- overlap-add, emit the out hop, shift
        const float* ty = reinterpret_cast<const float*>(tile);
        float nv[SPW];
#pragma unroll
        for (int i = 0; i < SPW; ++i) {
            const int n = lane + 64 * i;
            const float yv = ty[2 * G_::pad(n >> 1) + (n & 1)];
            olab[n] = __builtin_fmaf(yv, gainl[n], olab[n]);
        }
        wave_lds_sync();
        for (int j = lane; j < hs; j += 64) outc[(long long)f * hs + j] = olab[j];
#pragma unroll
        for (int i = 0; i < SPW; ++i) {
            const int n = lane + 64 * i;
            nv[i] = (n < tl) ? olab[n + hs] : 0.0f;
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < SPW; ++i) olab[lane + 64 * i] = nv[i];
        // input window moves by one hop
#pragma unroll
        for (int i = 0; i < SPW; ++i) {
            const int n = lane + 64 * i;
            nv[i] = (n < keep) ? buf[n + hop] : 0.0f;
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < SPW; ++i) {
            const int n = lane + 64 * i;
            if (n < keep) buf[n] = nv[i];
        }
        wave_lds_sync();
    }
    // ---- state back to HBM
    for (int j = lane; j < keep; j += 64) hist[j] = buf[j];
    for (int j = lane; j < tl; j += 64) olag[j] = olab[j];
    {
        int* Mg = p.M + (long long)c * p.bins_pad;
        float* Pg = p.phprev + (long long)c * p.bins_pad;
        PV_FOR_BINS(E, lane, { Mg[k] = M[i]; Pg[k] = phprev[i]; })
    }
    if (lane == 0) p.tcount[c] = t;
}

size_t rt_lds_bytes(int L) {
    switch (L) {
        case 128: return RtGeo<128>::BYTES;
        case 256: return RtGeo<256>::BYTES;
        case 512: return RtGeo<512>::BYTES;
        case 1024: return RtGeo<1024>::BYTES;
    }
    return 0;
}

int rt_waves_per_group(int L) { return L <= 512 ? 4 : 2; }

// mode: 0 STANDARD stretch, 2 STANDARD pitch
hipError_t launch_rt(int L, int mode, const RtParams& p, hipStream_t s) {
    const int W = rt_waves_per_group(L);
    dim3 grid((p.channels + W - 1) / W), block(64 * W);
    const bool qp = p.q_pow2 && p.q <= (1ull << 24);
#define PV_RT_L(LL_)                                                                              \
    if (mode == 2 && qp) hipLaunchKernelGGL((k_rt<LL_, 2, true>), grid, block, RtGeo<LL_>::BYTES, s, p); \
    else if (mode == 2) hipLaunchKernelGGL((k_rt<LL_, 2, false>), grid, block, RtGeo<LL_>::BYTES, s, p); \
    else if (qp) hipLaunchKernelGGL((k_rt<LL_, 0, true>), grid, block, RtGeo<LL_>::BYTES, s, p);   \
    else hipLaunchKernelGGL((k_rt<LL_, 0, false>), grid, block, RtGeo<LL_>::BYTES, s, p);
    switch (L) {
        case 128: PV_RT_L(128); break;
        case 256: PV_RT_L(256); break;
        case 512: PV_RT_L(512); break;
        case 1024: PV_RT_L(1024); break;
        default: return hipErrorInvalidValue;
    }
#undef PV_RT_L
    return hipGetLastError();
}

}  // namespace pv
