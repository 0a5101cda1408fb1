// pv_analysis.hip — K1, the analysis kernels (STANDARD and REF_COMPAT), gfx950.
//
// Its own translation unit, compiled without SLP vectorisation (the per-run body is in
// pv_ana_run.hpp; the synthesis, whose packed code is hand-written, is faster with SLP on).
// Pipeline and geometry: pv_kernels.hip header, DESIGN.md §4.
#include "pv_ana_run.hpp"

namespace pv {

// ------------------------------------------------------------------ K1 STANDARD
// One wave = one run of F consecutive frames (plus the halo frame t0-1, transformed only
// for its phase).  The unwrap decision m(t) = f(phi[t], phi[t-1]) is accumulated in
// registers: S = sum over t in (t0, t0+F) and m0 = m(t0) go to the run record.
// EKL: the expected advance e_k from an LDS table; otherwise (64 a multiple of the hop
// divisor, so e_k depends on k mod 64 only) one register per lane, e_k = ek[lane].
#ifndef PV_ANA_WAVES512
#define PV_ANA_WAVES512 4
#endif
#ifndef PV_ANA_WAVES1024
#define PV_ANA_WAVES1024 3  // 154 VGPRs; LDS (with PV_ANA_TWSHARE) allows 3 workgroups per CU
#endif
// D > 0: hop = 128 D samples, so frame u+1's register q is frame u's register q + D and a
// frame costs only its D new sample pairs per lane (the other E - D are shifted in
// registers): 1/E of the frame's bytes leave L2 instead of all of them.
// PACKED: the pv.h PV_SPEC_PACKED row layout (bin L folded into slot 0).
template <int L, bool EKL, int D, bool PACKED>
__global__ __launch_bounds__(256, (L < 512) ? 4 : (L == 512) ? PV_ANA_WAVES512 : (L == 1024) ? PV_ANA_WAVES1024 : 1) void k_std_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr int B = L + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int TWN = ana_twl_n<L>();
    float2* twl = reinterpret_cast<float2*>(smem);   // TWN stage-major twiddles (L, or L/4)
    float2* twsl = twl + TWN;                         // L+1 split twiddles (+1 pad)
    float2* tiles = twsl + (L + 2);                   // 4 x TILE
    float* winl = reinterpret_cast<float*>(tiles + 4 * G_::TILE);  // N
    float* ekl = winl + N;                            // B

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[Geo<L>::E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < TWN; i += 256) twl[i] = p.tw[i];
    for (int i = tid; i < B; i += 256) {
        twsl[i] = p.tws[i];
        if (EKL) ekl[i] = p.ek[i];
    }
    const float e_lane = EKL ? 0.0f : p.ek[tid & 63];
    for (int i = tid; i < N; i += 256) winl[i] = p.win[i];
    __syncthreads();
    const int run = blockIdx.x * 4 + w, c = blockIdx.y;
    if (run >= p.nruns) return;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    // run record {S, m0}: m0 (the decision of the run's first frame) is stored as soon as
    // it is known, S after the loop
    int* rec = (p.runsum != nullptr) ? p.runsum + ((long long)c * p.nruns + run) * 2 * p.bins_pad : nullptr;
    float phprev[E + 1], sacc[E + 1];
    ana_run<L, EKL, D, PACKED>(p, AnaLds{twl, twsl, winl, ekl}, tiles + w * G_::TILE, tw0, lane, c, t0, nfr,
                               e_lane, rec, phprev, sacc);
}

// ------------------------------------------------------------------ K1 REF_COMPAT
// kernel.cu:299-348: window (Hamming), zero-phase shift + zero pad to 2N, C2C 2N,
// (|X|, atanf(Im/Re)) for all 2N bins.  The 2N-point transform of the real padded frame
// is computed as an L = N point complex FFT + real split; bins > N by symmetry.
template <int L>
__global__ __launch_bounds__(256) void k_compat_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = L;  // window length
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);
    float2* twsl = twl + L;                            // L+1 split twiddles (+1 pad)
    float2* tiles = twsl + (L + 2);
    float* winl = reinterpret_cast<float*>(tiles + 4 * G_::TILE);  // N window samples

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[Geo<L>::E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < L; i += 256) twl[i] = p.tw[i];
    for (int i = tid; i <= L; i += 256) twsl[i] = p.tws[i];
    for (int i = tid; i < N; i += 256) winl[i] = p.win[i];
    __syncthreads();
    const int run = blockIdx.x * 4 + w, c = blockIdx.y;
    if (run >= p.nruns) return;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    float2* tile = tiles + w * G_::TILE;
    const float* xc = p.x + (long long)c * p.ldx;
    float2* specc = p.spec + (long long)c * p.ld_spec;

    for (int u = 0; u < nfr; ++u) {
        const int t = t0 + u;
        const long long base = (long long)t * p.hop;
        float2 z[E];
#pragma unroll
        for (int q = 0; q < E; ++q) {
            const int i = lane + 64 * q;
            // b[2i], b[2i+1] of the shifted/padded 2N buffer (kernel.cu:25-32)
            int src = -1;
            if (2 * i < N / 2) src = 2 * i + N / 2;
            else if (2 * i >= 3 * N / 2) src = 2 * i - 3 * N / 2;
            float b0 = 0.0f, b1 = 0.0f;
            if (src >= 0) {
                const long long s = base + src;
                const float x0 = (s < p.n) ? xc[s] : 0.0f;
                const float x1 = (s + 1 < p.n) ? xc[s + 1] : 0.0f;
                b0 = x0 * winl[src];
                b1 = x1 * winl[src + 1];
            }
            z[q] = make_float2(b0, b1);
        }
        fft_run<L, false>(z, tile, twl, tw0, lane);
        float2* srow = specc + (long long)t * p.spec_stride;
        PV_FOR_BINS(E, lane, {
            const float2 X = real_split<L>(tile, twsl, k);
            const float mag = __builtin_sqrtf(X.x * X.x + X.y * X.y);
            float ph = atanf(X.y / X.x);
            if (X.x == 0.0f && X.y == 0.0f) ph = p.nan_faithful ? __builtin_nanf("") : 0.0f;
            srow[k] = make_float2(mag, ph);
            if (k != 0 && k != L) srow[2 * N - k] = make_float2(mag, -ph);
        })
        wave_lds_sync();
    }
}


// ------------------------------------------------------------------ launchers
template <int L>
static size_t ana_lds_std(bool ekl) {
    return sizeof(float2) * (ana_twl_n<L>() + (L + 2) + 4 * Geo<L>::TILE) + sizeof(float) * (2 * L + (ekl ? L + 1 : 0));
}
template <int L>
static size_t ana_lds_compat() {
    return sizeof(float2) * (L + (L + 2) + 4 * Geo<L>::TILE) + sizeof(float) * L;
}
// twiddles + 4 tiles + 4 rings (tails) [+ gain] + ek/jk + pitch map; with register
// overlap-add at L <= 512 the gains live in registers and gainl is not allocated

#define PV_DISPATCH_L(L_, EXPR)                       \
    switch (L_) {                                     \
        case 128: { constexpr int LL = 128; EXPR; } break;   \
        case 256: { constexpr int LL = 256; EXPR; } break;   \
        case 512: { constexpr int LL = 512; EXPR; } break;   \
        case 1024: { constexpr int LL = 1024; EXPR; } break; \
        case 2048: { constexpr int LL = 2048; EXPR; } break; \
        default: return hipErrorInvalidValue;         \
    }

template <bool PK>
static hipError_t launch_std_analysis_t(int L, dim3 grid, const AnaParams& p, hipStream_t s) {
    PV_DISPATCH_L(L, {
        // shifted-register input when hop = 128 D (D < E)
        const int d = (p.aligned && p.hop % 128 == 0) ? p.hop / 128 : 0;
        if (p.ek_lane && LL >= 256 && LL <= 1024 && (d == 1 || d == 2 || d == 4) && d < LL / 64) {
            constexpr int E_ = LL / 64;  // D < E (instantiated for every L, run for the checked ones)
            if (d == 1) hipLaunchKernelGGL((k_std_analysis<LL, false, (1 < E_) ? 1 : 0, PK>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
            else if (d == 2) hipLaunchKernelGGL((k_std_analysis<LL, false, (2 < E_) ? 2 : 0, PK>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
            else hipLaunchKernelGGL((k_std_analysis<LL, false, (4 < E_) ? 4 : 0, PK>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
        } else if (p.ek_lane) hipLaunchKernelGGL((k_std_analysis<LL, false, 0, PK>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
        else hipLaunchKernelGGL((k_std_analysis<LL, true, 0, PK>), grid, dim3(256), ana_lds_std<LL>(true), s, p);
    });
    return hipGetLastError();
}

hipError_t launch_std_analysis(int L, int channels, const AnaParams& p, hipStream_t s) {
    const dim3 grid((p.nruns + 3) / 4, channels);
    return p.packed ? launch_std_analysis_t<true>(L, grid, p, s) : launch_std_analysis_t<false>(L, grid, p, s);
}

hipError_t launch_compat_analysis(int L, int channels, const AnaParams& p, hipStream_t s) {
    dim3 grid((p.nruns + 3) / 4, channels);
    PV_DISPATCH_L(L, {
        hipLaunchKernelGGL(k_compat_analysis<LL>, grid, dim3(256), ana_lds_compat<LL>(), s, p);
    });
    return hipGetLastError();
}


}  // namespace pv
