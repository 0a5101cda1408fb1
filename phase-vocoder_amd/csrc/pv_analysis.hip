// pv_analysis.hip — K1, the analysis kernels (STANDARD and REF_COMPAT), gfx950.
//
// Its own translation unit so that it is compiled without SLP vectorisation
// (-fno-slp-vectorize, Makefile): the per-bin scalar chains (real split, atan2, unwrap)
// then stay scalar instead of being paired into v_pk_* operations that need register
// moves and sign flips to assemble their operands (measured: analysis -6 %, while the
// synthesis, whose packed code is hand-written, is faster with SLP on).
// Pipeline and geometry: pv_kernels.hip header, DESIGN.md §4.
#include "pv_frame.hpp"
#include "pv_kernels.h"

#ifndef PV_NT_SPEC
#define PV_NT_SPEC 1  // non-temporal spectrum row stores in the analysis
#endif
#ifndef PV_SPLIT2X
#define PV_SPLIT2X 1  // real split without its four halvings (split_chunk TWICE): analysis -2 %
#endif
#if PV_SPLIT2X && PV_PK_SPLIT
#error "PV_SPLIT2X is implemented for the scalar real split only"
#endif
#ifndef PV_BINL_FULL
#define PV_BINL_FULL 0  // bin L as a whole 64-byte segment with the row padding (measured: no gain)
#endif
#ifndef PV_ANA_SHIFT
#define PV_ANA_SHIFT 1  // shifted-register input when hop = 128 D (k_std_analysis<L, false, D>)
#endif
#ifndef PV_ANA_PF2
#define PV_ANA_PF2 0  // analysis input prefetch distance 2 (shifted-register path)
#endif
#ifndef PV_ANA_CH
#define PV_ANA_CH 3  // analysis: bins per batch of LDS reads + atan2 chains
#endif

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
// D > 0: hop = 128 D samples, so frame u+1's register q is frame u's register q + D and a
// frame costs only its D new sample pairs per lane (the other E - D are shifted in
// registers): 1/E of the frame's bytes leave L2 instead of all of them.
template <int L, bool EKL, int D = 0>
__global__ __launch_bounds__(256, (L < 512) ? 4 : (L == 512) ? PV_ANA_WAVES512 : (L == 1024) ? 2 : 1) void k_std_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr int B = L + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);   // L   stage-major twiddles
    float2* twsl = twl + L;                           // L+1 split twiddles (+1 pad)
    float2* tiles = twsl + (L + 2);                   // 4 x TILE
    float* winl = reinterpret_cast<float*>(tiles + 4 * G_::TILE);  // N
    float* ekl = winl + N;                            // B
    const int BP = p.bins_pad;

    const int tid = threadIdx.x, lane = tid & 63;
    #ifdef PV_NO_RFL_ANA
    const int w = tid >> 6;
#else
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
#endif
    float2 tw0[Geo<L>::E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < L; i += 256) twl[i] = p.tw[i];
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

    float2* tile = tiles + w * G_::TILE;
    const float* xc = p.x + (long long)c * p.ldx;
    float2* specc = p.spec + (long long)c * p.ld_spec;
    float phprev[E + 1];
    float sacc[E + 1];  // -(sum of the run's decisions): exact small integers in fp32
    PV_FOR_BINS(E, lane, { phprev[i] = 0.0f; sacc[i] = 0.0f; })
    // run record {S, m0}: m0 (the decision of the run's first frame) is stored as soon as
    // it is known, S after the loop
    int* rec = (p.runsum != nullptr) ? p.runsum + ((long long)c * p.nruns + run) * 2 * BP : nullptr;

    // One frame: window + FFT + split + atan2 (+ spectrum row, decisions) from raw samples.
    // HALO (frame t0 - 1): phase only, it seeds phprev.
    auto window = [&](const float2 (&xr)[E], float2 (&z)[E]) {
        const float2* wl = reinterpret_cast<const float2*>(winl) + lane;
#pragma unroll
        for (int q = 0; q < E; ++q) {
            const float2 wv = lds_ld(&wl[64 * q]);  // window samples 2 (lane + 64 q) + {0,1}
            z[q].x = xr[q].x * wv.x;
            z[q].y = xr[q].y * wv.y;
        }
    };
    auto frame = [&](int u, float2 (&z)[E], auto halo_tag) {
        constexpr bool HALO = decltype(halo_tag)::value;
        float2* srow = specc + (long long)(t0 + u) * p.spec_stride + lane;
        (void)srow;
#ifdef PV_ABL_NOFFT  // timing-only ablation: the tile holds the windowed input, no FFT
        pass_store<L, Geo<L>::NPASS - 1>(z, tile, lane);
        wave_lds_sync();
#else
        fft_run<L, false>(z, tile, twl, tw0, lane);
#endif
        // bins in chunks of CH (bounded live registers), all reads of a chunk batched
        constexpr int CH = PV_ANA_CH;
#pragma unroll
        for (int i0 = 0; i0 <= E; i0 += CH) {
            float2 X[CH];
            split_chunk<L, CH, PV_SPLIT2X>(tile, twsl, lane, i0, X);
#pragma unroll
            for (int c2 = 0; c2 < CH; ++c2) {
                const int i = i0 + c2;
                if (i > E) break;
                const int k = (i == E) ? L : lane + 64 * i;
#ifdef PV_ABL_NOATAN  // timing-only ablation: no atan2 (phases wrong)
                const float ph = X[c2].y;
#else
                const float ph = atan2_pv(X[c2].y, X[c2].x);
#endif
                if constexpr (!HALO) {
                    // hardware v_sqrt_f32 (<= 1 ulp): magnitudes only scale the output;
                    // the phase, which drives the unwrap decisions, stays bit-exact
                    float mag = __builtin_amdgcn_sqrtf(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
                    if (PV_SPLIT2X) mag *= 0.5f;  // X came out doubled (split_chunk TWICE)
                    // bin L (i = E) has the same value and address on every lane
#if PV_NT_SPEC && PV_BINL_FULL
                    // non-temporal: the rows are read back by another launch, long after
                    // they would have left L2 (measured: analysis -7 %).  Bin L goes out
                    // with the row's 7 padding bins (zeros) as one whole 64-byte segment
                    // from lanes 0..7 instead of an 8-byte partial write (stride = L + 8).
                    if (i == E) {
                        if (lane < 8)
                            __builtin_nontemporal_store(lane == 0 ? f2v{mag, ph} : f2v{0.0f, 0.0f},
                                                        reinterpret_cast<f2v*>(&srow[L]));
                    } else {
                        __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[64 * i]));
                    }
#elif PV_NT_SPEC
#ifdef PV_ABL_NOSTORE  // timing-only ablation: the stores never execute (p.frames > 0)
                    if (p.frames < 0)
#endif
                    __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[(i == E) ? L - lane : 64 * i]));
#else
                    srow[(i == E) ? L - lane : 64 * i] = make_float2(mag, ph);
#endif
                    // m = -mr; the run's first decision is the record's m0, not part of S:
                    // it is subtracted like every other and added back in the (wave-
                    // uniform, once per run) u == 0 branch
                    const float mr = unwrap_round(ph, phprev[i], EKL ? lds_ld(&ekl[k]) : e_lane);
                    sacc[i] += mr;
                    if (u == 0) {
                        sacc[i] -= mr;
                        if (rec != nullptr && (i < E || lane == 0)) rec[BP + k] = -(int)mr;
                    }
                }
                phprev[i] = ph;
            }
        }
        wave_lds_sync();  // tile reads done before the next frame's pass_store
    };
    auto load_fast = [&](int u, float2 (&xr)[E]) {
        const float* src = xc + (long long)(t0 + u) * p.hop;
#pragma unroll
        for (int q = 0; q < E; ++q) xr[q] = *reinterpret_cast<const float2*>(src + 2 * (lane + 64 * q));
    };
    auto load_checked = [&](int u, float2 (&xr)[E]) {
        const long long base = (long long)(t0 + u) * p.hop;
#pragma unroll
        for (int q = 0; q < E; ++q) {
            const long long s = base + 2 * (lane + 64 * q);
            xr[q].x = (s < p.n) ? xc[s] : 0.0f;
            xr[q].y = (s + 1 < p.n) ? xc[s + 1] : 0.0f;
        }
    };
    // frames whose N samples are all inside [0, n) take the vector-load path; the (at most
    // N/hop) frames at the end of a channel take the bounds-checked path.
    // last frame fully inside: floor((n - N) / hop), -1 when n < N (C++ division truncates
    // toward zero, which for N - hop < n < N would give 0 and read frame 0 past the end)
    const long long lastfull = (p.aligned && p.n >= N) ? (p.n - N) / p.hop : -1;
    if (t0 > 0) {
        float2 xh[E], z[E];
        if (t0 - 1 <= lastfull) load_fast(-1, xh); else load_checked(-1, xh);
        window(xh, z);
        frame(-1, z, std::true_type{});
    }
    const int ufast = (int)min((long long)nfr, max(0LL, lastfull - t0 + 1));
#ifdef PV_CLOCK_PROBE
    // diagnostic build only (MI355X_MICROARCH.md DVFS item 6): shader-clock ticks and
    // 100 MHz real-time ticks around the frame loop; clock = dmemtime / drealtime * 100 MHz
    const unsigned long long clk_c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    // steady state, trip u: [load x(u+1)] [compute frame u: E + 1 row stores]
    // [vmcnt(E + 1): x(u+1) landed, the row stores may still be in flight] [window x(u+1)].
    // The prefetch index is clamped (the last trip reloads its own frame), so the loads
    // and stores are unconditional and the count is exact (gload_pairs / vm_wait).
    if constexpr (D > 0 && PV_ANA_PF2 && 2 * (E + 1) + D <= 63) {  // vmcnt holds 6 bits
        // prefetch distance 2: the wait for x(u+1) (issued at the top of trip u-1, before
        // frame u-1's row stores) no longer has to drain frame u-1's stores (vmcnt counts in
        // issue order), so a frame's stores stay in flight for two trips.  Unrolled by two so
        // the two in-flight buffers never move.
        static_assert(D < E, "shifted input: hop < N / 2");
        if (ufast > 0) {
            float2 xr[E], z[E];
            load_fast(0, xr);
            window(xr, z);
            f2v xa[D], xb[D];
            gload_tail<D, E>(xa, xc + (long long)(t0 + min(1, ufast - 1)) * p.hop + 2 * lane);
            auto shift_in = [&](f2v (&xv)[D]) {
#pragma unroll
                for (int q = 0; q < E - D; ++q) xr[q] = xr[q + D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[E - D + j] = make_float2(xv[j].x, xv[j].y);
                window(xr, z);
            };
            int u = 0;
            for (; u + 1 < ufast; u += 2) {
                gload_tail<D, E>(xb, xc + (long long)(t0 + min(u + 2, ufast - 1)) * p.hop + 2 * lane);
                frame(u, z, std::false_type{});
                // x(u+1): frame u-1's and u's stores may stay in flight (the first pair has
                // no frame u-1 stores between xa and xb, so its count is E + 1 smaller)
                if (u == 0) vm_wait<(E + 1) + D>(xa);
                else vm_wait<2 * (E + 1) + D>(xa);
                shift_in(xa);
                gload_tail<D, E>(xa, xc + (long long)(t0 + min(u + 3, ufast - 1)) * p.hop + 2 * lane);
                frame(u + 1, z, std::false_type{});
                vm_wait<2 * (E + 1) + D>(xb);
                shift_in(xb);
            }
            if (u < ufast) frame(u, z, std::false_type{});  // odd count: the last frame
            vm_wait<0>(xa);  // xa's (clamped) prefetch lands before its registers are reused
        }
    } else if constexpr (D > 0) {
        static_assert(D < E, "shifted input: hop < N / 2");
        if (ufast > 0) {
            float2 xr[E], z[E];
            load_fast(0, xr);
            window(xr, z);
            for (int u = 0; u < ufast; ++u) {
                f2v xv[D];  // the D new pairs of frame u+1: registers E-D .. E-1
                gload_tail<D, E>(xv, xc + (long long)(t0 + min(u + 1, ufast - 1)) * p.hop + 2 * lane);
                frame(u, z, std::false_type{});  // exactly E + 1 row stores (+ records at u = 0)
                vm_wait<E + 1>(xv);
#pragma unroll
                for (int q = 0; q < E - D; ++q) xr[q] = xr[q + D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[E - D + j] = make_float2(xv[j].x, xv[j].y);
                window(xr, z);
            }
        }
    } else if (L <= 1024 && ufast > 0) {
        float2 z[E];
        {
            float2 xr[E];
            load_fast(0, xr);
            window(xr, z);
        }
        for (int u = 0; u < ufast; ++u) {
            f2v xv[E];
            gload_pairs<E>(xv, xc + (long long)(t0 + min(u + 1, ufast - 1)) * p.hop + 2 * lane);
            frame(u, z, std::false_type{});  // exactly E + 1 row stores
            vm_wait<E + 1>(xv);
            float2 xr[E];
#pragma unroll
            for (int q = 0; q < E; ++q) xr[q] = make_float2(xv[q].x, xv[q].y);
            window(xr, z);
        }
    } else if (ufast > 0) {  // L = 2048: compiler-tracked prefetch (the kernel uses AGPRs)
        float2 xr[E];
        load_fast(0, xr);
        for (int u = 0; u < ufast; ++u) {
            float2 z[E];
            window(xr, z);
            load_fast(min(u + 1, ufast - 1), xr);
            frame(u, z, std::false_type{});
        }
    }
    for (int u = ufast; u < nfr; ++u) {
        float2 xr[E], z[E];
        load_checked(u, xr);
        window(xr, z);
        frame(u, z, std::false_type{});
    }
    if (rec != nullptr) PV_FOR_BINS(E, lane, { rec[k] = -(int)sacc[i]; })
#ifdef PV_CLOCK_PROBE
    const unsigned long long clk_c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long clk_r1 = __builtin_amdgcn_s_memrealtime();
    if (p.clk != nullptr && lane == 0) {
        const long long wv = (long long)c * p.nruns + run;
        p.clk[2 * wv] = clk_c1 - clk_c0;
        p.clk[2 * wv + 1] = clk_r1 - clk_r0;
    }
#endif
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
    return sizeof(float2) * (L + (L + 2) + 4 * Geo<L>::TILE) + sizeof(float) * (2 * L + (ekl ? L + 1 : 0));
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

hipError_t launch_std_analysis(int L, int channels, const AnaParams& p, hipStream_t s) {
    dim3 grid((p.nruns + 3) / 4, channels);
    PV_DISPATCH_L(L, {
        const int d = (p.aligned && p.hop % 128 == 0) ? p.hop / 128 : 0;
        if (PV_ANA_SHIFT && p.ek_lane && LL >= 256 && LL <= 1024 && (d == 1 || d == 2 || d == 4) && d < LL / 64) {
            constexpr int E_ = LL / 64;  // D < E (instantiated for every L, run for the checked ones)
            if (d == 1) hipLaunchKernelGGL((k_std_analysis<LL, false, (1 < E_) ? 1 : 0>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
            else if (d == 2) hipLaunchKernelGGL((k_std_analysis<LL, false, (2 < E_) ? 2 : 0>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
            else hipLaunchKernelGGL((k_std_analysis<LL, false, (4 < E_) ? 4 : 0>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
        } else if (p.ek_lane) hipLaunchKernelGGL((k_std_analysis<LL, false>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
        else hipLaunchKernelGGL((k_std_analysis<LL, true>), grid, dim3(256), ana_lds_std<LL>(true), s, p);
    });
    return hipGetLastError();
}

hipError_t launch_compat_analysis(int L, int channels, const AnaParams& p, hipStream_t s) {
    dim3 grid((p.nruns + 3) / 4, channels);
    PV_DISPATCH_L(L, {
        hipLaunchKernelGGL(k_compat_analysis<LL>, grid, dim3(256), ana_lds_compat<LL>(), s, p);
    });
    return hipGetLastError();
}


}  // namespace pv
