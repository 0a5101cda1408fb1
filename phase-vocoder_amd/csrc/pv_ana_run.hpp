// pv_ana_run.hpp — one wave's STANDARD analysis run (window -> real FFT -> {mag, phase}
// rows -> unwrap decisions) of the split path's K1 (k_std_analysis, pv_analysis.hip).
//
// Its translation unit is compiled without SLP vectorisation (-fno-slp-vectorize,
// Makefile): the per-bin scalar chains (real split, atan2, unwrap) then stay scalar instead
// of being paired into v_pk_* operations that need register moves and sign flips to
// assemble their operands (measured: analysis -6 %).
#pragma once
#include "pv_frame.hpp"
#include "pv_kernels.h"

#ifndef PV_NT_SPEC
#define PV_NT_SPEC 1  // non-temporal spectrum row stores in the split path's analysis
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
#ifndef PV_ANA_TWSHARE
#define PV_ANA_TWSHARE 1  // L = 1024: the last pass's twiddles from the split table (fft_pass
                          // TWS_MIN), 6 KB less LDS: 3 workgroups per CU instead of 2
#endif
namespace pv {
template <int L>
constexpr int ana_tws_min() { return (PV_ANA_TWSHARE && L == 1024) ? L / 4 : 0; }
// stage-major twiddle entries the analysis keeps in LDS
template <int L>
constexpr int ana_twl_n() { return ana_tws_min<L>() > 0 ? ana_tws_min<L>() : L; }
}  // namespace pv
#ifndef PV_ANA_CH
#define PV_ANA_CH 2  // analysis: bins per batch of LDS reads + atan2 chains (measured with the
                     // bpermute split: 2 vs 3 -> c3 analysis -0.7 %, c4 +-0.3 %; 4 +0.2 %)
#endif

#ifdef PV_ABL_NOFFT
#define PV_ABL_NOFFT_ON 1
#else
#define PV_ABL_NOFFT_ON 0
#endif

namespace pv {

// LDS tables the analysis reads (the kernels' carve-ups differ)
struct AnaLds {
    const float2* twl;   // stage-major twiddles, L-point
    const float2* twsl;  // split twiddles e^{-2 pi i k/N}, k <= L
    const float* winl;   // analysis window, N
    const float* ekl;    // expected advance e_k per bin (EKL) — else e_lane
};

// One wave = one run of frames t0 .. t0 + nfr - 1 of channel c.  The frame t0 - 1 (halo)
// is transformed too (phase only) to seed phprev, so the run's first decision m0 = m(t0)
// is known here and goes to the run record.  On return phprev = phi of the run's last
// frame and sacc = -(sum of the decisions of frames t0 + 1 .. t0 + nfr - 1) as exact small
// integers in fp32.
// NT: non-temporal row stores (the rows are read back by another launch, long after they
// would have left the caches).  rec (nullable): the run record {S, m0}.
template <int L, bool EKL, int D, bool NT>
__device__ __forceinline__ void ana_run(const AnaParams& p, const AnaLds& lt, float2* tile,
                                        const float2 (&tw0)[Geo<L>::E], int lane, int c, int t0, int nfr,
                                        float e_lane, int* rec, float (&phprev)[Geo<L>::E + 1],
                                        float (&sacc)[Geo<L>::E + 1]) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr bool SPLIT_BP = PV_SPLIT_BP && !PV_ABL_NOFFT_ON;
    const int BP = p.bins_pad;
    const float2* twl = lt.twl;
    const float2* twsl = lt.twsl;
    const float* winl = lt.winl;
    const float* ekl = lt.ekl;
    (void)ekl;
    const float* xc = p.x + (long long)c * p.ldx;
    float2* specc = p.spec + (long long)c * p.ld_spec;
    PV_FOR_BINS(E, lane, { phprev[i] = 0.0f; sacc[i] = 0.0f; })

    // One frame: window + FFT + split + atan2 (+ spectrum row, decisions) from raw samples.
    // IS_HALO (frame t0 - 1): phase only, it seeds phprev.
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
        constexpr bool IS_HALO = decltype(halo_tag)::value;
        float2* srow = specc + (long long)(t0 + u) * p.spec_stride + lane;
        (void)srow;
#ifdef PV_ABL_NOFFT  // timing-only ablation: the tile holds the windowed input, no FFT
        pass_store<L, Geo<L>::NPASS - 1>(z, tile, lane);
        wave_lds_sync();
#else
        // SPLIT_BP: the last pass's registers feed the split directly (no final image)
        fft_run<L, false, !SPLIT_BP, 0, ana_tws_min<L>()>(z, tile, twl, tw0, lane, twsl);
#endif
        // bins in chunks of CH (bounded live registers), all reads of a chunk batched
        constexpr int CH = PV_ANA_CH;
        static_for<0, (E + CH) / CH>([&](auto ic) {
            constexpr int i0 = decltype(ic)::value * CH;
            float2 X[CH];
            if constexpr (SPLIT_BP) split_chunk_bp<L, CH, PV_SPLIT2X, i0>(z, twsl, lane, X);
            else split_chunk<L, CH, PV_SPLIT2X>(tile, twsl, lane, i0, X);
#pragma unroll
            for (int c2 = 0; c2 < CH; ++c2) {
                const int i = i0 + c2;
                if (i > E) break;
                const int k = (i == E) ? L : lane + 64 * i;
                (void)k;
#ifdef PV_ABL_NOATAN  // timing-only ablation: no atan2 (phases wrong)
                const float ph = X[c2].y;
#else
                const float ph = atan2_pv(X[c2].y, X[c2].x);
#endif
                if constexpr (!IS_HALO) {
                    // hardware v_sqrt_f32 (<= 1 ulp): magnitudes only scale the output;
                    // the phase, which drives the unwrap decisions, stays bit-exact
                    float mag = __builtin_amdgcn_sqrtf(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
                    if (PV_SPLIT2X) mag *= 0.5f;  // X came out doubled (split_chunk TWICE)
                    // bin L (i = E) has the same value and address on every lane
                    if constexpr (NT && PV_BINL_FULL) {
                        // bin L goes out with the row's 7 padding bins (zeros) as one whole
                        // 64-byte segment from lanes 0..7 instead of an 8-byte partial write
                        if (i == E) {
                            if (lane < 8)
                                __builtin_nontemporal_store(lane == 0 ? f2v{mag, ph} : f2v{0.0f, 0.0f},
                                                            reinterpret_cast<f2v*>(&srow[L]));
                        } else {
                            __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[64 * i]));
                        }
                    } else if constexpr (NT) {
#ifdef PV_ABL_NOSTORE  // timing-only ablation: the stores never execute (p.frames > 0)
                        if (p.frames < 0)
#endif
#ifdef PV_TMP_NOBINL
                        if (i < E)
#endif
                        __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[(i == E) ? L - lane : 64 * i]));
                    } else {
                        *reinterpret_cast<f2v*>(&srow[(i == E) ? L - lane : 64 * i]) = f2v{mag, ph};
                    }
                    // m = -mr; the run's first decision is the record's m0 (or the
                    // caller's), not part of S: it is subtracted like every other and added
                    // back in the (wave-uniform, once per run) u == 0 branch
                    const float mr = unwrap_round(ph, phprev[i], EKL ? lds_ld(&ekl[k]) : e_lane);
                    sacc[i] += mr;
                    if (u == 0) {
                        sacc[i] -= mr;
                        if (rec != nullptr && (i < E || lane == 0)) rec[BP + k] = -(int)mr;
                    }
                }
                phprev[i] = ph;
            }
        });
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
        const long long wv = (long long)c * p.nruns + t0 / p.F;
        p.clk[2 * wv] = clk_c1 - clk_c0;
        p.clk[2 * wv + 1] = clk_r1 - clk_r0;
    }
#endif
}

}  // namespace pv
