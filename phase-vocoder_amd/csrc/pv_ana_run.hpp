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

namespace pv {

// L = 1024: the last FFT pass's twiddles come from the split table (fft_pass TWS_MIN), 6 KB
// less LDS: 3 workgroups per CU instead of 2
template <int L>
constexpr int ana_tws_min() { return L == 1024 ? L / 4 : 0; }
// stage-major twiddle entries the analysis keeps in LDS
template <int L>
constexpr int ana_twl_n() { return ana_tws_min<L>() > 0 ? ana_tws_min<L>() : L; }

// bins per batch of LDS reads + atan2 chains (measured with the bpermute split: 2 vs 3 ->
// config-3 analysis -0.7 %, config 4 +-0.3 %; 4: +0.2 %; with the packed atan2 of a pair,
// 2 vs 4: -1 %)
constexpr int kAnaChunk = 2;

// The per-bin sum of a run's unwrap decisions: at L <= 512 the decision bits unwrap_t summed
// as uint32 (one v_add_u32 per bin and frame); at L = 1024, whose kernels sit at their
// 168-VGPR bound and spill with the integer sums (25 VGPRs), the decisions as exact small
// integers in fp32 (one subtraction more per bin).
template <int L>
using ana_acc_t = typename std::conditional<(L <= 512), unsigned, float>::type;
template <typename Acc>
__device__ __forceinline__ Acc decision_term(float phi, float phi_prev, float e) {
    if constexpr (std::is_same<Acc, unsigned>::value) return __float_as_uint(unwrap_t(phi, phi_prev, e));
    else return unwrap_round(phi, phi_prev, e);
}
// S = the sum of the decisions m of the run's frames after its first (n of them)
__device__ __forceinline__ int decision_sum(unsigned acc, int n) { return (int)((unsigned)n * kRintMagicBits - acc); }
__device__ __forceinline__ int decision_sum(float acc, int) { return -(int)acc; }

// LDS tables the analysis reads
struct AnaLds {
    const float2* twl;   // stage-major twiddles, L-point
    const float2* twsl;  // split twiddles e^{-2 pi i k/N}, k <= L
    const float* winl;   // analysis window, N
    const float* ekl;    // expected advance e_k per bin (EKL) — else e_lane
};

// Row slots per frame: the natural layout writes the lane's bins lane + 64 i (i < E) and
// bin L (E + 1 stores, the last an 8-byte partial write); the packed layout (pv.h
// PV_SPEC_PACKED) folds bin L into slot 0 (E whole-segment stores).  The self-tracked
// prefetch's vmcnt waits count exactly these stores.
template <int E, bool PACKED>
constexpr int row_stores() { return PACKED ? E : E + 1; }

// One wave = one run of frames t0 .. t0 + nfr - 1 of channel c.  The run's first decision
// m0 = m(t0) needs phi(t0 - 1), the previous run's last frame: it is not recomputed here (no
// halo frame) but made by k_carry from the two runs' records.  On return phprev = phi of the
// run's last frame and sacc = the sum over frames t0 + 1 .. t0 + nfr - 1 of the decision
// terms (ana_acc_t).  Rows go out with non-temporal stores (they are read back by
// another launch, long after they would have left the caches).  rec (nullable): the run
// record {S, phi(t0), phi(t0 + nfr - 1)} (kRecFields rows of bins_pad words, phases as their
// float bits).
template <int L, bool EKL, int D, bool PACKED, int RING = 0, int NA = Geo<L>::E>
__device__ __forceinline__ void ana_run(const AnaParams& p, const AnaLds& lt, float2* tile, float* ring,
                                        const float2 (&tw0)[Geo<L>::E], int lane, int c, int t0, int nfr,
                                        float e_lane, int* rec, float (&phprev)[Geo<L>::E + 1],
                                        ana_acc_t<L> (&sacc)[Geo<L>::E + 1]) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr int CH = kAnaChunk;
    // row stores per frame: every slot, or with NA < E the NA analysed ones (+ bin L's
    // separate store in the natural layout, zeros)
    constexpr int NST = (NA < E) ? (PACKED ? NA : NA + 1) : row_stores<E, PACKED>();
    // (PV_ABL_*: diagnostic timing-only ablations for A/B runs, wrong outputs: NOSTORE drops
    // the row stores (the magnitudes go to a sink so that they are still computed), NOATAN
    // the atan2, NOFFT the forward transform, NOWIN the window's LDS reads, L2IN the input's
    // HBM reads: every frame re-reads the run's first frame)
#ifdef PV_ABL_NOSTORE
    constexpr int NSTW = 0;
    float sink = 0.0f;
#else
    constexpr int NSTW = NST;
#endif
    static_assert(!PACKED || CH >= 2, "packed rows: bins 0 and L in one chunk");
    const int BP = p.bins_pad;
    const float2* twl = lt.twl;
    const float2* twsl = lt.twsl;
    const float* winl = lt.winl;
    const float* ekl = lt.ekl;
    (void)ekl;
    // e_k of bin L (with per-lane constants, lane 0's: L is a multiple of 64)
    const float e_L = EKL ? lds_ld(&ekl[L]) : __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(e_lane)));
    const float* xc = p.x + (long long)c * p.ldx;
    float2* specc = p.spec + (long long)c * p.ld_spec;
    using Acc = ana_acc_t<L>;
    PV_FOR_BINS(E, lane, { phprev[i] = 0.0f; sacc[i] = Acc(0); })

    // One frame: window + FFT + split + atan2, spectrum row, decisions, from raw samples.
    auto window = [&](const float2 (&xr)[E], float2 (&z)[E]) {
        const float2* wl = reinterpret_cast<const float2*>(winl) + lane;
#pragma unroll
        for (int q = 0; q < E; ++q) {
#ifdef PV_ABL_NOWIN
            const float2 wv = make_float2(1.0f, 1.0f);
            (void)wl;
#else
            const float2 wv = lds_ld(&wl[64 * q]);  // window samples 2 (lane + 64 q) + {0,1}
#endif
            z[q].x = xr[q].x * wv.x;
            z[q].y = xr[q].y * wv.y;
        }
    };
    // NA < E (pv_process without a spectrum output, pitch > 1: the launcher's instantiation
    // for p.src_hi): only the lane registers p < NA (bins < 64 NA) are analysed, bin L only
    // when NA = E.  Compile-time, so the frame has no data-dependent branch (a runtime one
    // made the compiler copy in-flight prefetch registers: scripts/prefetch_hazards.py)
    static_assert(NA % CH == 0 && NA >= CH && NA <= E, "whole chunks");
    auto frame = [&](int u, float2 (&z)[E]) {
        float2* srow = specc + (long long)(t0 + u) * p.spec_stride + lane;
        (void)srow;
        // the last pass's registers feed the split directly (no final image in LDS)
#ifndef PV_ABL_NOFFT
        fft_run<L, false, false, 0, ana_tws_min<L>()>(z, tile, twl, tw0, lane, twsl);
#endif
        // bin L first (the packed slot 0 pairs it with bin 0): it is real, so its contract
        // phase is +0 or pi and needs no atan2 — computed once, wave-uniformly, instead of as
        // a ninth generic bin on every lane (bin_l_real)
        float magL = 0.0f, phL = 0.0f;
        if constexpr (NA == E) {
        bin_l_real<L, true>(z, twsl, magL, phL);
        // bin L's decision (wave-uniform; lane 0's copy is the one recorded).  Frame t0's
        // decision is against phprev = 0, not phi(t0 - 1): it is taken back out of S at once
        // (wave-uniform branch, once per run) and the phase goes to the record instead.
        {
            const Acc mb = decision_term<Acc>(phL, phprev[E], e_L);
            sacc[E] += mb;
            if (u == 0) {
                sacc[E] -= mb;
                if (rec != nullptr && lane == 0) rec[BP + L] = __float_as_int(phL);
            }
        }
        phprev[E] = phL;
        }
        // bins 0 .. E-1 of the lane in chunks of CH (bounded live registers), all reads of a
        // chunk batched, phases of each pair through the packed atan2
        static_for<0, E / CH>([&](auto ic) {
            constexpr int p0 = decltype(ic)::value * CH;
            // (chunks p0 >= NA: nothing — no bin of theirs is read, their row slots are not
            // written, and NST counts the stores that are)
            if constexpr (p0 >= NA) return;
            float2 X[CH];
            split_chunk_bp<L, CH, true, p0, false>(z, twsl, lane, X);
            float phs[CH];
            static_for<0, CH / 2>([&](auto jj) {
                constexpr int j = 2 * decltype(jj)::value;
#ifdef PV_ABL_NOATAN
                const f2v ph2 = f2v{X[j].y, X[j + 1].y};
#else
                const f2v ph2 = atan2_pv2(X[j].y, X[j].x, X[j + 1].y, X[j + 1].x);
#endif
                phs[j] = ph2.x;
                phs[j + 1] = ph2.y;
            });
            static_for<0, CH>([&](auto cc) {
                constexpr int c2 = decltype(cc)::value;
                constexpr int i = p0 + c2;
                const int k = lane + 64 * i;
                (void)k;
                const float ph = phs[c2];
                {
                    // hardware v_sqrt_f32 (<= 1 ulp): magnitudes only scale the output;
                    // the phase, which drives the unwrap decisions, stays bit-exact.  X
                    // came out doubled (split_chunk_bp TWICE): halve the magnitude.
                    const float mag = 0.5f * __builtin_amdgcn_sqrtf(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
#ifdef PV_ABL_NOSTORE
                    sink += mag;
                    if constexpr (false) {
#else
                    if constexpr (PACKED && i == 0) {
#endif
                        // slot 0: lane 0 carries bins 0 and L (both real), the others bin lane
                        const f2v s0 = (lane == 0) ? f2v{pack_real_bin(mag, ph), pack_real_bin(magL, phL)}
                                                   : f2v{mag, ph};
                        __builtin_nontemporal_store(s0, reinterpret_cast<f2v*>(&srow[0]));
                    } else {
                        __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[64 * i]));
                    }
#ifdef PV_ABL_NOSTORE
                    if constexpr (false) {
#else
                    if constexpr (!PACKED && i == 0) {
#endif
                        // bin L: the same value and address on every lane
                        __builtin_nontemporal_store(f2v{magL, phL}, reinterpret_cast<f2v*>(&srow[L - lane]));
                    }
                    // decision bits (frame t0: as bin L above)
                    const Acc mb = decision_term<Acc>(ph, phprev[i], EKL ? lds_ld(&ekl[k]) : e_lane);
                    sacc[i] += mb;
                    if (u == 0) {
                        sacc[i] -= mb;
                        if (rec != nullptr) rec[BP + k] = __float_as_int(ph);
                    }
                }
                phprev[i] = ph;
            });
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
    const int ufast = (int)min((long long)nfr, max(0LL, lastfull - t0 + 1));
    // steady state, trip u: [load x(u+1)] [compute frame u: NST row stores]
    // [vmcnt(NST): x(u+1) landed, the row stores may still be in flight] [window x(u+1)].
    // The prefetch index is clamped (the last trip reloads its own frame), so the loads
    // and stores are unconditional and the count is exact (gload_pairs / vm_wait).
    if constexpr (D > 0 && RING > 0) {
        // LDS-DMA input ring (RING slots of hop samples per wave): frame v's hop new samples
        // are one or two global_load_lds_dwordx4 (NDMA = hop / 256) into slot v mod RING,
        // issued RING frames ahead of their use, so no VGPR holds samples in flight.
        // Trip u: [frame u: NST row stores] [vmcnt: x(u+1) landed] [ds_read the lane's D
        // pairs of x(u+1)] [window] [DMA x(u+1+RING) into the slot just read].  Ops issued
        // after x(u+1): (RING-1) (NST + NDMA) + NST in the steady state, (RING-1) NDMA +
        // (u+1) NST in the first trips (x(1..RING) issued before the loop) — the wait below
        // uses that lower bound (extra record stores at u = 0 only make it conservative).
        static_assert(D < E, "shifted input: hop < N / 2");
        static_assert(D == 2 || D == 4, "the ring moves 1 KiB DMA pieces: hop = 256 or 512");
        constexpr int NDMA = D / 2;
        constexpr int HOPF = 128 * D;  // floats per slot
        if (ufast > 0) {
            float2 xr[E], z[E];
            const unsigned rbase = __builtin_amdgcn_readfirstlane(lds_addr(ring));
            auto dma = [&](int v, int slot) {
                const float* g = xc + (long long)(t0 + min(v, ufast - 1)) * p.hop + (N - HOPF) + 4 * lane;
#pragma unroll
                for (int j = 0; j < NDMA; ++j) glds16(g + 256 * j, rbase + (unsigned)(slot * HOPF + 256 * j) * 4u);
            };
            {
                f2v x0[E];
                gload_pairs<E>(x0, xc + (long long)t0 * p.hop + 2 * lane);
#pragma unroll
                for (int v = 1; v <= RING; ++v) dma(v, v % RING);
                vm_wait<RING * NDMA>(x0);
#pragma unroll
                for (int q = 0; q < E; ++q) xr[q] = make_float2(x0[q].x, x0[q].y);
                window(xr, z);
            }
            int slot = 1 % RING;  // slot of x(u + 1)
            for (int u = 0; u < ufast; ++u) {
                frame(u, z);  // exactly NST row stores (+ records at u = 0)
                {
                    const int m = min(u, RING - 1);
                    static_for<0, RING>([&](auto mc) {
                        constexpr int M = decltype(mc)::value;
                        constexpr int K = (RING - 1) * NDMA + (M + 1) * NSTW;
                        if (m == M) vm_wait_n<(K < 63 ? K : 63)>();
                    });
                }
                const float* rs = ring + slot * HOPF + 2 * lane;
#pragma unroll
                for (int q = 0; q < E - D; ++q) xr[q] = xr[q + D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[E - D + j] = lds_ld(reinterpret_cast<const float2*>(rs + 128 * j));
                window(xr, z);
                dma(u + 1 + RING, slot);
                slot = (slot + 1 == RING) ? 0 : slot + 1;
            }
        }
    } else if constexpr (D > 0) {
        static_assert(D < E, "shifted input: hop < N / 2");
        if (ufast > 0) {
            float2 xr[E], z[E];
            load_fast(0, xr);
            window(xr, z);
#ifdef PV_ABL_L2IN
            // (timing only: every frame re-reads the run's first frame, an L2 hit)
            auto src = [&](int u) { (void)u; return xc + (long long)t0 * p.hop + 2 * lane; };
#else
            auto src = [&](int u) { return xc + (long long)(t0 + min(u, ufast - 1)) * p.hop + 2 * lane; };
#endif
            auto consume = [&](const f2v (&xv)[D]) {
#pragma unroll
                for (int q = 0; q < E - D; ++q) xr[q] = xr[q + D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[E - D + j] = make_float2(xv[j].x, xv[j].y);
                window(xr, z);
            };
            for (int u = 0; u < ufast; ++u) {
                f2v xv[D];  // the D new pairs of frame u+1: registers E-D .. E-1
                gload_tail<D, E>(xv, src(u + 1));
                frame(u, z);  // exactly NST row stores (+ records at u = 0)
                vm_wait<NSTW>(xv);
                consume(xv);
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
            frame(u, z);  // exactly NST row stores
            vm_wait<NSTW>(xv);
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
            frame(u, z);
        }
    }
    for (int u = ufast; u < nfr; ++u) {
        float2 xr[E], z[E];
        load_checked(u, xr);
        window(xr, z);
        frame(u, z);
    }
    if (rec != nullptr)
        PV_FOR_BINS(E, lane, { rec[k] = decision_sum(sacc[i], nfr - 1); rec[2 * BP + k] = __float_as_int(phprev[i]); })
#ifdef PV_ABL_NOSTORE
    if (sink == 1234.5f && rec != nullptr) rec[lane] = 0;  // keeps the magnitudes computed
#endif
}

}  // namespace pv
