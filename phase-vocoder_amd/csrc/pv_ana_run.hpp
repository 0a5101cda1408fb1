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
template <int L, bool EKL, int D, bool PACKED, int NA = Geo<L>::E>
__device__ __forceinline__ void ana_run(const AnaParams& p, const AnaLds& lt, float2* tile,
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
    // mirrored-pair split (frame below): every bin analysed, L <= 512 (the L = 1024 kernels
    // sit at their VGPR bound)
#ifdef PV_ANA_NOPAIR
    constexpr bool PAIR = false;
#else
    constexpr bool PAIR = (NA == E) && (L <= 512);
#endif
    constexpr int H = E / 2;
    const int rev = ((64 - lane) & 63) << 2;            // lane reversal l -> (64 - l) mod 64
    const float2* baseT = twsl + lane;                  // split twiddles of the lane's bins
    const int offP = L - lane;                          // partner bins L - lane - 64 i
    const int offP0 = (lane == 0) ? L / 2 : L - lane;   // pair 0's partner (lane 0: bin L/2)
    const float2* baseP = twsl + offP;
    const float2* baseP0 = twsl + offP0;
    const float* eklP = ekl + offP;
    const float* eklP0 = ekl + offP0;
    // e_k of the partner bins: k mod 64 = (64 - lane) mod 64
    const float e_lane_p = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(e_lane)));
    (void)H; (void)baseT; (void)baseP; (void)baseP0; (void)eklP; (void)eklP0; (void)e_lane_p;

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
        float2* prow = specc + (long long)(t0 + u) * p.spec_stride;  // the row
        float2* srow = prow + lane;
        float2* rrow = prow + ((64 - lane) & 63);  // lane-reversed block positions
        (void)srow; (void)prow; (void)rrow;
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
        if constexpr (PAIR) {
            // Mirrored pairs: pair i of lane l is bin k = l + 64 i (i < E/2, slot i) and bin
            // L - k (slot E-1-i), whose split operands are the same A = Z[k], B = Z[L - k]
            // swapped: er, or are the same sums, ei, oi the negated differences (exact), so
            // both bins come from one permute and one set of terms — bit for bit the
            // per-bin formula (contract v2).  Lane 0's partners are bins 64 (E - i), and its
            // pair 0 is (bin 0, bin L/2), bin L/2 being the one bin that is its own mirror:
            // its operands (Z[L/2] twice) come in by a lane-0 select.
            // Row stores: pair i's own bins fill block i; its partners fill block E-1-i at
            // positions 64 (E-1-i) + (64 - l) (l >= 1), whose position 0 is lane 0's partner of
            // pair i + 1 (of pair 0 for the last block, bin L/2).  So each partner store waits
            // for the next pair and takes lane 0's value from it: every store is one aligned
            // 512-byte block (a straddling store measured 15 % slower).
            f2v pprev;         // the previous pair's partner {mag, phase}
            unsigned h0m = 0, h0p = 0;  // lane 0's pair-0 partner (bin L/2), as SGPR bits
            static_for<0, H>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                const float2 A = z[slot_reg<L>(i)];
                const float2 o = z[slot_reg<L>(E - 1 - i)];
                const float2 m = z[slot_reg<L>((E - i) & (E - 1))];
                float2 Bz;
                Bz.x = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(o.x)));
                Bz.y = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(o.y)));
                lane0_mov2(Bz.x, Bz.y, m.x, m.y);  // lane 0 read itself: its partner is m
                const float2 tw = lds_ld(&baseT[64 * i]);
                const float2 twp = lds_ld(i == 0 ? baseP0 : &baseP[-64 * i]);
                const float er = A.x + Bz.x, ei = A.y - Bz.y, orr = A.y + Bz.y, oi = Bz.x - A.x;
                float Xr = __builtin_fmaf(orr, tw.x, __builtin_fmaf(-oi, tw.y, er));  // contract v2
                float Xi = __builtin_fmaf(orr, tw.y, __builtin_fmaf(oi, tw.x, ei));
                float Xrp, Xip;
                if constexpr (i == 0) {
                    if (lane == 0) Xi = 0.0f;  // bin 0 is real
                    // the partner's own operands (B, A), on lane 0 (Z[L/2], Z[L/2])
                    const float2 h = z[slot_reg<L>(H)];
                    const bool l0 = lane == 0;
                    const float ax = l0 ? h.x : Bz.x, ay = l0 ? h.y : Bz.y;
                    const float bx = l0 ? h.x : A.x, by = l0 ? h.y : A.y;
                    const float erp = ax + bx, eip = ay - by, orp = ay + by, oip = bx - ax;
                    Xrp = __builtin_fmaf(orp, twp.x, __builtin_fmaf(-oip, twp.y, erp));
                    Xip = __builtin_fmaf(orp, twp.y, __builtin_fmaf(oip, twp.x, eip));
                } else {
                    // partner terms (er, -ei, or, -oi)
                    Xrp = __builtin_fmaf(orr, twp.x, __builtin_fmaf(oi, twp.y, er));
                    Xip = __builtin_fmaf(orr, twp.y, __builtin_fmaf(-oi, twp.x, -ei));
                }
#ifdef PV_ABL_NOATAN
                const f2v ph2 = f2v{Xi, Xip};
#else
                const f2v ph2 = atan2_pv2(Xi, Xr, Xip, Xrp);
#endif
                const float mag = half_sqrt(__builtin_fmaf(Xr, Xr, Xi * Xi));
                const float magp = half_sqrt(__builtin_fmaf(Xrp, Xrp, Xip * Xip));
                constexpr int sp = E - 1 - i;  // the partner's slot
                const Acc mb = decision_term<Acc>(ph2.x, phprev[i], EKL ? lds_ld(&ekl[lane + 64 * i]) : e_lane);
                const Acc mp = decision_term<Acc>(ph2.y, phprev[sp], EKL ? lds_ld(i == 0 ? &eklP0[0] : &eklP[-64 * i]) : e_lane_p);
                sacc[i] += mb;
                sacc[sp] += mp;
                if (u == 0) {
                    sacc[i] -= mb;
                    sacc[sp] -= mp;
                    if (rec != nullptr) {
                        rec[BP + lane + 64 * i] = __float_as_int(ph2.x);
                        rec[BP + (i == 0 ? offP0 : offP - 64 * i)] = __float_as_int(ph2.y);
                    }
                }
                phprev[i] = ph2.x;
                phprev[sp] = ph2.y;
#ifdef PV_ABL_NOSTORE
                sink += mag + magp;
#else
                if constexpr (PACKED && i == 0) {
                    const f2v s0 = (lane == 0) ? f2v{pack_real_bin(mag, ph2.x), pack_real_bin(magL, phL)}
                                               : f2v{mag, ph2.x};
                    __builtin_nontemporal_store(s0, reinterpret_cast<f2v*>(&srow[0]));
                } else {
                    __builtin_nontemporal_store(f2v{mag, ph2.x}, reinterpret_cast<f2v*>(&srow[64 * i]));
                }
                if constexpr (!PACKED && i == 0)
                    __builtin_nontemporal_store(f2v{magL, phL}, reinterpret_cast<f2v*>(&srow[L - lane]));
                if constexpr (i == 0) {
                    h0m = __builtin_amdgcn_readfirstlane(__float_as_uint(magp));
                    h0p = __builtin_amdgcn_readfirstlane(__float_as_uint(ph2.y));
                } else {
                    // block E - i: the previous pair's partners, lane 0's from this pair
                    float sx = pprev.x, sy = pprev.y;
                    lane0_mov2(sx, sy, magp, ph2.y);
                    __builtin_nontemporal_store(f2v{sx, sy}, reinterpret_cast<f2v*>(&rrow[64 * (E - i)]));
                }
                pprev = f2v{magp, ph2.y};
                if constexpr (i == H - 1) {
                    // block H: the last pair's partners, lane 0's bin L/2
                    float sx = pprev.x, sy = pprev.y;
                    lane0_mov2(sx, sy, __uint_as_float(h0m), __uint_as_float(h0p));
                    __builtin_nontemporal_store(f2v{sx, sy}, reinterpret_cast<f2v*>(&rrow[64 * H]));
                }
#endif
            });
        } else
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
                    const float mag = half_sqrt(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
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
    if constexpr (D > 0) {
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
            int u = 0;
#ifndef PV_ANA_NOROT
            // Register rotation: frames are walked in groups of RR = E / D, after which the
            // window has moved by E registers.  Frame u + r (r < RR) holds its pair q in
            // register (q + D r) mod E, so its D new pairs land in the registers frame u + r - 1
            // no longer needs and no register is shifted (the shifting form costs 2 (E - D)
            // v_mov per frame); the groups end at rotation 0, where the loop below continues.
            // (groups of at most 4 frames: longer unrolled groups blow up the compile)
            // (L = 1024 only with packed rows and at most 12 lane registers analysed — config 4
            // without a spectrum output, 163 VGPRs: with all 16, or natural rows, the rotated
            // loop spills at its 168-VGPR bound; config 4's analysis -4.9 %,
            // profiles/r06_ab_c4_analysis_rot.txt)
            constexpr bool ROT_FITS = L <= 512 || (L == 1024 && NA <= 12 && PACKED);
            if constexpr (E % D == 0 && E / D <= 4 && ROT_FITS) {
                constexpr int RR = E / D;
                const int umain = ufast - ufast % RR;
                auto window_rot = [&](auto rc) {
                    constexpr int r = decltype(rc)::value;
                    const float2* wl = reinterpret_cast<const float2*>(winl) + lane;
#pragma unroll
                    for (int q = 0; q < E; ++q) {
#ifdef PV_ABL_NOWIN
                        const float2 wv = make_float2(1.0f, 1.0f);
#else
                        const float2 wv = lds_ld(&wl[64 * q]);
#endif
                        const float2 s = xr[(q + D * r) % E];
                        z[q].x = s.x * wv.x;
                        z[q].y = s.y * wv.y;
                    }
                };
                for (; u < umain; u += RR) {
                    static_for<0, RR>([&](auto rc) {
                        constexpr int r = decltype(rc)::value;
                        f2v xv[D];  // frame u + r + 1's new pairs (logical E - D .. E - 1)
                        gload_tail<D, E>(xv, src(u + r + 1));
                        frame(u + r, z);  // exactly NST row stores (+ records at u = 0)
                        vm_wait<NSTW>(xv);
#pragma unroll
                        for (int j = 0; j < D; ++j) xr[(D * r + j) % E] = make_float2(xv[j].x, xv[j].y);
                        window_rot(IC<(r + 1) % RR>{});
                    });
                }
            }
#endif
            auto consume = [&](const f2v (&xv)[D]) {
#pragma unroll
                for (int q = 0; q < E - D; ++q) xr[q] = xr[q + D];
#pragma unroll
                for (int j = 0; j < D; ++j) xr[E - D + j] = make_float2(xv[j].x, xv[j].y);
                window(xr, z);
            };
            for (; u < ufast; ++u) {
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
    if (rec != nullptr) {
        if constexpr (PAIR) {
            // slot i < H: bin lane + 64 i; slot E-1-i: its partner; slot E (lane 0): bin L
            PV_FOR_BINS(E, lane, {
                const int kb = (i < H) ? k : (i == E) ? L : (i == E - 1) ? offP0 : offP - 64 * (E - 1 - i);
                rec[kb] = decision_sum(sacc[i], nfr - 1);
                rec[2 * BP + kb] = __float_as_int(phprev[i]);
            })
        } else {
            PV_FOR_BINS(E, lane, { rec[k] = decision_sum(sacc[i], nfr - 1); rec[2 * BP + k] = __float_as_int(phprev[i]); })
        }
    }
#ifdef PV_ABL_NOSTORE
    if (sink == 1234.5f && rec != nullptr) rec[lane] = 0;  // keeps the magnitudes computed
#endif
}

}  // namespace pv
