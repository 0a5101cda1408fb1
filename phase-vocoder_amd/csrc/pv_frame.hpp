// pv_frame.hpp — per-frame building blocks shared by the batched kernels (pv_kernels.hip)
// and the real-time kernel (pv_rt.hip): the real-FFT split of the analysis transform and
// the whole synthesis of one frame (phase propagation -> polar->rect -> C2R pre-split ->
// inverse FFT).
#pragma once
#include "pv_device.hpp"


namespace pv {

// Real-FFT split of bin k (0 <= k <= L) from the natural-order L-point transform in tile.
template <int L>
__device__ __forceinline__ float2 real_split(const float2* tile, const float2* __restrict__ tws, int k) {
    using G_ = Geo<L>;
    const float2 A = tile[G_::pad(k & (L - 1))];
    const float2 Bz = tile[G_::pad((L - k) & (L - 1))];
    const float er = 0.5f * (A.x + Bz.x);
    const float ei = 0.5f * (A.y - Bz.y);
    const float orr = 0.5f * (A.y + Bz.y);
    const float oi = 0.5f * (Bz.x - A.x);
    const float2 tw = tws[k];
    float Xr = __builtin_fmaf(orr, tw.x, __builtin_fmaf(-oi, tw.y, er));  // contract v2
    float Xi = __builtin_fmaf(orr, tw.y, __builtin_fmaf(oi, tw.x, ei));
    if (k == 0 || k == L) Xi = 0.0f;
    return make_float2(Xr, Xi);
}

// Bins i0 .. i0+CH-1 of a lane (reads batched; entries past E are dummies).
// TWICE: X is returned scaled by exactly 2 (the four halvings dropped).  Scaling by a
// power of two commutes with every rounding here, so 2X is bit-exactly twice the
// contract's X and atan2 of it is the contract's phase bit for bit (a = min/max and the
// sign tests are scale-free); the caller halves the magnitude.
template <int L, int CH, bool TWICE = false>
__device__ __forceinline__ void split_chunk(const float2* tile, const float2* twsl, int lane, int i0,
                                            float2 (&X)[CH]) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    // A = Z[k], B = Z[(L-k) mod L], k = lane + 64 i: affine in i from two per-lane bases;
    // only (lane 0, i = 0) wraps (B = Z[0]) and bin L (i = E, lane 0) uses Z[0] twice.
    const float2* baseA = tile + G_::pad(lane);
    const float2* baseB = tile + G_::pad(L - lane);
    const float2* baseT = twsl + lane;
    float2 A[CH], Bz[CH], tw[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int i = i0 + c;
        if (i < E) {
            A[c] = lds_ld(&baseA[G_::padc(64 * i)]);
            Bz[c] = lds_ld((i == 0 && lane == 0) ? tile : &baseB[-G_::padc(64 * i)]);
            tw[c] = lds_ld(&baseT[64 * i]);
        } else {
            A[c] = lds_ld(tile);
            Bz[c] = A[c];
            tw[c] = lds_ld(&twsl[L]);
        }
    }
    // (scalar form: a packed-instruction split measured slower, latency-bound chains)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int i = i0 + c;
        constexpr float h = TWICE ? 1.0f : 0.5f;
        const float er = h * (A[c].x + Bz[c].x);
        const float ei = h * (A[c].y - Bz[c].y);
        const float orr = h * (A[c].y + Bz[c].y);
        const float oi = h * (Bz[c].x - A[c].x);
        float Xr = __builtin_fmaf(orr, tw[c].x, __builtin_fmaf(-oi, tw[c].y, er));  // contract v2
        float Xi = __builtin_fmaf(orr, tw[c].y, __builtin_fmaf(oi, tw[c].x, ei));
        if (i >= E || (i == 0 && lane == 0)) Xi = 0.0f;  // bins 0 and L are real
        X[c] = make_float2(Xr, Xi);
    }
}

// register index holding slot c after the last FFT pass (inverse of last_slot)
template <int L>
constexpr int slot_reg(int c) {
    for (int idx = 0; idx < Geo<L>::E; ++idx)
        if (last_slot<L>(idx) == c) return idx;
    return -1;
}

// Order in which a frame's bins are split: 0, 1, .., E (bin L last), or with PACKED
// 0, E, 1, .., E-1 (bins 0 and L in the first chunk: the packed row layout stores them in
// one slot).
template <int E, bool PACKED>
constexpr int bin_at(int pos) { return !PACKED ? pos : pos == 0 ? 0 : pos == 1 ? E : pos - 1; }

// split_chunk from the last FFT pass's registers instead of the natural-order image in LDS
// (no final tile store, no tile reads): lane l holds Z[l + 64 c] in register slot_reg(c), so
// A = Z[k], k = l + 64 i, is the lane's own register and B = Z[(L - k) mod L] =
// Z[(64 - l) + 64 (E - 1 - i)] is register slot E-1-i of lane 64 - l — a lane reversal by
// ds_bpermute (crossbar only).  Lane 0's partners are its own registers (Z[(L - 64 i) mod L]
// = slot (E - i) mod E): its permute reads itself and lane0_mov2 then puts them in.  Same
// operands, same operations as split_chunk: bit-identical bins.  Chunk positions P0 ..
// P0 + CH - 1 are bins bin_at<E, PACKED>(position) (positions past E are dummies).
template <int L, int CH, bool TWICE, int P0, bool PACKED = false>
__device__ __forceinline__ void split_chunk_bp(const float2 (&v)[Geo<L>::E], const float2* twsl, int lane,
                                               float2 (&X)[CH]) {
    constexpr int E = Geo<L>::E;
    const int rev = ((64 - lane) & 63) << 2;
    const float2* baseT = twsl + lane;
    float2 A[CH], Bz[CH], tw[CH];
    static_for<0, CH>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        constexpr int i = (P0 + c <= E) ? bin_at<E, PACKED>(P0 + c) : E;
        if constexpr (i < E) {
            A[c] = v[slot_reg<L>(i)];
            const float2 o = v[slot_reg<L>(E - 1 - i)];
            const float2 m = v[slot_reg<L>((E - i) & (E - 1))];
#ifdef PV_LANE0_PRESEL
            if constexpr (true) {
#else
            if constexpr (L >= 1024) {
#endif
                // (the L = 1024 kernels sit at their 168-VGPR bound: m is selected before the
                // permute rather than kept live across it, which spills there)
                const bool l0 = lane == 0;
                const float sx = l0 ? m.x : o.x, sy = l0 ? m.y : o.y;
                Bz[c].x = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(sx)));
                Bz[c].y = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(sy)));
            } else {
                Bz[c].x = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(o.x)));
                Bz[c].y = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(o.y)));
                lane0_mov2(Bz[c].x, Bz[c].y, m.x, m.y);  // lane 0 read itself: its partner is m
            }
            tw[c] = lds_ld(&baseT[64 * i]);
        } else {
            // bin L, computed by every lane (all store the same value to one address):
            // A = B = Z[0], lane 0's slot 0, broadcast
            const float2 z0 = v[slot_reg<L>(0)];
            A[c] = make_float2(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(z0.x))),
                               __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(z0.y))));
            Bz[c] = A[c];
            tw[c] = lds_ld(&twsl[L]);
        }
    });
    static_for<0, CH>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        constexpr int i = (P0 + c <= E) ? bin_at<E, PACKED>(P0 + c) : E;
        constexpr float h = TWICE ? 1.0f : 0.5f;
        const float er = h * (A[c].x + Bz[c].x);
        const float ei = h * (A[c].y - Bz[c].y);
        const float orr = h * (A[c].y + Bz[c].y);
        const float oi = h * (Bz[c].x - A[c].x);
        float Xr = __builtin_fmaf(orr, tw[c].x, __builtin_fmaf(-oi, tw[c].y, er));  // contract v2
        float Xi = __builtin_fmaf(orr, tw[c].y, __builtin_fmaf(oi, tw[c].x, ei));
        if (i >= E || (i == 0 && lane == 0)) Xi = 0.0f;  // bins 0 and L are real
        X[c] = make_float2(Xr, Xi);
    });
}

// Bin L of the real split, wave-uniform: A = B = Z[0] (lane 0's slot 0, broadcast), the same
// operations as split_chunk_bp's bin L, then {magnitude, contract phase} of a real bin.  With
// Im X = +0 the contract's atan2_pv(+0, X) has a = 0, so the polynomial gives +0 and only the
// x < 0 fix-up applies: pi for X < 0, +0 otherwise (X = -0 included) — bit for bit the generic
// bin's phase, without its reciprocal, polynomial and octant fix-ups.  The magnitude is the
// generic bin's formula (Im^2 = +0).  TWICE: X scaled by 2 as in split_chunk_bp (the caller's
// magnitude is halved here too, so magL is the contract's |X|).
template <int L, bool TWICE>
__device__ __forceinline__ void bin_l_real(const float2 (&v)[Geo<L>::E], const float2* twsl, float& magL,
                                           float& phL) {
    const float2 z0 = v[slot_reg<L>(0)];
    const float ax = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(z0.x)));
    const float ay = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(z0.y)));
    const float2 tw = lds_ld(&twsl[L]);
    constexpr float h = TWICE ? 1.0f : 0.5f;
    const float er = h * (ax + ax);
    const float orr = h * (ay + ay);
    const float oi = h * (ax - ax);
    const float Xr = __builtin_fmaf(orr, tw.x, __builtin_fmaf(-oi, tw.y, er));  // contract v2
    const float zero = 0.0f;
    const float m = __builtin_amdgcn_sqrtf(__builtin_fmaf(Xr, Xr, zero * zero));
    magL = TWICE ? 0.5f * m : m;
    phL = (Xr < 0.0f) ? kPi : 0.0f;
}

// bin_l_real from the natural-order image in LDS (the fused kernel's split reads the tile):
// Z[0] = tile[0], the same address on every lane
template <int L, bool TWICE>
__device__ __forceinline__ void bin_l_real_tile(const float2* tile, const float2* twsl, float& magL, float& phL) {
    const float2 z0 = lds_ld(tile);
    const float ax = z0.x, ay = z0.y;
    const float2 tw = lds_ld(&twsl[L]);
    constexpr float h = TWICE ? 1.0f : 0.5f;
    const float er = h * (ax + ax);
    const float orr = h * (ay + ay);
    const float oi = h * (ax - ax);
    const float Xr = __builtin_fmaf(orr, tw.x, __builtin_fmaf(-oi, tw.y, er));  // contract v2
    const float zero = 0.0f;
    const float m = __builtin_amdgcn_sqrtf(__builtin_fmaf(Xr, Xr, zero * zero));
    magL = TWICE ? 0.5f * m : m;
    phL = (Xr < 0.0f) ? kPi : 0.0f;
}

// bins of a lane: k = lane + 64 i (i < E), plus k = L on lane 0 (i == E)
#define PV_FOR_BINS(E_, lane_, ...)                              \
    _Pragma("unroll") for (int i = 0; i <= (E_); ++i) {          \
        if (i == (E_) && (lane_) != 0) break;                    \
        const int k = (i == (E_)) ? 64 * (E_) : (lane_) + 64 * i; \
        (void)k;                                                 \
        __VA_ARGS__                                              \
    }


// STANDARD phase propagation constants: phi_s = rho phi + 2 pi ((p M_tot) mod q) / q,
// M_tot = M_dec + (t+1) j_k
struct PhaseMap {
    float rho_rev;  // rho / (2 pi): output phases are carried in revolutions
    unsigned q, p_mod;
    int q_pow2;
    float inv_q;
    float p_over_q;  // (p mod q) / q (RACC)
    int multi;       // pitch ratio < 1: some bins have several sources (else at most one)
};

// LDS tables of the synthesis side (see the kernels' carve-up)
struct SynLds {
    const float2* twl;    // stage-major twiddles, L-point
    const float2* twsl;   // e^{-2 pi i k/N}, k <= L
    const float* ekl;     // expected advance e_k (STANDARD)
    const unsigned* jkl;  // (p j_k) mod q (STANDARD)
    const int* srcl;      // pitch map: {first source bin, source count} per bin [B] (MODE 2)
};

// One synthesis frame from the spectrum row sv (mag, phase of the lane's bins k = lane +
// 64 i, i < E, and k = L on lane 0).  MODE 0/2 STANDARD stretch/pitch (MODE 3: pitch with
// at most one source per bin — ratio >= 1 — fixed at compile time) (unwrap state M,
// phprev updated; add_decision = false for a run's first frame, whose decision the carry
// already holds), MODE 1 REF_COMPAT (kernel.cu:121-129 y-bug), MODE 5: sv is the output
// spectrum Y itself (k_fused MODE 4).  tq = (t + 1) mod q.
// Result: STORE_LAST: time samples in tile (natural order, padded); else the inverse
// FFT's last-pass registers z (point lane + 64 last_slot(idx)).
// QPOW2: the output-phase denominator q is a power of two <= 2^24 (compile-time path);
// otherwise the generic path handles any q the handle accepts.
// KREG: the per-bin unwrap constants e_k, (p j_k) mod q come from the caller's registers
// (ekr, jkr: frame-invariant, loaded once per wave) instead of LDS reads every frame.
// RACC (QPOW2 with q <= 4096): M[i] carries the float bits of R = ((p M) mod q) / q, the
// unwrap count's output-phase offset in revolutions, updated as fract(R - m p/q), and jkl
// holds (p j_k mod q) / q as floats; every value is a multiple of 1/q below 2^12, so all of
// it is exact in fp32 and equals the integer path's offset up to whole revolutions (which
// sin/cos ignore), for 3 VALU operations per bin less.
struct NoHook {
    __device__ void operator()() const {}
};
// where the inverse real-FFT pre-step takes its split twiddles from: LDS, or the caller's
// registers (v[q] = twiddle of bin lane + 64 q, loaded once per run)
struct NoTwReg {
    static constexpr bool ON = false;
};
template <int E>
struct TwReg {
    static constexpr bool ON = true;
    float2 v[E];
};
// hook(): called once the spectrum row sv has been consumed (before the inverse real-FFT
// pre-step) — the batched kernel issues the next row's loads there into the same registers.
// Q1: the output-phase denominator is q = 1 (integer ratio, e.g. pitch 2.0): the unwrap
// count drops out of the output phase (rho phi + 2 pi ((p M) mod 1) = rho phi), so the
// unwrap state is neither read nor updated; phc = fma(rho / 2 pi, phi, +0) is bit for bit
// what the RACC path computes with q = 1 (R = tj = +0).
template <int L, int MODE, bool STORE_LAST, bool QPOW2 = false, bool KREG = false, bool RACC = false,
          bool Q1 = false, typename Hook = NoHook, typename TwS = NoTwReg, bool V3X = false>
__device__ __forceinline__ void synth_frame(const float2 (&sv)[Geo<L>::E + 1], bool add_decision,
                                            unsigned tq, int (&M)[Geo<L>::E + 1],
                                            float (&phprev)[Geo<L>::E + 1], const PhaseMap& pm,
                                            const SynLds& tb, const float2 (&tw0)[Geo<L>::E],
                                            float2* tile, int lane, float2 (&z)[Geo<L>::E],
                                            const float (&ekr)[Geo<L>::E + 1],
                                            const unsigned (&jkr)[Geo<L>::E + 1],
                                            const Hook& hook = Hook{}, const TwS& twr = TwS{}) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int B = L + 1;
    const float2* twl = tb.twl;
    const float2* twsl = tb.twsl;
    const float* ekl = tb.ekl;
    const unsigned* jkl = tb.jkl;
    const int* srcl = tb.srcl;
    (void)ekl; (void)jkl; (void)srcl; (void)B;
    float mag[E + 1], ph[E + 1];
    PV_FOR_BINS(E, lane, { mag[i] = sv[i].x; ph[i] = sv[i].y; })
    float2 Yr[E + 1];  // Y of the lane's bins k = lane + 64 i (+ bin L on lane 0)
    if constexpr (MODE == 5) {
        // sv is Y itself (k_fused MODE 4's X^2 / |X|): no phase propagation
        (void)mag; (void)ph;
        PV_FOR_BINS(E, lane, {
            float2 y = sv[i];
            if (k == 0 || k == L) y.y = 0.0f;  // C2R ignores Im of DC and Nyquist
            Yr[i] = y;
        })
    } else if constexpr (MODE != 1) {
        float phc[E + 1];
        float ekv[E + 1];
        unsigned jkv[E + 1];
        if constexpr (Q1) {
            (void)ekv; (void)jkv;
        } else if constexpr (KREG) {
            PV_FOR_BINS(E, lane, { ekv[i] = ekr[i]; jkv[i] = jkr[i]; })
        } else {
            PV_FOR_BINS(E, lane, { ekv[i] = lds_ld(&ekl[k]); jkv[i] = lds_ld(&jkl[k]); })
        }
        if constexpr (Q1) {
            PV_FOR_BINS(E, lane, { phc[i] = __builtin_fmaf(pm.rho_rev, ph[i], 0.0f); })
        } else if constexpr (RACC) {
            // -(p mod q) / q; +0 on a run's first frame (wave-uniform, one scalar select):
            // R <- fract(fma(mr, +0, R)) = fract(R) = R bit for bit, since R is in [0, 1) and
            // mr is finite (contract v4) — no per-bin select
            const float npq = add_decision ? -pm.p_over_q : 0.0f;
            const float tqf = (float)tq;
            PV_FOR_BINS(E, lane, {
                // m = -rint(dev); R <- fract(R - m p/q) = fract(R + rint(dev) p/q)
                const float mr = unwrap_round(ph[i], phprev[i], ekv[i]);
                float R = __int_as_float(M[i]);
                R = __builtin_amdgcn_fractf(__builtin_fmaf(mr, npq, R));
                M[i] = __float_as_int(R);
                phprev[i] = ph[i];
                const float tj = __builtin_amdgcn_fractf(tqf * __uint_as_float(jkv[i]));
                phc[i] = __builtin_fmaf(pm.rho_rev, ph[i], R + tj);
            })
        } else {
        PV_FOR_BINS(E, lane, {
            const int mm = unwrap_count(ph[i], phprev[i], ekv[i]);
            M[i] += add_decision ? mm : 0;
            phprev[i] = ph[i];
        })
        // output phase in revolutions: rho phi / 2 pi + ((p M_tot) mod q) / q,
        // M_tot = M_dec + (t+1) j_k.  q = 2^e: wrapping 32-bit arithmetic is exact mod q
        // (24-bit multiplies while q <= 2^24, the operands are < q); otherwise
        // q <= 32768 and nothing wraps.
        const unsigned qq = pm.q, pmod = pm.p_mod;
        if (QPOW2) {
            PV_FOR_BINS(E, lane, {
                const unsigned x = __umul24(pmod, (unsigned)M[i] & (qq - 1u)) + __umul24(tq, jkv[i]);
                phc[i] = __builtin_fmaf(pm.rho_rev, ph[i], (float)(x & (qq - 1u)) * pm.inv_q);
            })
        } else if (pm.q_pow2) {
            PV_FOR_BINS(E, lane, {
                const unsigned x = pmod * ((unsigned)M[i] & (qq - 1u)) + tq * jkv[i];
                phc[i] = __builtin_fmaf(pm.rho_rev, ph[i], (float)(x & (qq - 1u)) * pm.inv_q);
            })
        } else {
            PV_FOR_BINS(E, lane, {
                int mdq = M[i] % (int)qq;
                mdq += (mdq < 0) ? (int)qq : 0;
                const unsigned x = pmod * (unsigned)mdq + tq * jkv[i];
                phc[i] = __builtin_fmaf(pm.rho_rev, ph[i], (float)(x % qq) * pm.inv_q);
            })
        }
        }  // !RACC
        // (PV_ABL_*: diagnostic ablations for A/B timing only — wrong results)
#ifdef PV_ABL_NOGATHER
        if constexpr (false) {
#else
        if constexpr (MODE == 2 || MODE == 3) {
#endif
            float2 Y[E + 1];
            if constexpr (MODE == 3) {
                // at most one source per bin (pitch ratio >= 1): srcl holds each bin's source as a
                // byte offset into the tile, slot L + 1 (a zero written here every frame) when no
                // source maps there.  Every lane gathers every bin, bin L included (lanes != 0
                // read bin L's source too and ignore it: no exec-masked blocks), and no selects:
                // 4-byte map reads, one tile read and the sin/cos per bin.
                PV_FOR_BINS(E, lane, { if (i < E) tile[k] = make_float2(mag[i], phc[i]); })
                {
                    // bin L from lane 0, the zero slot from the others (one store, no branch)
                    const bool l0 = lane == 0;
                    tile[l0 ? L : L + 1] = make_float2(l0 ? mag[E] : 0.0f, l0 ? phc[E] : 0.0f);
                }
                wave_lds_sync();
                const unsigned* srco = reinterpret_cast<const unsigned*>(srcl);
                const char* tb = reinterpret_cast<const char*>(tile);
                constexpr int G = (L >= 1024) ? 4 : 1;
                constexpr int NGRP = (E + G) / G;
                auto offs_reads = [&](auto ig, unsigned (&o)[G]) {
                    static_for<0, G>([&](auto jj) {
                        constexpr int i = decltype(ig)::value * G + decltype(jj)::value;
                        if constexpr (i <= E) o[decltype(jj)::value] = lds_ld(&srco[(i == E) ? L : lane + 64 * i]);
                    });
                };
                // (L >= 1024: the next group's offsets are read while this group computes; at
                // L <= 512 the kernels sit at their VGPR budgets, one group at a time)
                unsigned on[G];
                if constexpr (L >= 1024) offs_reads(std::integral_constant<int, 0>{}, on);
                static_for<0, NGRP>([&](auto ig) {
                    constexpr int i0 = decltype(ig)::value * G;
                    unsigned o[G];
                    float2 f[G];
                    if constexpr (L >= 1024) {
#pragma unroll
                        for (int j = 0; j < G; ++j) o[j] = on[j];
                    } else {
                        offs_reads(ig, o);
                    }
                    static_for<0, G>([&](auto jj) {
                        constexpr int j = decltype(jj)::value;
                        if constexpr (i0 + j <= E) f[j] = lds_ld(reinterpret_cast<const float2*>(tb + o[j]));
                    });
                    if constexpr (L >= 1024 && decltype(ig)::value + 1 < NGRP)
                        offs_reads(std::integral_constant<int, decltype(ig)::value + 1>{}, on);
                    static_for<0, G>([&](auto jj) {
                        constexpr int j = decltype(jj)::value;
                        if constexpr (i0 + j <= E) {
                            float sn, cs;
                            sincos_rev(f[j].y, &sn, &cs);
                            Y[i0 + j] = make_float2(f[j].x * cs, f[j].x * sn);
                        }
                    });
                });
            } else {
                PV_FOR_BINS(E, lane, { tile[G_::pad(k)] = make_float2(mag[i], phc[i]); })
                wave_lds_sync();
                // {first source, count} in one 8-byte read; the first source's {mag, phase}
                // in one read, without a branch (zero when no source maps here); more sources
                // (ratios < 1) are summed in order like the oracle.  The ratio test is hoisted
                // out of the bin loop (wave-uniform): inside it the compiler merges it with the
                // per-lane count test into an exec-masked branch per bin (17 at L = 1024).
                // The LDS reads are issued in groups of G bins (all map reads, then all tile
                // reads, then the arithmetic): the volatile LDS loads keep program order, so bin
                // by bin every map read -> tile read pair would be two serialized LDS round trips
                // per bin (34 per frame at L = 1024).
                // (config 4 synthesis -2.5 %; 1 at L <= 512, whose kernels sit at their VGPR budget)
                // At L >= 1024 the groups are software-pipelined: group g + 1's map reads are
                // issued right after group g's tile reads, so they are in flight while group g
                // computes and one LDS round trip per group is exposed instead of two.
                constexpr int G = (L >= 1024) ? 4 : 1;
                constexpr int NGRP = (E + G) / G;
                auto map_reads = [&](auto ig, i2v (&sc)[G]) {
                    constexpr int i0 = decltype(ig)::value * G;
                    static_for<0, G>([&](auto jj) {
                        constexpr int j = decltype(jj)::value;
                        constexpr int i = i0 + j;
                        if constexpr (i <= E) {
                            const int k = (i == E) ? L : lane + 64 * i;
                            if (i < E || lane == 0) sc[j] = lds_ld2i(&srcl[2 * k]);
                        }
                    });
                };
                auto gather = [&](auto multi_tag) {
                    constexpr bool MULTI = decltype(multi_tag)::value;
                    i2v scn[G];  // the next group's map entries (in flight)
                    if constexpr (L >= 1024) map_reads(std::integral_constant<int, 0>{}, scn);
                    static_for<0, NGRP>([&](auto ig) {
                        constexpr int i0 = decltype(ig)::value * G;
                        i2v sc[G];
                        float2 f[G];
            #ifdef PV_LANE0_PRESEL
                if constexpr (true) {
#else
                if constexpr (L >= 1024) {
#endif
#pragma unroll
                            for (int j = 0; j < G; ++j) sc[j] = scn[j];
                        } else {
                            map_reads(ig, sc);
                        }
                        static_for<0, G>([&](auto jj) {
                            constexpr int j = decltype(jj)::value;
                            constexpr int i = i0 + j;
                            if constexpr (i <= E) {
                                const int sidx = sc[j].x;
                                if (i < E || lane == 0) f[j] = lds_ld(&tile[G_::pad(sidx >= 0 ? sidx : 0)]);
                            }
                        });
                        if constexpr (L >= 1024 && decltype(ig)::value + 1 < NGRP)
                            map_reads(std::integral_constant<int, decltype(ig)::value + 1>{}, scn);
                        static_for<0, G>([&](auto jj) {
                            constexpr int j = decltype(jj)::value;
                            constexpr int i = i0 + j;
                            if constexpr (i <= E) {
                                if (i < E || lane == 0) {
                                    const int sidx = sc[j].x;
                                    float ms = (sidx >= 0) ? f[j].x : 0.0f;
                                    const float pc = (sidx >= 0) ? f[j].y : 0.0f;
                                    if constexpr (MULTI)
                                        for (int qq = 1; qq < sc[j].y; ++qq) ms += tile[G_::pad(sidx + qq)].x;
                                    float sn, cs;
                                    sincos_rev(pc, &sn, &cs);
                                    Y[i] = make_float2(ms * cs, ms * sn);
                                }
                            }
                        });
                    });
                };
                if (pm.multi) {
                    gather(std::true_type{});
                } else {
                    gather(std::false_type{});
                }
            }  // MODE 2 (several sources per bin)
            wave_lds_sync();
            PV_FOR_BINS(E, lane, {
                float2 y = Y[i];
                if (k == 0 || k == L) y.y = 0.0f;  // C2R ignores Im of DC and Nyquist
                Yr[i] = y;
            })
        } else {
            PV_FOR_BINS(E, lane, {
                float sn, cs;
#ifdef PV_ABL_NOSINCOS
                sn = phc[i]; cs = 1.0f - phc[i];
#else
                sincos_rev(phc[i], &sn, &cs);
#endif
                float2 y = make_float2(mag[i] * cs, mag[i] * sn);
                if (k == 0 || k == L) y.y = 0.0f;
                Yr[i] = y;
            })
        }
    } else {
        PV_FOR_BINS(E, lane, {
            float sn, cs;
            sincos_rev(ph[i] * kInv2Pi, &sn, &cs);
            const float xr = mag[i] * cs;                 // kernel.cu:127
            float2 y = make_float2(xr, xr * sn);          // kernel.cu:128 (updated x)
            if (k == 0 || k == L) y.y = 0.0f;
            Yr[i] = y;
        })
    }
    hook();
    // inverse real-FFT pre-step: Z[i] = Fe + i Fo, pass-0 layout i = lane + 64 q, from
    // A = Y[i] (this lane's register q) and B = Y[L - i].  For lane l >= 1, bin L - i =
    // (64 - l) + 64 (E - 1 - q) is register E-1-q of lane 64 - l: a lane reversal by
    // ds_bpermute (crossbar only, no LDS memory traffic); lane 0's partners are its own
    // registers E - q (bin L - 64 q, q = 0 -> bin L).
    const int src_lane = ((64 - lane) & 63) << 2;
    float2 Bp[E];
#pragma unroll
    for (int q = 0; q < E; ++q) {
        const float2 o = Yr[E - 1 - q];
        Bp[q].x = __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane, __float_as_int(o.x)));
        Bp[q].y = __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane, __float_as_int(o.y)));
    }
    wave_lds_sync();  // the FFT's first tile store stays after the reads above (MODE 2, 3)
#pragma unroll
    for (int q = 0; q < E; ++q) {
        const float2 A = Yr[q];
        // lane 0: its own register E - q.  (A select, not lane0_mov2: here the exec-masked
        // moves measured ~1 % slower, profiles/r04_ab_lane0.txt — they must wait for the
        // permute before the moves, the select can sit at the use.)
        const float2 Bc = (lane == 0) ? Yr[E - q] : Bp[q];
        float2 tw;  // e^{-2 pi i k/N}, k = lane + 64 q
        if constexpr (TwS::ON) tw = twr.v[q];
        else tw = lds_ld(&twsl[lane + 64 * q]);
        // packed pre-step, same roundings as the scalar form fer - Foi, fei + For with
        // For = fma(dr, tw.x, di tw.y), Foi = fma(di, tw.x, -(dr tw.y)).
        // V = (dr, di) = (A.x - B.x, A.y + B.y), W = (fer, fei) = (A.x + B.x, A.y - B.y):
        // one v_pk_add each, the sign flips by neg_lo / neg_hi;
        // R = (di tw.y, -(dr tw.y)); Q = (For, Foi) = V tw.x + R; z = (fer - Foi, fei + For)
        const f2v a = f2v{A.x, A.y}, b = f2v{Bc.x, Bc.y}, w = f2v{tw.x, tw.y};
        f2v V, W, R, Q, Z;
        asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(V) : "v"(a), "v"(b));
        asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(W) : "v"(a), "v"(b));
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1] neg_hi:[1,0]" : "=v"(R) : "v"(V), "v"(w));
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(Q) : "v"(V), "v"(w), "v"(R));
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(Z) : "v"(W), "v"(Q));
        z[q] = make_float2(Z.x, Z.y);
    }
    wave_lds_sync();
#ifndef PV_ABL_NOFFT
    fft_run<L, true, STORE_LAST, 0, 0, V3X>(z, tile, twl, tw0, lane);
#endif
}

}  // namespace pv
