// pv_syn_run.hpp — one wave's synthesis run (phase propagation -> polar->rect -> inverse
// real FFT -> window -> overlap-add -> final samples to `out`) of the split path's K3
// (k_synthesis, pv_kernels.hip), and the in-launch seam hand-off of the single-launch q = 1
// path (pv_fused.hip).  Geometry and overlap-add: pv_kernels.hip, K3.
#pragma once
#include "pv_frame.hpp"
#include "pv_kernels.h"

namespace pv {

// Register-resident synthesis gains (the register overlap-add kernels, L <= 512, and L = 1024
// with out hop 512: config 4, 252 VGPRs, free below the 2 waves/SIMD its LDS sets; smaller
// out hops would need AGPRs).
template <int L, int DT>
constexpr bool syn_gains_in_regs() { return DT > 0 && (L <= 512 || (L == 1024 && DT == 4)); }

// sc1 (write-through) stores / loads of the inter-workgroup hand-offs (pv_fused.hip;
// MI355X_MICROARCH.md "Valid forms")
__device__ __forceinline__ void st_sc1(float* p, float v) {
    asm volatile("global_store_dword %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1(float* p, f2v v) {
    asm volatile("global_store_dwordx2 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float ld_sc1(const float* p) {
    float v;
    asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// counter add after every store of the wave has left (relaxed: the sc1 stores need no fence)
__device__ __forceinline__ int arrive(int* flag, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __shfl(old, 0);
}

// K write-through 8-byte loads of a lane's positions base + 128 m (m < K), all in flight at
// once; the caller's sc1_wait makes them (and everything else outstanding) land
template <int K>
__device__ __forceinline__ void ld_sc1_issue(f2v (&v)[K], const float* base) {
#pragma unroll
    for (int m = 0; m < K; ++m) {
        const float* pm = base + 1024 * (m >> 3);  // 13-bit signed immediate offsets
        asm volatile("global_load_dwordx2 %0, %1, off offset:%2 sc1" : "=v"(v[m]) : "v"(pm), "n"(512 * (m & 7)) : "memory");
    }
}
template <int K>
__device__ __forceinline__ void sc1_wait(f2v (&v)[K]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int m = 0; m < K; ++m) asm volatile("" : "+v"(v[m]));  // uses stay after the wait
}

// After a register overlap-add run (wave w of a workgroup of 4 consecutive runs, workgroup
// index wg of nwg along the channel): the run's tail -> ring (LDS, over the tiles), the three
// intra-workgroup seams from the neighbours' tails, and the inter-workgroup seams in the
// same launch.  Seam b (workgroup b-1's last tail overlaps workgroup b's head, which wave 0
// of workgroup b stored write-through as if final) is closed by whichever side arrives
// second: each side publishes its part write-through (the tail to `tails`, the head to
// `out`), waits for its stores and adds 1 to the seam's counter; the side whose add returns
// 1 reads the other part (sc1 loads), writes head + tail and resets the counter for the next
// launch.  Nobody waits for anybody, so there is no dispatch-order assumption; head + tail
// is the same float whoever adds it.  Every wave of the workgroup must call this.
//
// The overlap (TL = N - out hop) is TM = TL / 128 float2 per lane at positions 2 lane + 128 m:
// every read-back of a seam is issued as one batch and waited for once (per element, a load
// and its wait were 12 serialized round trips; config 2 stamps, scripts/fused_stamps.py: the
// seams were 5.8 us of a 27.6 us wave, 11.3 us on wave 3).  Unaligned `out` takes the
// per-sample path.
template <int L, int NS, int D>
__device__ __forceinline__ void close_seams_inline(const float2 (&acc)[NS], float2* tiles, int w, int lane, int c,
                                                   int wg, int nwg, long long obase, int F, int hs, float* outc,
                                                   long long out_len, bool out_aligned, float* tails, int tail_len,
                                                   int* seam_flags) {
    constexpr int N = 2 * L;
    constexpr int TL = N - 128 * D;  // = N - hs
    constexpr int TM = TL / 128;
    static_assert(TL % 128 == 0 && TM >= 1 && TM <= 16, "overlap in whole 128-sample blocks");
    __syncthreads();
    float* rings = reinterpret_cast<float*>(tiles);
    float* ring = rings + w * N;
    {
        float2* r2 = reinterpret_cast<float2*>(ring);
#pragma unroll
        for (int s = 0; s < NS - D; ++s) r2[64 * s + lane] = acc[s];
    }
    __syncthreads();
    const bool last = (wg + 1 >= nwg);
    const long long nbase = obase + (long long)F * hs;  // workgroup wg+1's first position
    if (!out_aligned) {
        // seams: run w's tail overlaps run w+1's head
        if (w > 0) {
            const float* prev = rings + (w - 1) * N;
            for (int j = lane; j < TL; j += 64) {
                const long long gp = obase + j;
                if (gp < out_len) outc[gp] += prev[j];
            }
        }
        if (w == 3) {
            float* tdst = tails + ((long long)c * nwg + wg) * tail_len;
            for (int j = lane; j < TL; j += 64) {
                const float v = ring[j];
                if (last) {
                    const long long gp = nbase + j;
                    if (gp < out_len) outc[gp] = v;
                } else {
                    st_sc1(tdst + j, v);
                }
            }
            if (!last) {
                int* flag = seam_flags + (long long)c * nwg + wg;
                if (arrive(flag, lane) == 1) {  // workgroup wg+1's head is in out
                    for (int j = lane; j < TL; j += 64) {
                        const long long gp = nbase + j;
                        if (gp < out_len) outc[gp] = ld_sc1(outc + gp) + ring[j];
                    }
                    if (lane == 0) __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        if (w == 0 && wg > 0) {
            int* flag = seam_flags + (long long)c * nwg + (wg - 1);
            if (arrive(flag, lane) == 1) {  // workgroup wg-1's tail is in tails
                const float* tsrc = tails + ((long long)c * nwg + (wg - 1)) * tail_len;
                for (int j = lane; j < TL; j += 64) {
                    const long long gp = obase + j;
                    if (gp < out_len) outc[gp] = ld_sc1(outc + gp) + ld_sc1(tsrc + j);
                }
                if (lane == 0) __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    // 8-byte path: positions are even and out_len is even (frames * hs + N - hs), so a pair
    // is either wholly inside out or wholly past it
    const float2* own2 = reinterpret_cast<const float2*>(ring) + lane;
    // (1) w > 0: this run's head (stored in the frame loop) back, all loads in flight
    f2v head[TM];
    if (w > 0) {
#pragma unroll
        for (int m = 0; m < TM; ++m) {
            const long long gp = obase + 2 * lane + 128 * m;
            head[m] = (gp < out_len) ? *reinterpret_cast<const f2v*>(outc + gp) : f2v{0.0f, 0.0f};
        }
    }
    // (2) w = 3: the workgroup's last tail — final samples if this is the channel's last
    // workgroup, else published write-through for seam wg + 1, then arrive
    bool second = false;
    if (w == 3) {
        if (last) {
#pragma unroll
            for (int m = 0; m < TM; ++m) {
                const long long gp = nbase + 2 * lane + 128 * m;
                const float2 v = own2[64 * m];
                if (gp < out_len) __builtin_nontemporal_store(f2v{v.x, v.y}, reinterpret_cast<f2v*>(outc + gp));
            }
        } else {
            float* tdst = tails + ((long long)c * nwg + wg) * tail_len + 2 * lane;
#pragma unroll
            for (int m = 0; m < TM; ++m) {
                const float2 v = own2[64 * m];
                st_sc1(tdst + 128 * m, f2v{v.x, v.y});
            }
            second = arrive(seam_flags + (long long)c * nwg + wg, lane) == 1;
        }
    }
    // (3) intra-workgroup seam: head + run w-1's tail
    if (w > 0) {
        const float2* prev2 = reinterpret_cast<const float2*>(rings + (w - 1) * N) + lane;
#pragma unroll
        for (int m = 0; m < TM; ++m) {
            const long long gp = obase + 2 * lane + 128 * m;
            const float2 t = prev2[64 * m];
            if (gp < out_len)
                __builtin_nontemporal_store(f2v{head[m].x + t.x, head[m].y + t.y}, reinterpret_cast<f2v*>(outc + gp));
        }
    }
    // (4) w = 3, second at seam wg + 1: workgroup wg+1's head is in out (inside out: that
    // workgroup has frames)
    if (second) {
        f2v hd[TM];
        ld_sc1_issue<TM>(hd, outc + nbase + 2 * lane);
        sc1_wait<TM>(hd);
#pragma unroll
        for (int m = 0; m < TM; ++m) {
            const float2 v = own2[64 * m];
            __builtin_nontemporal_store(f2v{hd[m].x + v.x, hd[m].y + v.y},
                                        reinterpret_cast<f2v*>(outc + nbase + 2 * lane + 128 * m));
        }
        if (lane == 0) __hip_atomic_store(seam_flags + (long long)c * nwg + wg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // (5) w = 0 of workgroup wg > 0: arrive at seam wg; second: its head (inside out: wave 0
    // has frames) + workgroup wg-1's tail
    if (w == 0 && wg > 0) {
        int* flag = seam_flags + (long long)c * nwg + (wg - 1);
        if (arrive(flag, lane) == 1) {
            f2v hd[TM], tl[TM];
            ld_sc1_issue<TM>(hd, outc + obase + 2 * lane);
            ld_sc1_issue<TM>(tl, tails + ((long long)c * nwg + (wg - 1)) * tail_len + 2 * lane);
            sc1_wait<TM>(hd);
            sc1_wait<TM>(tl);
#pragma unroll
            for (int m = 0; m < TM; ++m)
                __builtin_nontemporal_store(f2v{hd[m].x + tl[m].x, hd[m].y + tl[m].y},
                                            reinterpret_cast<f2v*>(outc + obase + 2 * lane + 128 * m));
            if (lane == 0) __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// LDS carve-up pointers of the synthesis (the kernels lay them out differently)
struct SynCarve {
    const float2* twl;   // stage-major twiddles, L-point
    const float2* twsl;  // e^{-2 pi i k/N}, k <= L
    float2* tiles;       // 4 x TILE
    float* rings;        // DT = 0: 4 x N overlap-add rings (live through the loop)
    const float* gainl;  // N gains (unless GREG)
    const float* ekl;    // e_k
    const unsigned* jkl; // (p j_k) mod q, or its float / q (RACC)
    const int* srcl;     // pitch map {first, count}
};

template <int L, int MODE, int DT, bool QPOW2>
struct SynTraits {
    static constexpr bool ROLA = DT > 0;
    static constexpr int E = Geo<L>::E;
    static constexpr int NS = ROLA ? E : 1;  // register overlap-add slots
    static constexpr int D = ROLA ? DT : 1;  // slots completed per frame (ROLA)
    static constexpr bool GREG = syn_gains_in_regs<L, DT>();
    // revolution accumulator (synth_frame RACC; measured: synthesis -2.5 %); the host takes
    // the QPOW2 kernels only for q <= 4096
    static constexpr bool RACC = QPOW2 && MODE != 1;
};

// The frame loop of one wave's run: frames t0 .. t0 + F - 1 of channel c (frames >= nfr are
// zero), unwrap state M / phprev initialised by the caller (M = the carry at t0, in the RACC
// form when RACC).  On return acc holds the run's overlap tail (ROLA; slots D..NS-1) or
// the ring does (DT = 0).
// LANEK: the unwrap constants are per-lane (e_k and (p j_k) mod q depend on k mod 64 only:
// 64 a multiple of the hop divisor and q of 64 / hop divisor, checked by the host —
// config 3 and 4): two registers (and bin L's j constant) instead of two LDS reads per bin
// and frame.
// NR: row slots read per frame (lane registers i < NR, bins < 64 NR): every slot, or for a
// pitch ratio > 1 only those some output bin takes its source from (src_hi) — the other slots
// are never gathered, and without a spectrum output the analysis does not write them
// (k_std_analysis NA): they stay zero in the registers, no load, no stale bytes read.
template <int L, int MODE, int DT, bool QPOW2, bool LANEK = false, int NR = Geo<L>::E>
__device__ __forceinline__ void syn_run(const SynParams& p, const SynCarve& sc, const float2 (&tw0)[Geo<L>::E],
                                        int lane, int w, int c, int t0, int nfr,
                                        int (&M)[Geo<L>::E + 1], float (&phprev)[Geo<L>::E + 1],
                                        float2 (&acc)[SynTraits<L, MODE, DT, QPOW2>::NS]) {
    using G_ = Geo<L>;
    using T_ = SynTraits<L, MODE, DT, QPOW2>;
    constexpr bool ROLA = T_::ROLA;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr int SPW = N / 64;  // samples per lane per frame
    constexpr int NS = T_::NS;
    constexpr int D = T_::D;
    constexpr bool GREG = T_::GREG;
    constexpr bool RACC = T_::RACC;
    const int hs = p.hs;
    const int TL = N - hs;
    (void)TL;
    float2* tile = sc.tiles + w * G_::TILE;
    float* ring = sc.rings + w * N;
    const float* gainl = sc.gainl;
    (void)gainl; (void)ring;
    const float2* specc = p.spec + (long long)c * p.ld_spec;
    float* outc = p.out + (long long)c * p.ldo;
    const long long obase = (long long)t0 * hs;

    float2 gn[GREG ? NS : 1];
    if (ROLA) {
        const float2* g2 = reinterpret_cast<const float2*>(p.gain);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            acc[s] = make_float2(0.0f, 0.0f);
            if constexpr (GREG) gn[s] = g2[64 * s + lane];
        }
    }

    // unwrap constants of the lane's bins in registers for the whole run (per-lane kernels)
    constexpr bool KREG = LANEK && MODE != 1;
    float ekr[E + 1];
    unsigned jkr[E + 1];
    if constexpr (LANEK && MODE != 1) {
        const float e_lane = lds_ld(&sc.ekl[lane]);
        const unsigned j_lane = lds_ld(&sc.jkl[lane]);
        const unsigned j_last = lds_ld(&sc.jkl[L]);  // bin L (lane 0)
#pragma unroll
        for (int i = 0; i <= E; ++i) {
            ekr[i] = e_lane;  // e_L = e_0: lane 0 is the only one that uses bin L
            jkr[i] = (i == E) ? j_last : j_lane;
        }
    } else if constexpr (KREG) {
        PV_FOR_BINS(E, lane, { ekr[i] = lds_ld(&sc.ekl[k]); jkr[i] = lds_ld(&sc.jkl[k]); })
    }
    const PhaseMap pmap{p.rho * kInv2Pi, (unsigned)p.q, (unsigned)p.p_mod, p.q_pow2, p.inv_q,
                        (float)p.p_mod * p.inv_q, p.rho < 1.0f ? 1 : 0};
    const SynLds stb{sc.twl, sc.twsl, sc.ekl, sc.jkl, sc.srcl};
    // the pre-step's split twiddles of the lane's bins in registers for the run: L = 1024
    // (2 waves per SIMD are set by LDS, so VGPRs up to 256 cost no occupancy) and the L = 512
    // per-lane kernels (within their 3 waves/SIMD budget)
    // (not the L = 512 pitch kernel with out hop 128: with the contract-v3 FFT it would spill)
    using TwS = typename std::conditional<((L == 1024 || (L == 512 && LANEK && !(MODE >= 2 && DT == 1))) && ROLA),
                                          TwReg<E>, NoTwReg>::type;
    TwS twr;
    if constexpr (TwS::ON) {
#pragma unroll
        for (int q = 0; q < E; ++q) twr.v[q] = lds_ld(&sc.twsl[lane + 64 * q]);
    }
    const unsigned q32 = (unsigned)p.q;  // <= 2^24 (QPOW2) or <= 32768
    auto synth = [&](int u, int t, const float2 (&sv)[E + 1], float2 (&z)[E], const auto& hk) {
        // (t_off: a segment's first frame index in its whole stream, mod q)
        const unsigned tq = QPOW2 ? ((unsigned)(t + 1) + p.t_off) & (q32 - 1u) : ((unsigned)(t + 1) + p.t_off) % q32;
        using H = std::decay_t<decltype(hk)>;
        // (L = 1024: the radix-16/16/4 inverse FFT on the v3 pass table, p.tw)
        synth_frame<L, MODE, !ROLA, QPOW2, KREG, RACC, false, H, TwS, (L == 1024)>(
            sv, u > 0, tq, M, phprev, pmap, stb, tw0, tile, lane, z, ekr, jkr, hk, twr);
    };
    // PV_SPEC_PACKED rows: lane 0 finds bins 0 and L in slot 0 (the row has no slot L)
    const bool packed = p.packed != 0;
    auto unpack = [&](float2 (&sv)[E + 1]) {
        if (packed && lane == 0) unpack_real_bins(sv[0], sv[0], sv[E]);
    };
    // ROLA: register z[idx] = samples 2 (lane + 64 cr) + {0,1}; REF_COMPAT's half swap
    // moves raw slot cr to OLA slot cr + E/2 (mod E)
    auto ola_regs = [&](const float2 (&z)[E]) {
#pragma unroll
        for (int idx = 0; idx < E; ++idx) {
            const int cr = last_slot<L>(idx);
            const int cs = (MODE == 1) ? ((cr + E / 2) & (E - 1)) : cr;
            const float2 g = GREG ? gn[GREG ? cs : 0]
                                  : lds_ld(reinterpret_cast<const float2*>(gainl) + 64 * cs + lane);
            acc[cs].x = __builtin_fmaf(z[idx].x, g.x, acc[cs].x);
            acc[cs].y = __builtin_fmaf(z[idx].y, g.y, acc[cs].y);
        }
    };
    // ROLA flush of frame u: positions [u*hs, (u+1)*hs) = slots 0..D-1 are final
    auto flush_regs = [&](int u, auto fast_tag) {
        constexpr bool FAST = decltype(fast_tag)::value;
        const long long pb = obase + (long long)u * hs + 2 * lane;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const long long gp = pb + 128 * d;
            if (FAST || (p.out_aligned && gp + 1 < p.out_len)) {
                // non-temporal output stores: -0.5 %
                __builtin_nontemporal_store(f2v{acc[d].x, acc[d].y}, reinterpret_cast<f2v*>(outc + gp));
            } else {
                if (gp < p.out_len) outc[gp] = acc[d].x;
                if (gp + 1 < p.out_len) outc[gp + 1] = acc[d].y;
            }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) acc[s] = (s + D < NS) ? acc[(s + D < NS) ? s + D : 0] : make_float2(0.0f, 0.0f);
    };

    // the self-tracked prefetch needs registers that are never spilled or copied while the
    // loads are in flight: only at L = 512, where the kernels fit without spills and no
    // register copy sits between a row load and its vmcnt (scripts/prefetch_hazards.py,
    // tests/test_abi.py; at L <= 256 the compiler copies the row buffers)
    constexpr bool FASTOK = ROLA && L == 512;
    const bool fast = FASTOK && nfr == p.F && p.out_aligned && obase + (long long)p.F * hs <= p.out_len;
    if (FASTOK && fast) {
        // every store of the run is in bounds: trip u = [load row u+1] [frame u] [D stores]
        // [vmcnt(D): row u+1 landed, the stores may still be in flight].  Two row buffers
        // alternate (F is even), so no register copies carry a row across trips.
#ifdef PV_ABL_L2ROWS
        // (timing only: every frame re-reads the run's first row, an L2 hit)
        auto rowp = [&](int u) { (void)u; return specc + (long long)t0 * p.spec_stride; };
#else
        auto rowp = [&](int u) { return specc + (long long)(t0 + min(u, p.F - 1)) * p.spec_stride; };
#endif
        auto step = [&](int u, const f2v (&row)[E + 1]) {
            float2 sv[E + 1];
#pragma unroll
            for (int i = 0; i <= E; ++i) sv[i] = make_float2(row[i].x, row[i].y);
            unpack(sv);
            float2 z[E];
            synth(u, t0 + u, sv, z, NoHook{});
            ola_regs(z);
            flush_regs(u, std::true_type{});  // exactly D stores
        };
        // (packed rows: no bin-L load; vmcnt(D) still waits for every row load)
        f2v ra[E + 1], rb[E + 1];
        gload_row<E>(ra, rowp(0) + lane, rowp(0) + L, !packed);
        vm_wait<0>(ra);
        for (int u = 0; u < p.F; u += 2) {
            gload_row<E>(rb, rowp(u + 1) + lane, rowp(u + 1) + L, !packed);
            step(u, ra);
            vm_wait<D>(rb);
            gload_row<E>(ra, rowp(u + 2) + lane, rowp(u + 2) + L, !packed);
            step(u + 1, rb);
            vm_wait<D>(ra);
        }
    } else {
        // L >= 1024 (ROLA): the next row's loads are issued once the frame has consumed the
        // current row (synth_frame's hook, before the pre-step), into the same registers —
        // no copy of the row (34 VGPR moves per frame); the loads have the inverse FFT and
        // the overlap-add to land
        constexpr bool LATE = ROLA && L >= 1024 && MODE != 2;  // (MODE 2: 260 VGPRs, 1 wave/SIMD)
        const bool fast_st = ROLA && p.out_aligned && obase + (long long)p.F * hs <= p.out_len;
        (void)fast_st;
        static_assert(NR == E || (MODE == 3 && NR < E), "partial rows: single-source pitch only");
        float2 sv[E + 1];  // spectrum row of the next frame, loaded one frame ahead
#pragma unroll
        for (int i = NR; i < E; ++i) sv[i] = make_float2(0.0f, 0.0f);
        if (NR < E) sv[E] = make_float2(0.0f, 0.0f);
        auto load_row = [&](const float2* srow) {
            PV_FOR_BINS(E, lane, {
                if (i < NR || (i == E && NR == E && !packed)) sv[i] = srow[k];
            })
        };
        if (nfr > 0) load_row(specc + (long long)t0 * p.spec_stride);
        for (int u = 0; u < p.F; ++u) {
            const int t = t0 + u;
            if (u < nfr) {
                float2 z[E];
                if constexpr (LATE) {
                    unpack(sv);
                    // (unconditional: the run's last frame re-reads its own row, so the
                    // registers take no merge of loaded and kept values)
                    const int tn = (u + 1 < nfr) ? t + 1 : t;
                    synth(u, t, sv, z, [&]() { load_row(specc + (long long)tn * p.spec_stride); });
                } else {
                float2 cur[E + 1];
#pragma unroll
                for (int i = 0; i <= E; ++i) cur[i] = sv[i];
                unpack(cur);  // at use: unpacking at the load would wait for it at once
                if (u + 1 < nfr) load_row(specc + (long long)(t + 1) * p.spec_stride);
                synth(u, t, cur, z, NoHook{});
                }
                if constexpr (ROLA) {
                    ola_regs(z);
                    // the next row has had the whole frame to land: wait for it here, before
                    // the frame's output stores, so the compiler's wait for the row's
                    // registers at the loop edge does not also wait for those stores
                    __builtin_amdgcn_s_waitcnt(kVmcnt0);
                } else {
                    // overlap-add the frame into the ring (lane-distinct positions)
                    // y[nn], nn = (n + ROT) mod N, n = lane + 64 i: float index
                    // 2 pad(nn >> 1) + (nn & 1) = per-lane base + compile-time offset
                    constexpr int ROT = (MODE == 1) ? N / 2 : 0;
                    const float* ty = reinterpret_cast<const float*>(tile) + 2 * G_::pad(lane >> 1) + (lane & 1);
                    const int rbase = u * hs + lane;
#pragma unroll
                    for (int i = 0; i < SPW; ++i) {
                        const int n = lane + 64 * i;
                        const int cc = ((64 * i + ROT) & (N - 1)) >> 1;
                        const float yv = ty[2 * G_::padc(cc)];
                        const int pos = (rbase + 64 * i) & (N - 1);
                        ring[pos] = __builtin_fmaf(yv, gainl[n], ring[pos]);
                    }
                    wave_lds_sync();
                }
            }
            if constexpr (ROLA) {
                // a run whose stores are all in bounds takes the unconditional stores
                // (wave-uniform test): per-lane bounds-checked stores sit in exec-masked
                // blocks, after which the compiler waits for every store of the frame
                // (vmcnt(0)) before the next row's registers may be moved
                if (fast_st) flush_regs(u, std::true_type{});
                else flush_regs(u, std::false_type{});
            } else {
                // positions [u*hs, (u+1)*hs) are final for this run
                for (int j = lane; j < hs; j += 64) {
                    const int pl = u * hs + j;
                    const int slot = pl & (N - 1);
                    const float v = ring[slot];
                    ring[slot] = 0.0f;
                    if (obase + pl < p.out_len) outc[obase + pl] = v;
                }
                wave_lds_sync();
            }
        }
    }
}

}  // namespace pv
