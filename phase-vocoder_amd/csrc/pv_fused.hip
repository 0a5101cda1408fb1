// pv_fused.hip — analysis -> processing -> resynthesis in ONE launch, for STANDARD
// configurations whose output phase does not depend on the unwrap count (q = 1: an integer
// ratio, e.g. BASELINE config 2, pitch 2.0).
//
// Why only q = 1: the output phase is rho phi + 2 pi ((p M) mod q) / q,
// and M, the running unwrap count, needs every earlier frame of the channel — the split
// path's analysis -> k_carry scan -> synthesis.  With q = 1 the last term is 0, so frame t's
// output depends on frame t's spectrum alone: a wave can analyse a frame, keep its
// {mag, phase} row in registers, resynthesise it at once and overlap-add it, with no halo
// frame, no run records and no second pass over the spectrum.  The spectrum row is still
// stored (the caller's spectrum buffer is an output of pv_process), but it is
// never read back: per frame 4 hop_a + 8 (N/2+1) + 4 hop_s bytes instead of the split
// path's 4 hop_a + 16 (N/2+1) + 4 hop_s, and one launch instead of two (with spec = NULL
// the rows are not stored at all).  Config 2, a single stream, runs as exactly 3 workgroups
// per CU (balanced runs, below), bound by the shared issue of the 3 waves per SIMD, not by
// bytes (per-wave stamps).
//
// The per-frame arithmetic is k_std_analysis's (window, FFT, split, atan2, sqrt) and
// k_synthesis's (synth_frame, register overlap-add, tails, seams) operation for operation,
// so the spectrum and the output are bit-identical to the split path (tests/test_gpu_fused.py)
// — except MODE 4, whose output is the same sum rounded differently (within 1e-6).
// MODE 4 (pitch exactly 2, L >= 256): output bin k' = 2 s takes source bin s and the odd
// output bins are empty, so the output frame is periodic with period N/2 — it is resynthesised
// by an N/2-point inverse real FFT of bins 0 .. L/2 (the analysis registers 0 .. E/2, bin L/2
// on lane 0 of register E/2, exactly the half-size transform's layout) and repeated: half the
// inverse FFT and pre-step work, no gather; and since q = 1 makes the output phase exactly
// 2 phi, its input Y_s = |X_s| e^{2 i phi_s} = X_s^2 / |X_s| comes from the split's X without
// atan2 or sin/cos (the contract phases are computed only for a spectrum output).  Results
// within rounding of MODE 3.
// Geometry as k_synthesis: a wave = a run of F frames of one channel, 4 runs per workgroup,
// the intra-workgroup seams closed after one barrier, the inter-workgroup seams by the
// second of the two workgroups to finish (no k_seam launch).
#include "pv_syn_run.hpp"

namespace pv {

// Inter-workgroup hand-offs: st_sc1 / ld_sc1 / arrive / close_seams_inline (pv_syn_run.hpp),
// write-through `sc1` stores of every handed-off byte, the storing wave's vmcnt(0) before its
// counter add, `sc1` loads of them after the add has returned (MI355X_MICROARCH.md "Valid
// forms"): an agent-scope release/acquire pair would write back / invalidate whole caches
// (buffer_wbl2 / buffer_inv) per workgroup.

template <int L>
struct FuGeo {
    static constexpr int N = 2 * L;
    static constexpr int B = L + 1;
    // float offsets
    static constexpr int O_TW = 0;                            // L float2
    static constexpr int O_TWS = O_TW + 2 * L;                // L+1 float2 (+1 pad)
    static constexpr int O_TILE = O_TWS + 2 * (L + 2);        // 4 x TILE float2
    static constexpr int O_WIN = O_TILE + 2 * 4 * Geo<L>::TILE;  // N
    static constexpr int O_SRC = O_WIN + N;                   // 2B (+2) {first, count}
    static constexpr int FLOATS = O_SRC + 2 * B + 2;
    static constexpr size_t BYTES = sizeof(float) * FLOATS;
    static_assert(O_SRC % 2 == 0 && O_TILE % 4 == 0, "alignment of the LDS carve-up");
};

template <int L, int MODE, int DT>
// waves per SIMD k_fused is compiled for: 3 (<= 168 VGPRs; the balanced config-2 launch
// holds exactly 3 workgroups per CU) — at 4 (<= 128) the L = 512 kernels spilled 6-12 VGPRs
// to scratch; round 5 A/B: config 2 30.9 -> 30.1 us, and with the register split 29.6
#ifndef PV_FUSED_WAVES
#define PV_FUSED_WAVES 3
#endif
// 0: analyse every bin even without a spectrum output (A/B of the skip; same results)
// 1: the real split straight from the FFT's last-pass registers (split_chunk_bp, as
// k_std_analysis) instead of from a final image in LDS (0: the LDS-image split, A/B only)
#ifndef PV_FUSED_BPSPLIT
#define PV_FUSED_BPSPLIT 1
#endif
#ifndef PV_FUSED_SKIP_UNREAD
#define PV_FUSED_SKIP_UNREAD 1
#endif
// 0: every frame's samples loaded whole (A/B of the shifted-register input; same results)
#ifndef PV_FUSED_SHIFT
#define PV_FUSED_SHIFT 1
#endif
__global__ __launch_bounds__(256, PV_FUSED_WAVES) void k_fused(FusedParams p) {
    using G_ = Geo<L>;
    using FG = FuGeo<L>;
    constexpr int E = G_::E;
    constexpr int N = FG::N;
    constexpr int B = FG::B;
    constexpr int NS = E;  // overlap-add slots: positions u*hs + 128 s + 2 lane + {0,1}
    constexpr int D = DT;  // slots completed per frame (out hop = 128 DT)
    static_assert(DT == 1 || DT == 2 || DT == 4, "register overlap-add");
    extern __shared__ __attribute__((aligned(16))) float fsm[];
    float2* twl = reinterpret_cast<float2*>(fsm + FG::O_TW);
    float2* twsl = reinterpret_cast<float2*>(fsm + FG::O_TWS);
    float2* tiles = reinterpret_cast<float2*>(fsm + FG::O_TILE);
    float* winl = fsm + FG::O_WIN;
    int* srcl = reinterpret_cast<int*>(fsm + FG::O_SRC);
    // MODE 4: the half-size transform's stage-major twiddles (L/2) and split twiddles
    // e^{-2 pi i k/(N/2)}, k <= L/2, in the pitch map's area (2L + 2 <= 2B + 2 floats)
    static_assert(MODE != 4 || L >= 256, "half-size synthesis: L/2 >= 128");
    constexpr int LH = (MODE == 4) ? L / 2 : L;
    float2* twl_h = reinterpret_cast<float2*>(fsm + FG::O_SRC);
    float2* twsl_h = twl_h + LH;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
#ifdef PV_FUSED_STAMPS
    // diagnostic build (scripts/fused_stamps.py): s_memrealtime (100 MHz) at the phase
    // boundaries of every wave, written by lane 0 with vector stores
    unsigned long long* stp =
        p.stamps + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 + w) * kFusedStampSlots;
    const unsigned long long st_rt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long st_mt0 = __builtin_amdgcn_s_memtime();
    auto stamp = [&](int slot, unsigned long long v) {
        if (lane == 0 && slot < kFusedStampSlots) stp[slot] = v;
    };
#define PV_STAMP(slot_) stamp((slot_), __builtin_amdgcn_s_memrealtime())
#else
#define PV_STAMP(slot_) ((void)0)
#endif
    const int c = blockIdx.y;
    // this wave's run: F frames, or (balanced, p.n4 > 0) F or F + 1.  Balanced: the launch is
    // exactly `rounds` workgroups per CU (no CU holds one more than the others) and the n4
    // long runs are spread over the workgroups (floor((k+1) n4 / nwg) - floor(k n4 / nwg) =
    // 1 or 2 per workgroup) at wave positions rotated by the workgroup's dispatch round
    // (linear id / 256): the workgroups a CU holds — k, k + 256, k + 512 with the
    // dispatcher's round-robin over XCDs and CUs — put theirs on different SIMDs, so a SIMD
    // runs at most 2 long runs (3 waves: 11 frames instead of 4 waves: 12).  Any other
    // placement is still correct, only less balanced.
    int t0, fw;
    if (p.n4 > 0) {
        const int k = blockIdx.x;
        const long long a = (long long)k * p.n4 / p.nwg, b = (long long)(k + 1) * p.n4 / p.nwg;
        const int m = (int)(b - a);
        // (the rotation follows blockIdx.x alone, so a channel's runs — and its output bits —
        // do not depend on its position in the batch; for one channel it is the dispatch round)
        const int r = (int)(blockIdx.x >> 8) & 3;
        int pre = 0;
        for (int v = 0; v < w; ++v) pre += p.F + ((((v - r) & 3) < m) ? 1 : 0);
        t0 = 4 * p.F * k + (int)a + pre;
        fw = p.F + ((((w - r) & 3) < m) ? 1 : 0);
    } else {
        t0 = (blockIdx.x * 4 + w) * p.F;
        fw = p.F;
    }
    const int nfr = max(0, min(fw, p.frames - t0));  // real frames of this wave's run
    const int hs = p.hs;
    const int TL = N - hs;
    float2* tile = tiles + w * G_::TILE;
    const float* xc = p.x + (long long)c * p.ldx;
    // spec == nullptr (pv_process without a spectrum buffer): the rows stay in registers
    // only — SURVEY §8(d)'s fused mode, whose bytes are the input and the output
    const bool wspec = p.spec != nullptr;
    float2* specc = wspec ? p.spec + (long long)c * p.ld_spec : nullptr;
    float* outc = p.out + (long long)c * p.ldo;
    const long long obase = (long long)t0 * hs;

    // synth_frame's unwrap state and tables are not used with Q1
    int M[E + 1];
    float phprev[E + 1];
    float ekr[E + 1];
    unsigned jkr[E + 1];
    const PhaseMap pmap{p.rho * kInv2Pi, 1u, 0u, 1, 1.0f, 0.0f, p.rho < 1.0f ? 1 : 0};
    const SynLds stb{twl, twsl, nullptr, nullptr, srcl};

    float2 acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = make_float2(0.0f, 0.0f);

    // input frame t: samples t*hop + 2 (lane + 64 q) + {0,1}; frames whose N samples are all
    // inside [0, n) use vector loads, the last N/hop of a channel the bounds-checked path
    const long long lastfull = (p.aligned && p.n >= N) ? (p.n - N) / p.hop : -1;
    // registers E - DT .. E - 1 of frame t (its last 128 DT new sample pairs per lane)
    auto load_tail = [&](int t, float2 (&xr)[E]) {
        const long long base = (long long)t * p.hop;
        if (t <= lastfull) {
#pragma unroll
            for (int q = E - DT; q < E; ++q) xr[q] = *reinterpret_cast<const float2*>(xc + base + 2 * (lane + 64 * q));
        } else {
#pragma unroll
            for (int q = E - DT; q < E; ++q) {
                const long long s = base + 2 * (lane + 64 * q);
                xr[q].x = (s < p.n) ? xc[s] : 0.0f;
                xr[q].y = (s + 1 < p.n) ? xc[s + 1] : 0.0f;
            }
        }
    };
    const bool shift_in = PV_FUSED_SHIFT && p.hop == 128 * DT;  // pitch: analysis hop = out hop
    auto load = [&](int t, float2 (&xr)[E]) {
        const long long base = (long long)t * p.hop;
        if (t <= lastfull) {
#pragma unroll
            for (int q = 0; q < E; ++q) xr[q] = *reinterpret_cast<const float2*>(xc + base + 2 * (lane + 64 * q));
        } else {
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const long long s = base + 2 * (lane + 64 * q);
                xr[q].x = (s < p.n) ? xc[s] : 0.0f;
                xr[q].y = (s + 1 < p.n) ? xc[s + 1] : 0.0f;
            }
        }
    };

    // frame t0's samples are requested before the table set-up, whose latency hides theirs
    float2 xr[E];
    if (nfr > 0) load(t0, xr);

    // tables -> LDS: every load issued before the first LDS write, so the set-up costs one
    // round trip instead of one per loop trip (config 2 stamps: 2.6 us of a 27.6 us wave)
    float2 tw0[E];
    float2 tw0h[Geo<LH>::E];  // MODE 4: the half-size inverse transform's first-pass twiddles
    float2 gn[NS];  // synthesis gains of the lane's OLA slots (frame-invariant)
    {
        constexpr int KT = (L + 255) / 256, KB = (B + 255) / 256, KW = N / 256;
        constexpr int KTH = (LH + 255) / 256, KSH = (LH + 1 + 255) / 256;
        static_assert(N % 256 == 0, "window in whole 256-thread trips");
        float2 ttw[KT], tts[KB], tth[KTH], tsh[KSH];
        int tsf[KB], tsc[KB];
        float twn[KW];
        if constexpr (MODE == 4) {
#pragma unroll
            for (int k = 0; k < KTH; ++k)
                if (tid + 256 * k < LH) tth[k] = p.tw_half[tid + 256 * k];
#pragma unroll
            for (int k = 0; k < KSH; ++k)
                if (tid + 256 * k <= LH) tsh[k] = p.tws[2 * (tid + 256 * k)];
            load_tw0<LH>(tw0h, p.tw_half);
        }
#pragma unroll
        for (int k = 0; k < KT; ++k)
            if (tid + 256 * k < L) ttw[k] = p.tw[tid + 256 * k];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            const int i = tid + 256 * k;
            if (i < B) {
                tts[k] = p.tws[i];
                if (MODE == 2) { tsf[k] = p.src_first[i]; tsc[k] = p.src_cnt[i]; }
                if (MODE == 3) tsf[k] = p.src_first[i];
            }
        }
#pragma unroll
        for (int k = 0; k < KW; ++k) twn[k] = p.win[tid + 256 * k];
        load_tw0<L>(tw0, p.tw);
        const float2* g2 = reinterpret_cast<const float2*>(p.gain);
#pragma unroll
        for (int s = 0; s < NS; ++s) gn[s] = g2[64 * s + lane];
#pragma unroll
        for (int k = 0; k < KT; ++k)
            if (tid + 256 * k < L) twl[tid + 256 * k] = ttw[k];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            const int i = tid + 256 * k;
            if (i < B) {
                twsl[i] = tts[k];
                if (MODE == 2) { srcl[2 * i] = tsf[k]; srcl[2 * i + 1] = tsc[k]; }
                // MODE 3 (pitch >= 1): the source's byte offset in a wave's tile, zero slot L + 1
                if (MODE == 3) srcl[i] = (int)sizeof(float2) * (tsf[k] >= 0 ? tsf[k] : L + 1);
            }
        }
        if constexpr (MODE == 4) {
#pragma unroll
            for (int k = 0; k < KTH; ++k)
                if (tid + 256 * k < LH) twl_h[tid + 256 * k] = tth[k];
#pragma unroll
            for (int k = 0; k < KSH; ++k)
                if (tid + 256 * k <= LH) twsl_h[tid + 256 * k] = tsh[k];
        }
#pragma unroll
        for (int k = 0; k < KW; ++k) winl[tid + 256 * k] = twn[k];
    }
    __syncthreads();
    PV_STAMP(2);

    for (int u = 0; u < fw; ++u) {
        const int t = t0 + u;
        if (u < nfr) {
            float2 z[E];
            {
                const float2* wl = reinterpret_cast<const float2*>(winl) + lane;
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    const float2 wv = lds_ld(&wl[64 * q]);
                    z[q].x = xr[q].x * wv.x;
                    z[q].y = xr[q].y * wv.y;
                }
            }
            if (u == 0) PV_STAMP(10);  // frame 0's samples have landed (F <= 7)
            // next frame's samples fly during this frame.  Pitch (analysis hop = out hop =
            // 128 DT): frame t+1's register q is frame t's register q + DT, so only its DT
            // new pairs per lane are loaded (as k_std_analysis's shifted-register input)
            if (u + 1 < nfr) {
                if constexpr (MODE >= 2 && DT < E) {
                    if (shift_in) {
#pragma unroll
                        for (int q = 0; q + DT < E; ++q) xr[q] = xr[q + DT];
                        load_tail(t + 1, xr);
                    } else {
                        load(t + 1, xr);
                    }
                } else {
                    load(t + 1, xr);
                }
            }
            // ---- analysis (k_std_analysis's operations): spectrum row out, kept in sv.  The
            // split takes the partner bins from the last pass's registers by a lane reversal
            // (split_chunk_bp; bit-identical to the LDS-image split)
#if PV_FUSED_BPSPLIT
            fft_run<L, false, false>(z, tile, twl, tw0, lane);
#else
            fft_run<L, false, true>(z, tile, twl, tw0, lane);
#endif
            float2 sv[E + 1];
            // MODE 4: the half-size transform's input Y_s = |X_s| e^{2 i phi_s} = X_s^2 / |X_s|
            // (q = 1: the output phase is exactly 2 phi), bins s <= L/2 — no atan2, no sin/cos
            float2 yh[Geo<LH>::E + 1];
            float2* srow = specc + (long long)t * p.spec_stride + lane;
            // without a spectrum output only the bin pairs holding a bin some output bin reads
            // are analysed (pitch 2.0: bins 0 .. 256 of 512, so 3 of 4 pairs and no bin L): a
            // wave-uniform bound, the skipped bins' slots hold zeros that no gather reads
            const int shi = (wspec || !PV_FUSED_SKIP_UNREAD) ? L : p.src_hi;
            // bin L (real: A = B = Z[0]) once, wave-uniformly, as k_std_analysis's bin_l_real:
            // its contract phase is +0 or pi, no atan2 (bit-identical to the generic bin)
            if (shi >= L) {
                float magL, phL;
#if PV_FUSED_BPSPLIT
                bin_l_real<L, true>(z, twsl, magL, phL);
#else
                bin_l_real_tile<L, true>(tile, twsl, magL, phL);
#endif
                sv[E] = make_float2(magL, phL);
                if (wspec && !p.packed) __builtin_nontemporal_store(f2v{magL, phL}, reinterpret_cast<f2v*>(&srow[L - lane]));
            } else {
                sv[E] = make_float2(0.0f, 0.0f);
            }
            // bins 0 .. E-1 in pairs: the phases of a pair through the packed-fp32 atan2
            // (atan2_pv2, bit-identical to atan2_pv per half)
            constexpr int CH = 2;
            static_for<0, E / CH>([&](auto ic) {
                constexpr int i0 = decltype(ic)::value * CH;
                if (64 * i0 > shi) {
                    sv[i0] = sv[i0 + 1] = make_float2(0.0f, 0.0f);
                    return;
                }
                float2 X[CH];
#if PV_FUSED_BPSPLIT
                split_chunk_bp<L, CH, true, i0, false>(z, twsl, lane, X);
#else
                split_chunk<L, CH, true>(tile, twsl, lane, i0, X);
#endif
                if constexpr (MODE == 4) {
                    static_for<0, CH>([&](auto cc) {
                        constexpr int i = i0 + decltype(cc)::value;
                        if constexpr (i <= Geo<LH>::E) {
                            // X came out doubled (TWICE): Y = X2^2 / (2 |X2|); |X| = 0 -> 0
                            const float2 x2 = X[decltype(cc)::value];
                            const float r = __builtin_fmaf(x2.x, x2.x, x2.y * x2.y);
                            const float rs = (r > 0.0f) ? __builtin_amdgcn_rsqf(r) : 0.0f;
                            yh[i] = make_float2(0.5f * __builtin_fmaf(x2.x, x2.x, -(x2.y * x2.y)) * rs,
                                                x2.x * x2.y * rs);
                        }
                    });
                    if (!wspec) return;  // no row to write: no phase, no magnitude
                }
                float phs[CH];
                {
                    const f2v ph2 = atan2_pv2(X[0].y, X[0].x, X[1].y, X[1].x);
                    phs[0] = ph2.x;
                    phs[1] = ph2.y;
                }
                static_for<0, CH>([&](auto cc) {
                    constexpr int c2 = decltype(cc)::value;
                    constexpr int i = i0 + c2;
                    {
                        const float ph = phs[c2];
                        float mag = __builtin_amdgcn_sqrtf(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
                        mag *= 0.5f;  // X came out doubled (split_chunk TWICE)
                        sv[i] = make_float2(mag, ph);
                        // bins 0..63 go out below (slot 0)
                        if (wspec && i > 0) __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[64 * i]));
                    }
                });
            });
            if (wspec) {
                // slot 0: PV_SPEC_PACKED lane 0 carries bins 0 and L (both real)
                const bool pk0 = p.packed && lane == 0;
                const f2v s0 = pk0 ? f2v{pack_real_bin(sv[0].x, sv[0].y), pack_real_bin(sv[E].x, sv[E].y)}
                                   : f2v{sv[0].x, sv[0].y};
                __builtin_nontemporal_store(s0, reinterpret_cast<f2v*>(&srow[0]));
            }
            wave_lds_sync();
            // ---- processing + resynthesis: inverse FFT's last-pass registers
            if constexpr (MODE == 4) {
                // bins 0 .. L/2 - 1 are registers 0 .. EH - 1, bin L/2 is lane 0 of register
                // EH: the half-size transform's own layout
                constexpr int EH = Geo<LH>::E;
                float2 svh[EH + 1], zh[EH];
                int Mh[EH + 1];
                float phh[EH + 1], ekh[EH + 1];
                unsigned jkh[EH + 1];
#pragma unroll
                for (int i = 0; i <= EH; ++i) svh[i] = yh[i];
                const SynLds stbh{twl_h, twsl_h, nullptr, nullptr, nullptr};
                synth_frame<LH, 5, false, true, false, false, true>(svh, false, 0u, Mh, phh, pmap, stbh, tw0h,
                                                                    tile, lane, zh, ekh, jkh);
                // y[n] = y_half[n mod N/2]: slot s of the frame is the half frame's slot s mod EH
                float2 zs[EH];
#pragma unroll
                for (int idx = 0; idx < EH; ++idx) zs[last_slot<LH>(idx)] = zh[idx];
#pragma unroll
                for (int cs = 0; cs < E; ++cs) {
                    acc[cs].x = __builtin_fmaf(zs[cs % EH].x, gn[cs].x, acc[cs].x);
                    acc[cs].y = __builtin_fmaf(zs[cs % EH].y, gn[cs].y, acc[cs].y);
                }
            } else {
            synth_frame<L, MODE, false, true, false, false, true>(sv, false, 0u, M, phprev, pmap, stb, tw0, tile,
                                                                  lane, z, ekr, jkr);
            // ---- windowed overlap-add in registers
#pragma unroll
            for (int idx = 0; idx < E; ++idx) {
                const int cs = last_slot<L>(idx);
                acc[cs].x = __builtin_fmaf(z[idx].x, gn[cs].x, acc[cs].x);
                acc[cs].y = __builtin_fmaf(z[idx].y, gn[cs].y, acc[cs].y);
            }
            }
        }
        // positions [u*hs, (u+1)*hs) = slots 0..D-1 are final — except a workgroup's head
        // (wave 0, positions < N - hs), which the previous workgroup's tail still overlaps:
        // those go out write-through for the seam hand-off below
        const long long pb = obase + (long long)u * hs + 2 * lane;
        const bool head = (w == 0) && (blockIdx.x > 0) && (u * hs < TL);
        // the head positions of waves 1..3 are read back by close_seams_inline (intra-workgroup
        // seam): temporal stores keep them in L2 for that read (non-temporal ones stream past
        // it and the read-back waits for HBM)
#ifdef PV_FUSED_NT_HEAD
        const bool keep = false;
#else
        const bool keep = (w > 0) && (u * hs < TL);
#endif
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const long long gp = pb + 128 * d;
            if (p.out_aligned && gp + 1 < p.out_len) {
                if (head) st_sc1(outc + gp, f2v{acc[d].x, acc[d].y});
                else if (keep) *reinterpret_cast<f2v*>(outc + gp) = f2v{acc[d].x, acc[d].y};
                else __builtin_nontemporal_store(f2v{acc[d].x, acc[d].y}, reinterpret_cast<f2v*>(outc + gp));
            } else if (head) {
                if (gp < p.out_len) st_sc1(outc + gp, acc[d].x);
                if (gp + 1 < p.out_len) st_sc1(outc + gp + 1, acc[d].y);
            } else {
                if (gp < p.out_len) outc[gp] = acc[d].x;
                if (gp + 1 < p.out_len) outc[gp + 1] = acc[d].y;
            }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) acc[s] = (s + D < NS) ? acc[(s + D < NS) ? s + D : 0] : make_float2(0.0f, 0.0f);
        if (u < 6) PV_STAMP(3 + u);
    }
    PV_STAMP(11);  // frames end; slots 3..9 = frames 0..6
#ifdef PV_FUSED_STAMPS
    __syncthreads();
    PV_STAMP(9);  // the workgroup's slowest wave has finished its frames (F <= 6)
#endif
    close_seams_inline<L, NS, D>(acc, tiles, w, lane, c, blockIdx.x, p.nwg, obase, fw, hs, outc,
                                 p.out_len, p.out_aligned != 0, p.tails, p.tail_len, p.seam_flags);
#ifdef PV_FUSED_STAMPS
    {
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime(), mt1 = __builtin_amdgcn_s_memtime();
        stamp(0, st_rt0);
        stamp(1, st_mt0);
        stamp(12, rt1);
        stamp(13, mt1);
        // HW_ID (CU / SIMD / SE) and XCC_ID
        stamp(14, (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)));
        stamp(15, (unsigned long long)__builtin_amdgcn_s_getreg(20 | (15 << 11)));
    }
#endif
#undef PV_STAMP
}

bool fused_supported(int L, int hs) {
    return L >= 128 && L <= 512 && hs % 128 == 0 && (hs / 128 == 1 || hs / 128 == 2 || hs / 128 == 4) &&
           hs <= L;
}

// only the geometries fused_supported admits are instantiated (out hop <= L)
template <int LL, int MM, int DT>
static hipError_t launch_fused_t(dim3 grid, const FusedParams& p, hipStream_t s) {
    if constexpr (128 * DT <= LL) {
        hipLaunchKernelGGL((k_fused<LL, MM, DT>), grid, dim3(256), FuGeo<LL>::BYTES, s, p);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;
    }
}
template <int LL, int MM>
static hipError_t launch_fused_l(int dt, dim3 grid, const FusedParams& p, hipStream_t s) {
    switch (dt) {
        case 1: return launch_fused_t<LL, MM, 1>(grid, p, s);
        case 2: return launch_fused_t<LL, MM, 2>(grid, p, s);
        case 4: return launch_fused_t<LL, MM, 4>(grid, p, s);
        default: return hipErrorInvalidValue;
    }
}
template <int MM>
static hipError_t launch_fused_m(int L, int dt, dim3 grid, const FusedParams& p, hipStream_t s) {
    switch (L) {
        case 128: return launch_fused_l<128, MM>(dt, grid, p, s);
        case 256: return launch_fused_l<256, MM>(dt, grid, p, s);
        case 512: return launch_fused_l<512, MM>(dt, grid, p, s);
        default: return hipErrorInvalidValue;
    }
}

// mode: 0 STANDARD stretch, 2 STANDARD pitch (q = 1 only; the caller checks); pitch >= 1
// takes the MODE 3 kernels (one source per bin: the select-free gather, as k_synthesis)
hipError_t launch_fused(int L, int mode, int channels, const FusedParams& p, hipStream_t s) {
    const dim3 grid(p.nwg, channels);
    const int dt = p.hs / 128;
    // pitch exactly 2: the periodic half-size resynthesis (MODE 4)
    if (mode == 2 && p.rho == 2.0f && p.tw_half != nullptr) {
        if (L == 256) return launch_fused_l<256, 4>(dt, grid, p, s);
        if (L == 512) return launch_fused_l<512, 4>(dt, grid, p, s);
    }
    if (mode == 2 && p.rho >= 1.0f) return launch_fused_m<3>(L, dt, grid, p, s);
    return mode == 2 ? launch_fused_m<2>(L, dt, grid, p, s) : launch_fused_m<0>(L, dt, grid, p, s);
}

}  // namespace pv
