// pv_chain.hip — analysis -> unwrap scan -> resynthesis in ONE launch for STANDARD
// configurations whose output phase depends on the unwrap count (q > 1: BASELINE config 3's
// time stretch 0.5 and pitch ratios p/2^e), chained over the runs of each channel.
//
// The split path needs three launches because frame t's output phase needs M(t), the
// channel's unwrap count through frame t, i.e. every earlier frame's decisions (DESIGN.md
// §3.3): analysis -> k_carry scan -> synthesis, with the 7 GB spectrum written by one
// launch and read back by another long after it left the caches.  Here a workgroup (4
// waves = 4 consecutive runs of F frames of one channel, as in k_synthesis):
//   1. takes a ticket (atomic counter) that names its (run group, channel), time-major:
//      run group g of every channel before run group g + 1 of any, so a workgroup only ever
//      waits for one that started before it (no dispatch-order assumption: whoever holds
//      ticket t - C is resident or done);
//   2. analyses its 4 runs (pv_ana_run.hpp, no halo frame): spectrum rows out, each run's
//      decision sum for its frames 2..F and the phases of its first and last frame;
//   3. waits for the record of run group g - 1 of its channel (the unwrap count through
//      that group's last frame and that frame's phases), computes the boundary decision of
//      each run's first frame, the carry at each run's start and its own record, which it
//      publishes at once (before resynthesising, so the chain advances at analysis speed);
//   4. resynthesises its runs (pv_syn_run.hpp) re-reading the rows it wrote, and closes
//      every overlap-add seam in the same launch (close_seams_inline).
// Integer decisions and their sums are exact, so the carries — and every output sample —
// equal the split path's bit for bit (tests/test_gpu_chain.py); no halo frame, no run
// records, no k_carry / k_seam launch.
//
// Measured on config 3: 4.52 ms per step at F = 48 against the split
// path's 4.45 — one kernel holds the analysis and the resynthesis registers (154 VGPRs:
// 3 waves per SIMD where the split analysis runs 5), which costs more than the launches,
// halo frames and the spectrum's second HBM pass it saves.  So it is opt-in (PV_CHAIN=1).
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms"): the record is stored write-through (sc1)
// by one wave, which waits for its stores before its sc1 flag store (the launch's epoch);
// the consumer polls the flag with sc1 loads and reads the record with sc1 loads.  Every
// wait is bounded: a poll that exceeds ~1 s sets p.err and proceeds (wrong output, but the
// grid always drains).
#include "pv_ana_run.hpp"
#include "pv_syn_run.hpp"

#ifndef PV_CHAIN_WAVES
#define PV_CHAIN_WAVES 3  // waves per SIMD k_chain is compiled for
#endif
#ifndef PV_CHAIN_NT_SPEC
#define PV_CHAIN_NT_SPEC 1  // non-temporal row stores (measured: temporal stores, which the
                            // Infinity Cache keeps for the re-read, -0.5 %: the resynthesis
                            // is not memory-bound)
#endif
#ifndef PV_CHAIN_NT_ROWS
#define PV_CHAIN_NT_ROWS 1  // non-temporal row loads in the resynthesis (same measurement)
#endif

namespace pv {

__device__ __forceinline__ unsigned ld_sc1_u(const unsigned* p) {
    unsigned v;
    asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st_sc1_u(unsigned* p, unsigned v) {
    asm volatile("global_store_dword %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}

template <int L>
struct ChainGeo {
    static constexpr int N = 2 * L;
    static constexpr int B = L + 1;
    // float offsets of the LDS carve-up
    static constexpr int O_TW = 0;                            // L float2
    static constexpr int O_TWS = O_TW + 2 * L;                // L+1 float2 (+1 pad)
    static constexpr int O_TILE = O_TWS + 2 * (L + 2);        // 4 x TILE float2
    static constexpr int O_WIN = O_TILE + 2 * 4 * Geo<L>::TILE;  // N (analysis only)
    static constexpr int O_EK = O_WIN + N;                    // B (+3)
    static constexpr int O_JK = O_EK + B + 3;                 // B (+3)
    static constexpr int O_SRC = O_JK + B + 3;                // 2B (+2) {first, count}
    static constexpr int FLOATS = O_SRC + 2 * B + 2;
    static constexpr size_t BYTES = sizeof(float) * FLOATS;
    // exchange area after the analysis (tiles + window): 4 last-frame phase rows, the
    // predecessor's last phases, its unwrap count and the 4 runs' decision totals
    static constexpr int BP = (B + 7) & ~7;
    static_assert(10 * BP <= O_EK - O_TILE, "exchange area exceeds tiles + window");
    static_assert(O_SRC % 2 == 0 && O_TILE % 4 == 0, "alignment of the LDS carve-up");
};

// MODE 0 stretch / 2 pitch; DT = out hop / 128 (register overlap-add); D = hop / 128
// (shifted-register analysis input); e_k per lane (64 a multiple of the hop divisor);
// q a power of two <= 4096 (RACC synthesis).
template <int L, int MODE, int DT, int D>
__global__ __launch_bounds__(256, PV_CHAIN_WAVES) void k_chain(ChainParams p) {
    using G_ = Geo<L>;
    using CG = ChainGeo<L>;
    using T_ = SynTraits<L, MODE, DT, true>;
    static_assert(T_::ROLA && T_::RACC, "chained path: register overlap-add, power-of-two q");
    constexpr int E = G_::E;
    constexpr int N = CG::N;
    constexpr int B = CG::B;
    constexpr int NS = T_::NS;
    constexpr int DS = T_::D;
    constexpr bool GREG = T_::GREG;
    static_assert(GREG, "chained path: gains in registers");
    extern __shared__ __attribute__((aligned(16))) float csm[];
    float2* twl = reinterpret_cast<float2*>(csm + CG::O_TW);
    float2* twsl = reinterpret_cast<float2*>(csm + CG::O_TWS);
    float2* tiles = reinterpret_cast<float2*>(csm + CG::O_TILE);
    float* winl = csm + CG::O_WIN;
    float* ekl = csm + CG::O_EK;
    unsigned* jkl = reinterpret_cast<unsigned*>(csm + CG::O_JK);
    int* srcl = reinterpret_cast<int*>(csm + CG::O_SRC);
    __shared__ unsigned s_ticket;

    const AnaParams& pa = p.a;
    const SynParams& ps = p.s;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[E];
    load_tw0<L>(tw0, pa.tw);
    for (int i = tid; i < L; i += 256) twl[i] = pa.tw[i];
    for (int i = tid; i < B; i += 256) {
        twsl[i] = pa.tws[i];
        ekl[i] = ps.ek[i];
        jkl[i] = __float_as_uint((float)ps.jk_mod[i] * ps.inv_q);  // (p j_k mod q) / q, exact
        if (MODE == 2) { srcl[2 * i] = ps.src_first[i]; srcl[2 * i + 1] = ps.src_cnt[i]; }
    }
    for (int i = tid; i < N; i += 256) winl[i] = pa.win[i];
    const float e_lane = pa.ek[lane];
    if (tid == 0) s_ticket = __hip_atomic_fetch_add(p.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();

    // ---- 1. ticket -> (run group, channel), time-major
    const unsigned tk = __builtin_amdgcn_readfirstlane(s_ticket);
    const int C = p.channels;
    const int wg = (int)(tk / (unsigned)C), c = (int)(tk % (unsigned)C);
    const int F = pa.F;
    const int t0 = (wg * 4 + w) * F;
    const int nfr = max(0, min(F, pa.frames - t0));  // real frames of this wave's run
    const int BP = CG::BP;

    // ---- 2. analysis of the wave's run (no halo frame)
    float phl[E + 1], sacc[E + 1], phf[E + 1];
    if (nfr > 0)
        ana_run<L, false, D, false, (bool)PV_CHAIN_NT_SPEC>(pa, AnaLds{twl, twsl, winl, ekl}, tiles + w * G_::TILE, tw0, lane, c,
                                           t0, nfr, e_lane, nullptr, phl, sacc, phf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows have landed (re-read in step 4)
    __syncthreads();  // every wave is done with its tile and the window

    // ---- 3. exchange and chain
    float* xph = csm + CG::O_TILE;           // [4][BP] phase of each run's last frame
    float* xprev = xph + 4 * BP;             // [BP] phase of the previous run group's last frame
    int* xmin = reinterpret_cast<int*>(xprev + BP);  // [BP] unwrap count through that frame
    int* xtot = xmin + BP;                   // [4][BP] decisions of each run (first frame included)
    if (nfr > 0) PV_FOR_BINS(E, lane, { xph[w * BP + k] = phl[i]; })
    if (w == 0) {
        if (wg > 0) {
            const long long r = (long long)(wg - 1) * C + c;
#ifndef PV_CHAIN_NOWAIT  // timing-only ablation: never wait (carries wrong)
            if (lane == 0) {
                const unsigned* flag = p.flags + r;
                unsigned it = 0;
                while (ld_sc1_u(flag) != p.epoch) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++it > (1u << 24)) {  // ~1 s: never expected; drain the grid instead of hanging
                        __hip_atomic_fetch_or(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
#endif
            __builtin_amdgcn_wave_barrier();
            const float* rec = reinterpret_cast<const float*>(p.rec) + r * 2 * BP;
            PV_FOR_BINS(E, lane, {
                xmin[k] = __float_as_int(ld_sc1(rec + k));
                xprev[k] = ld_sc1(rec + BP + k);
            })
        } else {
            PV_FOR_BINS(E, lane, { xmin[k] = 0; xprev[k] = 0.0f; })  // phi(-1) = 0, M(-1) = 0
        }
    }
    __syncthreads();
    // the decision of the run's first frame against the previous frame (another run's last)
    int bnd[E + 1];
    PV_FOR_BINS(E, lane, {
        int b = 0, tot = 0;
        if (nfr > 0) {
            const float prev = (w == 0) ? xprev[k] : xph[(w - 1) * BP + k];
            b = unwrap_count(phf[i], prev, lds_ld(&ekl[k]));
            tot = b - (int)sacc[i];  // sacc = -(sum of the run's other decisions)
        }
        bnd[i] = b;
        xtot[w * BP + k] = tot;
    })
    __syncthreads();
    int carry[E + 1];
    PV_FOR_BINS(E, lane, {
        int m = xmin[k];
        for (int v = 0; v < w; ++v) m += xtot[v * BP + k];
        carry[i] = m + bnd[i];  // M(t0): every decision through the run's first frame
    })
    const int nwg = p.nwg;
    if (w == 3 && wg + 1 < nwg) {
        // this run group's record: the count through its last frame and that frame's phases
        float* rec = reinterpret_cast<float*>(p.rec) + ((long long)wg * C + c) * 2 * BP;
        PV_FOR_BINS(E, lane, {
            const int incl = xmin[k] + xtot[k] + xtot[BP + k] + xtot[2 * BP + k] + xtot[3 * BP + k];
            st_sc1(rec + k, __int_as_float(incl));
            st_sc1(rec + BP + k, xph[3 * BP + k]);
        })
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st_sc1_u(p.flags + (long long)wg * C + c, p.epoch);
    }
    __syncthreads();  // exchange reads done before the synthesis reuses the tiles

    // ---- 4. resynthesis of the wave's run from its rows, seams in the same launch
    int M[E + 1];
    float php[E + 1];
    {
        const unsigned qm = (unsigned)ps.q - 1u;
        PV_FOR_BINS(E, lane, {
            const unsigned mq = ((unsigned)ps.p_mod * ((unsigned)carry[i] & qm)) & qm;
            M[i] = __float_as_int((float)mq * ps.inv_q);
            php[i] = 0.0f;
        })
    }
    float2 acc[NS];
    syn_run<L, MODE, DT, true, (bool)PV_CHAIN_NT_ROWS, true>(ps, SynCarve{twl, twsl, tiles, nullptr, nullptr, ekl, jkl, srcl}, tw0,
                                            lane, w, c, t0, nfr, w == 0 && wg > 0, M, php, acc);
    close_seams_inline<L, NS, DS>(acc, tiles, w, lane, c, wg, nwg, (long long)t0 * ps.hs, F, ps.hs,
                                  ps.out + (long long)c * ps.ldo, ps.out_len, ps.tails, ps.tail_len, p.seam_flags);
}

bool chain_supported(int L, int hs, int hop, int hop_div) {
    const int dt = hs / 128, d = hop / 128;
    return (L == 256 || L == 512) && hs % 128 == 0 && (dt == 1 || dt == 2) && hs <= L && hop % 128 == 0 &&
           (d == 1 || d == 2) && d < L / 64 && 64 % hop_div == 0;
}

size_t chain_lds_bytes(int L) { return L == 256 ? ChainGeo<256>::BYTES : ChainGeo<512>::BYTES; }

// mode: 0 STANDARD stretch, 2 STANDARD pitch (chain_supported and q = 2^e <= 4096 checked
// by the caller); grid = channels x nwg workgroups, mapped by ticket
hipError_t launch_chain(int L, int mode, const ChainParams& p, hipStream_t s) {
    const dim3 grid((unsigned)((long long)p.channels * p.nwg));
    const int dt = p.s.hs / 128, d = p.a.hop / 128;
#define PV_CH(LL_, MM_, DT_, D_) hipLaunchKernelGGL((k_chain<LL_, MM_, DT_, D_>), grid, dim3(256), ChainGeo<LL_>::BYTES, s, p)
#define PV_CH_D(LL_, MM_, DT_)                 \
    if (d == 1) PV_CH(LL_, MM_, DT_, 1);       \
    else PV_CH(LL_, MM_, DT_, 2)
#define PV_CH_DT(LL_, MM_)                     \
    if (dt == 1) { PV_CH_D(LL_, MM_, 1); }     \
    else { PV_CH_D(LL_, MM_, 2); }
#define PV_CH_L(MM_)                           \
    if (L == 256) { PV_CH_DT(256, MM_); }      \
    else { PV_CH_DT(512, MM_); }
    if (mode == 2) { PV_CH_L(2); } else { PV_CH_L(0); }
#undef PV_CH_L
#undef PV_CH_DT
#undef PV_CH_D
#undef PV_CH
    return hipGetLastError();
}

}  // namespace pv
