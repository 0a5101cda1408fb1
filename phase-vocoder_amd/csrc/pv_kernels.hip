// pv_kernels.hip — the phase-vocoder hot path as hand-written CDNA4 (gfx950) kernels.
//
// Pipeline, all channels x frames in one launch per stage:
//   K1  k_std_analysis / k_compat_analysis   frame -> window -> real FFT -> {mag, phase}
//         (+ per-run sums of the integer unwrap decisions, STANDARD) — pv_analysis.hip
//   K2  k_carry (+ k_runsum when the spectrum did not come from K1)
//         exclusive integer scan of the decisions over runs -> unwrap count at run start
//   K3  k_synthesis<MODE>   phase propagation -> polar->rect -> inverse real FFT ->
//         window -> overlap-add of the run in an LDS ring -> plain stores
//   K4  k_seam   adds each workgroup's overlap tail into the next workgroup's head
//
// Geometry: one frame per wavefront, and each wave owns a RUN of F consecutive frames of
// one channel which it walks in order (the unwrap state stays in registers, the
// overlap-add in a per-wave LDS ring).  A workgroup = 4 waves = 4 consecutive runs.
#include "pv_syn_run.hpp"

namespace pv {

// ------------------------------------------------------------------ K2 scans
// run record from an existing spectrum (pv_resynthesis path), the layout K1 writes
// (kRecFields): S = the decisions of the frames after the run's first, phi(t0), phi(last).
__global__ __launch_bounds__(256) void k_runsum(ScanParams p) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int run = blockIdx.y, c = blockIdx.z;
    if (k > p.L) return;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    // PV_SPEC_PACKED rows: bins 0 and L are the sign bits of slot 0 {s0, sL}
    const bool real_bin = p.packed && (k == 0 || k == p.L);
    const float2* s = p.spec + (long long)c * p.ld_spec + (long long)t0 * p.spec_stride + (real_bin ? 0 : k);
    auto phase = [&](long long u) {
        const float2 v = s[u * p.spec_stride];
        if (!real_bin) return v.y;
        return (__float_as_uint(k == 0 ? v.x : v.y) >> 31) ? kPi : 0.0f;
    };
    const float e = p.ek[k];
    const float ph0 = phase(0);
    float prev = ph0;
    int acc = 0;
    for (int u = 1; u < nfr; ++u) {
        const float ph = phase(u);
        acc += unwrap_count(ph, prev, e);
        prev = ph;
    }
    int* dst = p.runsum + ((long long)c * p.nruns + run) * kRecFields * p.bins_pad;
    dst[k] = acc;
    dst[p.bins_pad + k] = __float_as_int(ph0);
    dst[2 * p.bins_pad + k] = __float_as_int(prev);
}

// carry[run] = M(t0) = sum over earlier runs of (m0 + S) + m0(run), where m0(run) = m(t0) is
// the decision of the run's first frame, made here from its record's phi(t0) and the previous
// run's phi(last) (phi(-1) = 0): the same operations as K1's decisions (unwrap_count).
// Block = 64 bins x SEG run segments (one wave each): pass 1 sums each segment, the
// segment offsets are scanned in LDS, pass 2 rescans the segment writing carries.  All
// integer, so the split of the scan changes no bit.
template <int SEG>
__global__ __launch_bounds__(64 * SEG) void k_carry(ScanParams p) {
    __shared__ int tot[SEG][64];
    const int lane = threadIdx.x & 63;
    const int sg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k = blockIdx.x * 64 + lane;
    const int c = blockIdx.y;
    const int BP = p.bins_pad;
    constexpr int RF = kRecFields;
    const int per = (p.nruns + SEG - 1) / SEG;
    const int r0 = min(p.nruns, sg * per), r1 = min(p.nruns, r0 + per);
    const bool on = k <= p.L;
    const int* rs = p.runsum + (long long)c * p.nruns * RF * BP + (on ? k : 0);
    int* cr = p.carry + (long long)c * p.nruns * BP + (on ? k : 0);
    const float e = p.ek[on ? k : 0];
    // S, phi(t0), phi(last) of run r
    auto S_of = [&](int r) { return rs[(long long)r * RF * BP]; };
    auto first_of = [&](int r) { return __int_as_float(rs[(long long)r * RF * BP + BP]); };
    auto last_of = [&](int r) { return __int_as_float(rs[(long long)r * RF * BP + 2 * BP]); };
    // phi(-1) = 0 and M = 0 before the stream, or a longer stream's state before this segment
    const float phi0 = (p.phi_in && on) ? p.phi_in[(long long)c * BP + k] : 0.0f;
    int M = 0;
    int run = r0;
    if constexpr (SEG > 1) {  // pass 1 only feeds the other segments' offsets
        int T = 0;
        float prev = (r0 > 0 && r0 < r1) ? last_of(r0 - 1) : phi0;
        for (; run + 4 <= r1; run += 4) {
            int sv[4];
            float fv[4], lv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                sv[j] = S_of(run + j);
                fv[j] = first_of(run + j);
                lv[j] = last_of(run + j);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                T += unwrap_count(fv[j], prev, e) + sv[j];
                prev = lv[j];
            }
        }
        for (; run < r1; ++run) {
            T += unwrap_count(first_of(run), prev, e) + S_of(run);
            prev = last_of(run);
        }
        tot[sg][lane] = T;
        __syncthreads();
        for (int j = 0; j < sg; ++j) M += tot[j][lane];
    }
    if (!on) return;
    if (p.carry_in) M += p.carry_in[(long long)c * BP + k];
    run = r0;
    float prev = (r0 > 0 && r0 < r1) ? last_of(r0 - 1) : phi0;
    for (; run + 4 <= r1; run += 4) {
        int sv[4];
        float fv[4], lv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sv[j] = S_of(run + j);
            fv[j] = first_of(run + j);
            lv[j] = last_of(run + j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            M += unwrap_count(fv[j], prev, e);
            cr[(long long)(run + j) * BP] = M;
            M += sv[j];
            prev = lv[j];
        }
    }
    for (; run < r1; ++run) {
        M += unwrap_count(first_of(run), prev, e);
        cr[(long long)run * BP] = M;
        M += S_of(run);
        prev = last_of(run);
    }
}

// ------------------------------------------------------------------ stream segments
// A stream cut into consecutive frame segments (one per rank, pv_segment_*): the unwrap count
// is an integer sum, so a segment's carries need only, per bin, the earlier segments' decision
// totals and their boundary phases — the decisions at the segment boundaries are made here
// with the same operations as everywhere else (unwrap_count), so the carries equal the whole
// stream's bit for bit.
// k_segsum: T = the decisions of the segment's frames after its first (run 0's S, then each
// later run's first decision against the previous run's last phase plus its S), phi(first),
// phi(last).
__global__ __launch_bounds__(256) void k_segsum(SegParams p) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (k > p.L) return;
    const int BP = p.bins_pad;
    constexpr int RF = kRecFields;
    const int* rs = p.runsum + (long long)c * p.nruns * RF * BP + k;
    const float e = p.ek[k];
    int T = rs[0];
    float prev = __int_as_float(rs[2 * BP]);
    for (int r = 1; r < p.nruns; ++r) {
        const int* rr = rs + (long long)r * RF * BP;
        T += unwrap_count(__int_as_float(rr[BP]), prev, e) + rr[0];
        prev = __int_as_float(rr[2 * BP]);
    }
    int* dst = p.summary + (long long)c * kSegFields * BP + k;
    dst[0] = T;
    dst[BP] = rs[BP];
    dst[2 * BP] = __float_as_int(prev);
}

// k_segcarry: the state before segment `seg` from the summaries of segments 0 .. seg - 1:
// M = sum over j of (m(first_j) against last_{j-1}, last_{-1} = 0) + T_j; phi_in = last_{seg-1}
__global__ __launch_bounds__(256) void k_segcarry(SegParams p) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (k >= p.bins_pad) return;
    const int BP = p.bins_pad;
    int M = 0;
    float prev = 0.0f;
    if (k <= p.L) {
        const float e = p.ek[k];
        for (int j = 0; j < p.seg; ++j) {
            const int* sj = p.summaries + ((long long)j * p.channels + c) * kSegFields * BP + k;
            M += unwrap_count(__int_as_float(sj[BP]), prev, e) + sj[0];
            prev = __int_as_float(sj[2 * BP]);
        }
    }
    p.carry_in[(long long)c * BP + k] = M;
    p.phi_in[(long long)c * BP + k] = prev;
}

// ------------------------------------------------------------------ K3 synthesis
// One wave = one run of F frames (virtually padded to F: frames >= `frames` are zero).
// MODE 0/2: STANDARD time stretch / pitch shift — output phase
//         rho*(phi + 2 pi (M_dec + (t+1) j_k)), Hann synthesis window with
//         the overlap normalisation folded into gain[].
// MODE 1: REF_COMPAT — kernel.cu:352-432: x' = m cos(phi), y' = x' sin(phi), C2R N, /N,
//         swap halves (rot = N/2), Hamming window (gain = w/N).
// Overlap-add: a position is final once the frame that starts after it has been added;
// final samples are stored straight to `out`.
//   DT > 0 (out hop = 128 DT, L <= 1024): in registers.  After the inverse FFT's last pass
//     lane holds points lane + 64 c, i.e. samples 2 lane + {0,1} + 128 c, so every
//     position a lane ever touches is congruent to 2 lane (+1) mod 128: acc[c] covers run
//     positions u*hs + 128 c + 2 lane + {0,1}; per frame the oldest DT slots are stored
//     and the rest shift down.  No LDS ring, no final FFT store.  Runs away from the ends
//     of the output take a loop with unconditional stores and a self-tracked prefetch
//     of the next spectrum row (gload_pairs / vm_wait, pv_device.hpp).
//   DT = 0 (any out hop): per-wave LDS ring of N samples.
// After the loop the three intra-workgroup seams are closed from the neighbours' tails in
// LDS (one barrier); the workgroup's last tail goes to `tails` for k_seam.
// waves per SIMD the synthesis is compiled for (__launch_bounds__): L = 512 at <= 168
// VGPRs; L = 1024 bounded at 1 only so that the compiler may use up to 256 VGPRs: the
// kernels compile to <= 256 without AGPRs, so the 2 waves/SIMD their LDS sets hold
// (tests/test_abi.py checks both)
constexpr int kSynWaves512 = 3;
constexpr int kSynWaves1024 = 1;
template <int L, int MODE, int DT, bool QPOW2 = false, bool LANEK = false, int NR = Geo<L>::E>
__global__ __launch_bounds__(256, (L <= 256) ? 4 : (L == 512) ? kSynWaves512 : (L == 1024) ? kSynWaves1024 : 1) void k_synthesis(SynParams p) {
    using G_ = Geo<L>;
    constexpr bool ROLA = DT > 0;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr int SPW = N / 64;  // samples per lane per frame
    constexpr int B = L + 1;
    constexpr bool GREG = SynTraits<L, MODE, DT, QPOW2>::GREG;  // ROLA gains in registers (else LDS)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);                     // L
    float2* twsl = twl + L;                                            // L (+2 pad)
    float2* tiles = twsl + (L + 2);                                    // 4 x TILE
    float* after_tiles = reinterpret_cast<float*>(tiles + 4 * G_::TILE);
    // 4 x N tails: ROLA writes them only after the frame loop, into the tile area
    // (4 TILE float2 >= 4 N floats); the LDS ring of DT = 0 is live throughout
    float* rings = ROLA ? reinterpret_cast<float*>(tiles) : after_tiles;
    float* gainl = ROLA ? after_tiles : rings + 4 * N;                 // N (unless GREG)
    float* ekl = gainl + (GREG ? 0 : N);                               // B (+pad)
    unsigned* jkl = reinterpret_cast<unsigned*>(ekl + (B + 3));        // B (+pad)
    int* srcl = reinterpret_cast<int*>(jkl + (B + 3));                 // 2 x B (pitch)
    const int hs = p.hs;
    const int TL = N - hs;
    constexpr bool RACC = SynTraits<L, MODE, DT, QPOW2>::RACC;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[Geo<L>::E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < L; i += 256) { twl[i] = p.tw[i]; twsl[i] = p.tws[i]; }
    if (!GREG)
        for (int i = tid; i < N; i += 256) gainl[i] = p.gain[i];
    if (MODE != 1) {
        for (int i = tid; i < B; i += 256) {
            ekl[i] = p.ek[i];
            // RACC: (p j_k mod q) / q as a float (exact: q <= 4096)
            jkl[i] = RACC ? __float_as_uint((float)p.jk_mod[i] * p.inv_q) : p.jk_mod[i];
            if (MODE == 2) { srcl[2 * i] = p.src_first[i]; srcl[2 * i + 1] = p.src_cnt[i]; }
            // MODE 3: the source's byte offset in a wave's tile, L + 1 (zero slot) if none
            if (MODE == 3) srcl[i] = (int)sizeof(float2) * (p.src_first[i] >= 0 ? p.src_first[i] : L + 1);
        }
    }
    float* ring = rings + w * N;  // ROLA: the run's tail, written after the frame loop
    if (!ROLA) {
#pragma unroll
        for (int i = 0; i < SPW; ++i) ring[lane + 64 * i] = 0.0f;
    }
    __syncthreads();

    const int c = blockIdx.y;
    const int run = blockIdx.x * 4 + w;
    const int t0 = run * p.F;
    const int nfr = max(0, min(p.F, p.frames - t0));  // real frames of this wave's run
    float* outc = p.out + (long long)c * p.ldo;
    const long long obase = (long long)t0 * hs;

    int M[E + 1];
    float phprev[E + 1];
    if (MODE != 1 && nfr > 0) {
        // no carries when the output phase does not depend on the unwrap count (q = 1)
        const int* cr = p.carry ? p.carry + ((long long)c * p.nruns + run) * p.bins_pad : nullptr;
        if constexpr (RACC) {
            const unsigned qm = (unsigned)p.q - 1u;
            PV_FOR_BINS(E, lane, {
                const unsigned mq = cr ? ((unsigned)p.p_mod * ((unsigned)cr[k] & qm)) & qm : 0u;
                M[i] = __float_as_int((float)mq * p.inv_q);
                phprev[i] = 0.0f;
            })
        } else {
            PV_FOR_BINS(E, lane, { M[i] = cr ? cr[k] : 0; phprev[i] = 0.0f; })
        }
    }
    constexpr int NS = SynTraits<L, MODE, DT, QPOW2>::NS, D = SynTraits<L, MODE, DT, QPOW2>::D;
    float2 acc[NS];
    syn_run<L, MODE, DT, QPOW2, LANEK, NR>(
        p, SynCarve{twl, twsl, tiles, rings, gainl, ekl, jkl, srcl}, tw0, lane, w, c, t0, nfr, M, phprev, acc);
    if constexpr (ROLA) {
        // the run's tail (positions F*hs + j, j < N - hs) -> ring[j], over the tiles
        __syncthreads();
        float2* r2 = reinterpret_cast<float2*>(ring);
#pragma unroll
        for (int s = 0; s < NS - D; ++s) r2[64 * s + lane] = acc[s];
    }
    __syncthreads();
    const int nwg = (p.nruns + 3) / 4;
    const bool last = (blockIdx.x + 1 >= nwg);
    if constexpr (ROLA && N > 128 * DT) {
        if (p.out_aligned) {
            // the overlap is TM = (N - 128 DT) / 128 float2 per lane at positions 2 lane +
            // 128 m; positions are even and out_len is even, so a pair is wholly inside out
            // or wholly past it.  The head read-back is one batch of loads and one wait (per
            // 64 samples, a load-add-store was one serialized round trip: 14 at config 3)
            constexpr int TM = (N - 128 * DT) / 128;
            const float2* own2 = reinterpret_cast<const float2*>(ring) + lane;
            if (w > 0) {
                const float2* prev2 = reinterpret_cast<const float2*>(rings + (w - 1) * N) + lane;
                f2v hd[TM];
#pragma unroll
                for (int m = 0; m < TM; ++m) {
                    const long long gp = obase + 2 * lane + 128 * m;
                    hd[m] = (gp < p.out_len) ? *reinterpret_cast<const f2v*>(outc + gp) : f2v{0.0f, 0.0f};
                }
#pragma unroll
                for (int m = 0; m < TM; ++m) {
                    const long long gp = obase + 2 * lane + 128 * m;
                    const float2 t = prev2[64 * m];
                    if (gp < p.out_len)
                        __builtin_nontemporal_store(f2v{hd[m].x + t.x, hd[m].y + t.y}, reinterpret_cast<f2v*>(outc + gp));
                }
            }
            if (w == 3) {
                const long long nb = obase + (long long)p.F * hs + 2 * lane;
                float* tdst = p.tails + ((long long)c * nwg + blockIdx.x) * p.tail_len + 2 * lane;
#pragma unroll
                for (int m = 0; m < TM; ++m) {
                    const float2 v = own2[64 * m];
                    if (last) {
                        if (nb + 128 * m < p.out_len)
                            __builtin_nontemporal_store(f2v{v.x, v.y}, reinterpret_cast<f2v*>(outc + nb + 128 * m));
                    } else {
                        *reinterpret_cast<f2v*>(tdst + 128 * m) = f2v{v.x, v.y};
                    }
                }
            }
            return;
        }
    }
    // seams: run w's tail (positions F*hs + j) overlaps run w+1's head
    if (w > 0) {
        const float* prev = rings + (w - 1) * N;
        for (int j = lane; j < TL; j += 64) {
            const long long gp = obase + j;
            if (gp < p.out_len) outc[gp] += prev[ROLA ? j : ((p.F * hs + j) & (N - 1))];
        }
    }
    if (w == 3) {
        float* tdst = p.tails + ((long long)c * nwg + blockIdx.x) * p.tail_len;
        for (int j = lane; j < TL; j += 64) {
            const float v = ring[ROLA ? j : ((p.F * hs + j) & (N - 1))];
            if (last) {
                const long long gp = obase + (long long)p.F * hs + j;
                if (gp < p.out_len) outc[gp] = v;
            } else {
                tdst[j] = v;
            }
        }
    }
}

// ------------------------------------------------------------------ K4 seam
// adds each workgroup's last tail into the next workgroup's head (and ola_in at 0)
__global__ __launch_bounds__(256) void k_seam(SeamParams p) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y, c = blockIdx.z;
    if (j >= p.tail_len) return;
    float* outc = p.out + (long long)c * p.ldo;
    if (b == 0) {
        if (p.ola_in != nullptr && j < p.out_len) outc[j] += p.ola_in[(long long)c * p.ld_ola + j];
    } else {
        const long long pos = (long long)b * 4 * p.F * p.hs + j;
        if (pos < p.out_len)
            outc[pos] += p.tails[((long long)c * p.nwg + (b - 1)) * p.tail_len + j];
    }
}

// ------------------------------------------------------------------ harmoniser mix
// Streams the K voice outputs once: each thread sums one sample position over the voices.
__global__ __launch_bounds__(256) void k_mix(MixParams p) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (i >= p.len) return;
    const float* src = p.src + (long long)c * p.ldo + i;
    float acc = 0.0f;
    for (int k = 0; k < p.voices; ++k) acc = __builtin_fmaf(p.gain[k], src[(long long)k * p.ld_voice], acc);
    p.dst[(long long)c * p.ld_mix + i] = acc;
}

hipError_t launch_mix(const MixParams& p, hipStream_t s) {
    dim3 grid((unsigned)((p.len + 255) / 256), p.channels);
    hipLaunchKernelGGL(k_mix, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

// ------------------------------------------------------------------ OVERLAPTEST
// kernel.cu:289-298: cudaWindow, cufftShift (out-of-place), cufftShift (in place),
// cudaWindow, cudaOverlapAdd -> out[k] = w[k]^2 x[k] + back[k + hop]
__global__ __launch_bounds__(256) void k_overlap_test(const float* __restrict__ in,
                                                       const float* __restrict__ win,
                                                       const float* __restrict__ back,
                                                       float* __restrict__ out, int n, int hop) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    float v = in[k] * win[k];
    v = v * win[k];
    if (k + hop < n) v += back[k + hop];
    out[k] = v;
}

hipError_t launch_overlap_test(const float* in, const float* win, const float* back, float* out,
                               int n, int hop, hipStream_t s) {
    hipLaunchKernelGGL(k_overlap_test, dim3((n + 255) / 256), dim3(256), 0, s, in, win, back, out, n, hop);
    return hipGetLastError();
}

// pv_set_window (REF_COMPAT): the caller's window becomes the analysis window and the
// synthesis gain win/N (kernel.cu:380 cudaDivVec then :406 cudaWindow; N is a power of two,
// so win * (1/N) is exactly win / N).
__global__ __launch_bounds__(256) void k_window_gain(const float* __restrict__ win, float* __restrict__ dwin,
                                                     float* __restrict__ gain, int n, float inv_n) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const float w = win[k];
    dwin[k] = w;
    gain[k] = w * inv_n;
}

hipError_t launch_window_gain(const float* win, float* dwin, float* gain, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_window_gain, dim3((n + 255) / 256), dim3(256), 0, s, win, dwin, gain, n, 1.0f / (float)n);
    return hipGetLastError();
}

// ------------------------------------------------------------------ launchers
template <int L>
static size_t syn_lds(int dt) {
    const int ring_floats = (dt > 0) ? 0 : 4 * 2 * L;               // ROLA: tails alias the tiles
    const int gain_floats = (dt > 0 && (L <= 512 || (L == 1024 && dt == 4))) ? 0 : 2 * L;  // syn_gains_in_regs
    return sizeof(float2) * (L + (L + 2) + 4 * Geo<L>::TILE) +
           sizeof(float) * (ring_floats + gain_floats) + sizeof(float) * 4 * (L + 1 + 3);
}

// register overlap-add slots per frame (out hop = 128 DT), 0 = LDS ring
static int syn_dt(int L, int hs) {
    if (L > 1024 || hs % 128 != 0) return 0;
    const int d = hs / 128;
    return (d == 1 || d == 2 || d == 4) ? d : 0;
}

size_t synthesis_lds_bytes(int L, int hs) {
    const int dt = syn_dt(L, hs);
    switch (L) {
        case 128: return syn_lds<128>(dt);
        case 256: return syn_lds<256>(dt);
        case 512: return syn_lds<512>(dt);
        case 1024: return syn_lds<1024>(dt);
        case 2048: return syn_lds<2048>(dt);
    }
    return 0;
}


hipError_t launch_runsum(int channels, const ScanParams& p, hipStream_t s) {
    dim3 grid((p.L + 1 + 255) / 256, p.nruns, channels);
    hipLaunchKernelGGL(k_runsum, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_segsum(const SegParams& p, hipStream_t s) {
    hipLaunchKernelGGL(k_segsum, dim3((p.L + 1 + 255) / 256, p.channels), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_segcarry(const SegParams& p, hipStream_t s) {
    hipLaunchKernelGGL(k_segcarry, dim3((p.bins_pad + 255) / 256, p.channels), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_carry(int channels, const ScanParams& p, hipStream_t s) {
    // segments per (channel, 64-bin block): enough waves to fill the chip when the batch
    // has few channels, few passes over the records when it has many
    dim3 grid((p.L + 1 + 63) / 64, channels);
    const long long blocks = (long long)grid.x * channels;
    if (blocks >= 2048 || p.nruns < 64) hipLaunchKernelGGL(k_carry<1>, grid, dim3(64), 0, s, p);
    else if (blocks >= 256) hipLaunchKernelGGL(k_carry<4>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_carry<16>, grid, dim3(1024), 0, s, p);
    return hipGetLastError();
}

// (A/B build: -DPV_SYN_FULLROWS reads whole rows for single-source pitch too)
#ifdef PV_SYN_FULLROWS
constexpr bool kSynFullRows = true;
#else
constexpr bool kSynFullRows = false;
#endif
// QPOW2 kernels (q a power of two <= 2^24: every STANDARD configuration with a power-of-two
// hop) for all overlap-add variants; the generic-q path uses the LDS ring (DT = 0).
template <int MODE, bool QP>
static hipError_t launch_synthesis_mode(int L, int dt, dim3 grid, const SynParams& p, hipStream_t s) {
#define PV_SYN_DT1(LL_, KL_)                                                                              \
    switch (dt) {                                                                                         \
        case 1: hipLaunchKernelGGL((k_synthesis<LL_, MODE, 1, QP, KL_>), grid, dim3(256), syn_lds<LL_>(1), s, p); break; \
        case 2: hipLaunchKernelGGL((k_synthesis<LL_, MODE, 2, QP, KL_>), grid, dim3(256), syn_lds<LL_>(2), s, p); break; \
        case 4:                                                                                           \
            if constexpr (MODE == 3 && LL_ == 1024 && KL_ && !kSynFullRows) {                            \
                /* single-source pitch (config 4): only the row slots of source bins <= src_hi */        \
                if (p.src_hi < 512) { hipLaunchKernelGGL((k_synthesis<LL_, MODE, 4, QP, KL_, 8>), grid, dim3(256), syn_lds<LL_>(4), s, p); break; } \
                if (p.src_hi < 768) { hipLaunchKernelGGL((k_synthesis<LL_, MODE, 4, QP, KL_, 12>), grid, dim3(256), syn_lds<LL_>(4), s, p); break; } \
            }                                                                                             \
            hipLaunchKernelGGL((k_synthesis<LL_, MODE, 4, QP, KL_>), grid, dim3(256), syn_lds<LL_>(4), s, p); break; \
        default: hipLaunchKernelGGL((k_synthesis<LL_, MODE, 0, QP>), grid, dim3(256), syn_lds<LL_>(0), s, p); break; \
    }
    // per-lane unwrap constants: register overlap-add STANDARD kernels (QP, MODE != 1)
#define PV_SYN_DT(LL_)                                        \
    if (QP && MODE != 1 && p.k_lane) { PV_SYN_DT1(LL_, (QP && MODE != 1)) } \
    else { PV_SYN_DT1(LL_, false) }
#define PV_SYN_DT0(LL_) hipLaunchKernelGGL((k_synthesis<LL_, MODE, 0, QP>), grid, dim3(256), syn_lds<LL_>(0), s, p)
    if constexpr (QP || MODE == 1) {
        switch (L) {
            case 128: PV_SYN_DT(128); break;
            case 256: PV_SYN_DT(256); break;
            case 512: PV_SYN_DT(512); break;
            case 1024: PV_SYN_DT(1024); break;
            case 2048: PV_SYN_DT0(2048); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (L) {
            case 128: PV_SYN_DT0(128); break;
            case 256: PV_SYN_DT0(256); break;
            case 512: PV_SYN_DT0(512); break;
            case 1024: PV_SYN_DT0(1024); break;
            case 2048: PV_SYN_DT0(2048); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef PV_SYN_DT
#undef PV_SYN_DT1
#undef PV_SYN_DT0
    return hipGetLastError();
}

// the QPOW2 kernels carry the output phase in the revolution accumulator (RACC), exact for
// power-of-two q <= 4096
bool synthesis_lane_kernel(int L, int mode, int hs, bool q_pow2, unsigned long long q) {
    const bool qp = q_pow2 && q <= 4096ull;
    return mode != 1 && qp && syn_dt(L, hs) != 0;
}

// mode: 0 STANDARD stretch, 2 STANDARD pitch, 1 REF_COMPAT (the kernels' MODE 3: pitch >= 1)
hipError_t launch_synthesis(int L, int mode, int channels, const SynParams& p, hipStream_t s) {
    dim3 grid((p.nruns + 3) / 4, channels);
    const bool qp = p.q_pow2 && p.q <= 4096ull;
    const int dt = (mode == 1 || qp) ? syn_dt(L, p.hs) : 0;
    if (mode == 0) return qp ? launch_synthesis_mode<0, true>(L, dt, grid, p, s)
                             : launch_synthesis_mode<0, false>(L, dt, grid, p, s);
    // pitch ratio >= 1: at most one source per bin, the gather fixed at compile time (MODE 3:
    // the per-bin source-count loops of ratios < 1 are not in the frame loop; config 4)
    if (mode == 2 && p.rho >= 1.0f) return qp ? launch_synthesis_mode<3, true>(L, dt, grid, p, s)
                                              : launch_synthesis_mode<3, false>(L, dt, grid, p, s);
    if (mode == 2) return qp ? launch_synthesis_mode<2, true>(L, dt, grid, p, s)
                             : launch_synthesis_mode<2, false>(L, dt, grid, p, s);
    return launch_synthesis_mode<1, false>(L, dt, grid, p, s);
}

hipError_t launch_seam(int channels, const SeamParams& p, hipStream_t s) {
    dim3 grid((p.tail_len + 255) / 256, p.nwg, channels);
    hipLaunchKernelGGL(k_seam, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace pv
