// pv_analysis.hip — K1, the analysis kernels (STANDARD and REF_COMPAT), gfx950.
//
// Its own translation unit, compiled without SLP vectorisation (the per-run body is in
// pv_ana_run.hpp; the synthesis, whose packed code is hand-written, is faster with SLP on).
// Pipeline and geometry: pv_kernels.hip header, DESIGN.md §4.
#include "pv_ana_run.hpp"

namespace pv {

// ------------------------------------------------------------------ K1 STANDARD
// One wave = one run of F consecutive frames.  The unwrap decision m(t) = f(phi[t],
// phi[t-1]) is accumulated in registers: S = sum over t in (t0, t0+F), phi(t0) and phi of the
// run's last frame go to the run record (k_carry makes m(t0) from them and the previous run's
// record).
// EKL: the expected advance e_k from an LDS table; otherwise (64 a multiple of the hop
// divisor, so e_k depends on k mod 64 only) one register per lane, e_k = ek[lane].
// waves per SIMD the analysis is compiled for (__launch_bounds__): L = 512 at <= 128 VGPRs
// (112 used with the 4-frame register rotation of ana_run; at 5 waves it spills), L = 1024
// at <= 168 (LDS with the twiddle sharing allows 3 workgroups per CU)
constexpr int kAnaWaves512 = 4;
constexpr int kAnaWaves1024 = 3;
// D > 0: hop = 128 D samples, so frame u+1's register q is frame u's register q + D and a
// frame costs only its D new sample pairs per lane (the other E - D are shifted in
// registers): 1/E of the frame's bytes leave L2 instead of all of them.
// PACKED: the pv.h PV_SPEC_PACKED row layout (bin L folded into slot 0).
// (Round 5 measured an LDS-DMA input ring R frames ahead in larger workgroups: no gain,
// profiles/r05_ab_ring.json; the code is kept out of the product as scripts/r05_ana_ring.patch.)
constexpr int kAnaWG = 4;  // waves (runs) per workgroup

// NA: lane registers analysed (Geo<L>::E = all; fewer: bins >= 64 NA not analysed and their
// row slots not written — pv_process without a spectrum output, ana_run; the synthesis
// reads only the written slots, k_synthesis NR)
template <int L, bool EKL, int D, bool PACKED, int NA = Geo<L>::E>
__global__ __launch_bounds__(64 * kAnaWG, (L < 512) ? 4 : (L == 512) ? kAnaWaves512 : (L == 1024) ? kAnaWaves1024 : 1) void k_std_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    constexpr int B = L + 1;
    constexpr int W = kAnaWG;
    constexpr int NT = 64 * W;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int TWN = ana_twl_n<L>();
    float2* twl = reinterpret_cast<float2*>(smem);    // TWN stage-major twiddles (L, or L/4)
    float2* twsl = twl + TWN;                         // L+1 split twiddles (+1 pad)
    float2* tiles = twsl + (L + 2);                   // W x TILE
    float* winl = reinterpret_cast<float*>(tiles + W * G_::TILE);  // N
    float* ekl = winl + N;                            // B

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[Geo<L>::E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < TWN; i += NT) twl[i] = p.tw[i];
    for (int i = tid; i < B; i += NT) {
        twsl[i] = p.tws[i];
        if (EKL) ekl[i] = p.ek[i];
    }
    const float e_lane = EKL ? 0.0f : p.ek[tid & 63];
    for (int i = tid; i < N; i += NT) winl[i] = p.win[i];
    __syncthreads();
    const int run = blockIdx.x * W + w, c = blockIdx.y;
    if (run >= p.nruns) return;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    // run record {S, phi(t0), phi(last)}: phi(t0) is stored as soon as it is known, the rest
    // after the loop
    int* rec = (p.runsum != nullptr) ? p.runsum + ((long long)c * p.nruns + run) * kRecFields * p.bins_pad : nullptr;
    float phprev[E + 1];
    ana_acc_t<L> sacc[E + 1];
    ana_run<L, EKL, D, PACKED, NA>(p, AnaLds{twl, twsl, winl, ekl}, tiles + w * G_::TILE, tw0, lane, c, t0, nfr, e_lane,
                                   rec, phprev, sacc);
}

// ------------------------------------------------------------------ K1 REF_COMPAT
// kernel.cu:299-348: window (Hamming), zero-phase shift + zero pad to 2N, C2C 2N,
// (|X|, atanf(Im/Re)) for all 2N bins.  The 2N-point transform of the real padded frame
// is an L = N point complex FFT + real split (bins 0 .. N); bins N+1 .. 2N-1 are the
// conjugates of bins N-1 .. 1 (real input), i.e. the same magnitude and the negated phase.
//
// Geometry as K1 STANDARD: a wave walks a run of F frames, 4 runs per workgroup, no halo
// (no unwrap).  Input: of the 2N padded samples only z[n] = (b[2n], b[2n+1]) with
// n < N/4 (frame samples N/2 .. N-1) and n >= 3N/4 (frame samples 0 .. N/2-1) are nonzero,
// so a lane's registers q < E/4 and q >= 3E/4 hold the frame's N samples (one contiguous
// vector load of E/2 pairs, prefetched one frame ahead, kernel.cu:25-32's shift folded
// into the register order) and the E/2 middle registers are compile-time zeros.
// Output: every row store is a whole 512-byte block.  Block i < E holds bins 64 i + lane
// (this lane's bins); mirror block j holds indices N + 64 j + lane = bins N - 64 j - lane,
// which lane (64 - lane) & 63 holds in register E - j - 1 (lane 0: its own register E - j,
// bin N itself for j = 0): a ds_bpermute lane reversal, as split_chunk_bp's partner read.
// Phase: atanf(y/x) without the division (atan_ratio_pv2); magnitude: hardware sqrt.
template <int L>
__global__ __launch_bounds__(256) void k_compat_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = L;          // window length
    constexpr int QA = E / 4;     // registers 0 .. QA-1 and E-QA .. E-1 carry samples
    constexpr int NST = 2 * E;    // row stores per frame (E blocks + E mirror blocks)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int TWN = ana_twl_n<L>();
    float2* twl = reinterpret_cast<float2*>(smem);  // TWN stage-major twiddles
    float2* twsl = twl + TWN;                        // L+1 split twiddles (+1 pad)
    float2* tiles = twsl + (L + 2);                  // 4 x TILE
    float* winl = reinterpret_cast<float*>(tiles + 4 * G_::TILE);  // N window samples

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[Geo<L>::E];
    load_tw0<L>(tw0, p.tw);
    for (int i = tid; i < TWN; i += 256) twl[i] = p.tw[i];
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
    const float2* w2 = reinterpret_cast<const float2*>(winl);
    const int rev = ((64 - lane) & 63) << 2;

    // frame samples 2 lane + 128 m + {0,1} (m < E/2) -> register q(m): m >= E/4 (samples
    // N/2 ..) to q = m - E/4, m < E/4 (samples 0 .. N/2-1) to q = 3E/4 + m; x (window)
    auto window = [&](const float2 (&xs)[E / 2], float2 (&z)[E]) {
#pragma unroll
        for (int m = 0; m < E / 2; ++m) {
            const int q = (m >= QA) ? m - QA : E - QA + m;
            const float2 wv = lds_ld(&w2[lane + 64 * m]);
            z[q] = make_float2(xs[m].x * wv.x, xs[m].y * wv.y);
        }
#pragma unroll
        for (int q = QA; q < E - QA; ++q) z[q] = make_float2(0.0f, 0.0f);
    };
    auto frame = [&](int u, float2 (&z)[E]) {
        float2* srow = specc + (long long)(t0 + u) * p.spec_stride;
        fft_run<L, false, false, 0, ana_tws_min<L>()>(z, tile, twl, tw0, lane, twsl);
        float pm = 0.0f, pp = 0.0f;  // the previous bin's {mag, phase} (mirror source)
        static_for<0, (E + 2) / 2>([&](auto ic) {
            constexpr int i0 = 2 * decltype(ic)::value;
            float2 X[2];
            split_chunk_bp<L, 2, true, i0>(z, twsl, lane, X);  // 2X (TWICE): scale-free phase
            const f2v ph2 = atan_ratio_pv2(X[0].y, X[0].x, X[1].y, X[1].x);
            static_for<0, 2>([&](auto cc) {
                constexpr int c2 = decltype(cc)::value;
                constexpr int i = i0 + c2;
                if constexpr (i <= E) {
                    const float mag = 0.5f * __builtin_amdgcn_sqrtf(__builtin_fmaf(X[c2].x, X[c2].x, X[c2].y * X[c2].y));
                    float ph = (c2 == 0) ? ph2.x : ph2.y;
                    // atanf(0/0) = NaN of an all-zero bin (digital silence) when asked
                    if (p.nan_faithful && X[c2].x == 0.0f && X[c2].y == 0.0f) ph = __builtin_nanf("");
                    if constexpr (i < E)
                        __builtin_nontemporal_store(f2v{mag, ph}, reinterpret_cast<f2v*>(&srow[64 * i + lane]));
                    if constexpr (i >= 1) {
                        // mirror block j = E - i: lane 0 sends bin 64 i (its register i), the
                        // other lanes bin 64 (i - 1) + lane (register i - 1) to lane 64 - lane
                        const float sm = (lane == 0) ? mag : pm;
                        const float sp = (lane == 0) ? ph : pp;
                        const float mm = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(sm)));
                        float mp = __int_as_float(__builtin_amdgcn_ds_bpermute(rev, __float_as_int(sp)));
                        if (!(i == E && lane == 0)) mp = -mp;  // conjugate; bin N is itself
                        __builtin_nontemporal_store(f2v{mm, mp}, reinterpret_cast<f2v*>(&srow[N + 64 * (E - i) + lane]));
                    }
                    pm = mag;
                    pp = ph;
                }
            });
        });
        wave_lds_sync();  // tile reads done before the next frame's pass_store
    };
    auto load_checked = [&](int u, float2 (&xs)[E / 2]) {
        const long long base = (long long)(t0 + u) * p.hop;
#pragma unroll
        for (int m = 0; m < E / 2; ++m) {
            const long long sidx = base + 2 * (lane + 64 * m);
            xs[m].x = (sidx < p.n) ? xc[sidx] : 0.0f;
            xs[m].y = (sidx + 1 < p.n) ? xc[sidx + 1] : 0.0f;
        }
    };
    // frames whose N samples lie inside [0, n) (and 8-byte aligned) take vector loads
    const long long lastfull = (p.aligned && p.n >= N) ? (p.n - N) / p.hop : -1;
    const int ufast = (int)min((long long)nfr, max(0LL, lastfull - t0 + 1));
    if constexpr (NST <= 63) {  // vmcnt holds 6 bits: the self-tracked prefetch (L <= 1024)
        if (ufast > 0) {
            float2 z[E];
            {
                f2v xv[E / 2];
                gload_pairs<E / 2>(xv, xc + (long long)t0 * p.hop + 2 * lane);
                vm_wait<0>(xv);
                float2 xs[E / 2];
#pragma unroll
                for (int m = 0; m < E / 2; ++m) xs[m] = make_float2(xv[m].x, xv[m].y);
                window(xs, z);
            }
            for (int u = 0; u < ufast; ++u) {
                f2v xv[E / 2];  // frame u+1 (clamped), in flight during frame u
                gload_pairs<E / 2>(xv, xc + (long long)(t0 + min(u + 1, ufast - 1)) * p.hop + 2 * lane);
                frame(u, z);  // exactly NST row stores
                vm_wait<NST>(xv);
                float2 xs[E / 2];
#pragma unroll
                for (int m = 0; m < E / 2; ++m) xs[m] = make_float2(xv[m].x, xv[m].y);
                window(xs, z);
            }
        }
    } else if (ufast > 0) {  // L = 2048: compiler-tracked prefetch
        float2 xs[E / 2];
        const float* src0 = xc + (long long)t0 * p.hop + 2 * lane;
#pragma unroll
        for (int m = 0; m < E / 2; ++m) xs[m] = *reinterpret_cast<const float2*>(src0 + 128 * m);
        for (int u = 0; u < ufast; ++u) {
            float2 z[E];
            window(xs, z);
            const float* src = xc + (long long)(t0 + min(u + 1, ufast - 1)) * p.hop + 2 * lane;
#pragma unroll
            for (int m = 0; m < E / 2; ++m) xs[m] = *reinterpret_cast<const float2*>(src + 128 * m);
            frame(u, z);
        }
    }
    for (int u = ufast; u < nfr; ++u) {
        float2 xs[E / 2], z[E];
        load_checked(u, xs);
        window(xs, z);
        frame(u, z);
    }
}


// ------------------------------------------------------------------ launchers
template <int L>
static size_t ana_lds_std(bool ekl) {
    return sizeof(float2) * (ana_twl_n<L>() + (L + 2) + kAnaWG * Geo<L>::TILE) + sizeof(float) * (2 * L + (ekl ? L + 1 : 0));
}
template <int L>
static size_t ana_lds_compat() {
    return sizeof(float2) * (ana_twl_n<L>() + (L + 2) + 4 * Geo<L>::TILE) + sizeof(float) * L;
}
// twiddles + 4 tiles + 4 rings (tails) [+ gain] + ek/jk + pitch map; with register
// overlap-add at L <= 512 the gains live in registers and gainl is not allocated

#define PV_DISPATCH_L(L_, ...)                        \
    switch (L_) {                                     \
        case 128: { constexpr int LL = 128; __VA_ARGS__; } break;   \
        case 256: { constexpr int LL = 256; __VA_ARGS__; } break;   \
        case 512: { constexpr int LL = 512; __VA_ARGS__; } break;   \
        case 1024: { constexpr int LL = 1024; __VA_ARGS__; } break; \
        case 2048: { constexpr int LL = 2048; __VA_ARGS__; } break; \
        default: return hipErrorInvalidValue;         \
    }

template <bool PK>
static hipError_t launch_std_analysis_t(int L, dim3 grid, const AnaParams& p, hipStream_t s) {
    PV_DISPATCH_L(L, {
        // shifted-register input when hop = 128 D (D < E)
        const int d = (p.aligned && p.hop % 128 == 0) ? p.hop / 128 : 0;
        if (p.ek_lane && LL >= 256 && LL <= 1024 && (d == 1 || d == 2 || d == 4) && d < LL / 64) {
            constexpr int E_ = LL / 64;  // D < E (instantiated for every L, run for the checked ones)
            constexpr int D1 = (1 < E_) ? 1 : 0, D2 = (2 < E_) ? 2 : 0, D4 = (4 < E_) ? 4 : 0;
            const size_t lds = ana_lds_std<LL>(false);
            auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(64 * kAnaWG), lds, s, p); };
            if (d == 1) go(k_std_analysis<LL, false, D1, PK>);
            else if (d == 2) go(k_std_analysis<LL, false, D2, PK>);
            else if (LL == 1024 && PK && p.src_hi < LL) {
                // bins above src_hi unread (config 4, pitch 1.5: 684 .. 1024): the registers
                // analysed, in whole chunks of kAnaChunk
                const int na = kAnaChunk * ((p.src_hi + 64 * kAnaChunk) / (64 * kAnaChunk));
                if (na <= 8) go(k_std_analysis<LL, false, D4, PK, (8 < E_ ? 8 : E_)>);
                else if (na <= 10) go(k_std_analysis<LL, false, D4, PK, (10 < E_ ? 10 : E_)>);
                else if (na <= 12) go(k_std_analysis<LL, false, D4, PK, (12 < E_ ? 12 : E_)>);
                else if (na <= 14) go(k_std_analysis<LL, false, D4, PK, (14 < E_ ? 14 : E_)>);
                else go(k_std_analysis<LL, false, D4, PK>);
            } else go(k_std_analysis<LL, false, D4, PK>);
        } else if (p.ek_lane) hipLaunchKernelGGL((k_std_analysis<LL, false, 0, PK>), grid, dim3(256), ana_lds_std<LL>(false), s, p);
        else hipLaunchKernelGGL((k_std_analysis<LL, true, 0, PK>), grid, dim3(256), ana_lds_std<LL>(true), s, p);
    });
    return hipGetLastError();
}

// workgroups of the STANDARD analysis kernel launch_std_analysis picks for an aligned input
// (hop = 128 d when that divides) that one CU holds at once (0 if the runtime cannot say),
// and its waves per workgroup
template <bool PK>
static int std_analysis_wgs_per_cu_t(int L, int hop, bool ek_lane, int* waves_per_wg) {
    int n = 0;
    *waves_per_wg = 4;
    if (L != 128 && L != 256 && L != 512 && L != 1024 && L != 2048) return 0;
        auto occ = [&](const void* k, int W, size_t lds) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64 * W, lds) != hipSuccess) n = 0;
        *waves_per_wg = W;
    };
    PV_DISPATCH_L(L, {
        const int d = (hop % 128 == 0) ? hop / 128 : 0;
        if (ek_lane && LL >= 256 && LL <= 1024 && (d == 1 || d == 2 || d == 4) && d < LL / 64) {
            constexpr int E_ = LL / 64;
            constexpr int D1 = (1 < E_) ? 1 : 0, D2 = (2 < E_) ? 2 : 0, D4 = (4 < E_) ? 4 : 0;
            if (d == 1) occ((const void*)k_std_analysis<LL, false, D1, PK>, kAnaWG, ana_lds_std<LL>(false));
            else if (d == 2) occ((const void*)k_std_analysis<LL, false, D2, PK>, kAnaWG, ana_lds_std<LL>(false));
            else occ((const void*)k_std_analysis<LL, false, D4, PK>, kAnaWG, ana_lds_std<LL>(false));
        } else if (ek_lane) occ((const void*)k_std_analysis<LL, false, 0, PK>, 4, ana_lds_std<LL>(false));
        else occ((const void*)k_std_analysis<LL, true, 0, PK>, 4, ana_lds_std<LL>(true));
    });
    return n;
}
int std_analysis_wgs_per_cu(int L, int hop, bool ek_lane, bool packed, int* waves_per_wg) {
    return packed ? std_analysis_wgs_per_cu_t<true>(L, hop, ek_lane, waves_per_wg)
                  : std_analysis_wgs_per_cu_t<false>(L, hop, ek_lane, waves_per_wg);
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
