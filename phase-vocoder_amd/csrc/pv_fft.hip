// pv_fft.hip — the standalone batched complex FFT op: the
// reference's hand-written radix-2 Stockham FFT, FFT::HPFFT::computeGPUFFT /
// computeGPUIFFT (karnel/hpfft.h:6-11, hpfft.cu:145-203), one launch for a whole batch.
//
// The reference runs log2(N) single-block launches per transform (GPU_FFT, one radix-2
// stage each, ping-ponging through global memory).  Here:
//   N in [128, 1024]: one transform per wavefront, the register-blocked Stockham engine of
//     the phase-vocoder kernels (fft_run, pv_device.hpp): the same radix-2 butterflies
//     with table twiddles, log2(N/64) stages per register pass, an LDS exchange per pass.
//   N = 2048: the same passes over two waves per transform (k_fft2w).
//   N = 32, 64 (round 5): T = N/8 lanes per transform, 8 points per lane — a radix-8 DIF
//     in each lane over its points t + T p, the W_N^{t k1} twiddles, an 8 x T transpose
//     through LDS within the wave, T-point DIFs, and T-lane-contiguous loads and stores
//     (k_fft_t8: the one-transform-per-lane form needs 2N VGPRs and strided accesses);
//   N in [2, 16]: one transform per LANE, every stage in registers (k_fft_reg); the
//     per-stage LDS form (the reference's FftIteration in LDS, one transform per wave)
//     remains for buffers that are not 16-byte aligned.
// Unnormalised in both directions, like the reference (GPU_FFT applies no 1/N).
#include "pv_device.hpp"
#include "pv_kernels.h"


namespace pv {

template <int L, bool INV>
__global__ __launch_bounds__(256) void k_fft(const float2* __restrict__ in, float2* out,
                                              const float2* __restrict__ tw, int batch) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);
    float2* tiles = twl + L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    float2 tw0[E];
    load_tw0<L>(tw0, tw);
    for (int i = tid; i < L; i += 256) twl[i] = tw[i];
    __syncthreads();
    const long long b = (long long)blockIdx.x * 4 + w;
    if (b >= batch) return;
    float2* tile = tiles + w * G_::TILE;
    const float2* src = in + b * L + lane;
    float2 z[E];
#pragma unroll
    for (int q = 0; q < E; ++q) z[q] = src[64 * q];
    fft_run<L, INV>(z, tile, twl, tw0, lane);
    // all loads of this transform precede every store: in-place (in == out) is safe
    float2* dst = out + b * L + lane;
#pragma unroll
    for (int q = 0; q < E; ++q) dst[64 * q] = lds_ld(&tile[G_::pad(lane + 64 * q)]);
}

// N <= 64: lanes j < N/2 run butterfly j of each radix-2 Stockham stage (hpfft.cu:145-167):
// v0 = x[j], v1 = x[j + N/2] * W(j mod Ns, Ns); y[expand(j,Ns,2)] = v0 + v1,
// y[expand(j,Ns,2) + Ns] = v0 - v1.  Twiddle W(m, Ns) = stage-major table entry Ns-1+m.
template <bool INV>
__global__ __launch_bounds__(256) void k_fft_small(const float2* __restrict__ in, float2* out,
                                                    const float2* __restrict__ tw, int n, int batch) {
    __shared__ float2 buf[4][2][64];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR arithmetic
    const long long b = (long long)blockIdx.x * 4 + w;
    if (b >= batch) return;
    float2* x = buf[w][0];
    float2* y = buf[w][1];
    if (lane < n) x[lane] = in[b * n + lane];
    wave_lds_sync();
    const int h = n >> 1;
    for (int Ns = 1; Ns < n; Ns <<= 1) {
        if (lane < h) {
            const float2 v0 = x[lane];
            float2 v1 = x[lane + h];
            const int m = lane & (Ns - 1);
            float2 t = tw[Ns - 1 + m];
            if (INV) t.y = -t.y;
            v1 = cmul(v1, t);
            const int d = (lane / Ns) * 2 * Ns + m;  // expand(j, Ns, 2)
            y[d] = make_float2(v0.x + v1.x, v0.y + v1.y);
            y[d + Ns] = make_float2(v0.x - v1.x, v0.y - v1.y);
        }
        wave_lds_sync();
        float2* t2 = x;
        x = y;
        y = t2;
    }
    if (lane < n) out[b * n + lane] = x[lane];
}

// N <= 64, register form: one transform per LANE, all log2 N radix-2 Stockham stages in
// registers with compile-time indices (the twiddle of every butterfly is a wave-uniform
// table entry -> scalar loads), W = 1 / exactly -i in the first two stages as in the
// register-blocked engine; 16-byte loads and stores of the lane's contiguous transform.
// N = 8, 16: the lane's transform is N/2 16-byte pieces N * 8 bytes apart from its
// neighbour lanes', so every load instruction of a wave spans 64 separate pieces; the block's
// 256 transforms (one contiguous stretch of 256 N points) are instead moved with wave-
// contiguous 16-byte loads / stores staged through LDS (rows of N/2 + 1 pieces: the pad
// spreads the lanes' row reads over the banks).
template <int N, bool INV>
__global__ __launch_bounds__(256) void k_fft_reg(const float2* __restrict__ in, float2* out,
                                                  const float2* __restrict__ tw, int batch) {
    constexpr bool STAGE = (N == 8 || N == 16);  // (N = 4 staged: 5.63 -> 5.62 TB/s, not kept)
    constexpr int H = N / 2, ROW = H + 1;  // 16-byte pieces per transform, LDS row length
    __shared__ float4 st[STAGE ? 256 * ROW : 1];
    const long long b0 = (long long)blockIdx.x * 256;
    const long long b = b0 + threadIdx.x;
    const int nv = (int)min(256LL, (long long)batch - b0);  // transforms of this block
    f2v x[N];
    if constexpr (STAGE) {
        const float4* src = reinterpret_cast<const float4*>(in + b0 * N);
#pragma unroll
        for (int q = 0; q < H; ++q) {
            const int e = threadIdx.x + 256 * q;  // piece e of the block: transform e / H
            if (e < nv * H) st[(e / H) * ROW + e % H] = src[e];
        }
        __syncthreads();
        if (b < batch) {
#pragma unroll
            for (int q = 0; q < H; ++q) {
                const float4 v = st[threadIdx.x * ROW + q];
                x[2 * q] = f2v{v.x, v.y};
                x[2 * q + 1] = f2v{v.z, v.w};
            }
        }
    } else {
    if (b >= batch) return;
    if constexpr (N == 2) {
        const float2 a0 = in[b * 2], a1 = in[b * 2 + 1];
        x[0] = f2v{a0.x, a0.y};
        x[1] = f2v{a1.x, a1.y};
    } else {
        const float4* src = reinterpret_cast<const float4*>(in + b * N);
#pragma unroll
        for (int q = 0; q < N / 2; ++q) {
            const float4 v = src[q];
            x[2 * q] = f2v{v.x, v.y};
            x[2 * q + 1] = f2v{v.z, v.w};
        }
    }
    }  // !STAGE
#pragma unroll
    for (int Ns = 1; Ns < N; Ns <<= 1) {
        f2v y[N];
#pragma unroll
        for (int j = 0; j < N / 2; ++j) {
            const int m = j & (Ns - 1);
            const f2v v0 = x[j], v1 = x[j + N / 2];
            const int d = (j / Ns) * 2 * Ns + m;  // expand(j, Ns, 2)
            if (Ns == 2 && m == 1) {              // W = exactly -i (+i when INV)
                y[d] = pk_add_swp<INV>(v0, v1);
                y[d + Ns] = pk_add_swp<!INV>(v0, v1);
                continue;
            }
            f2v t;
            if (Ns <= 2) {
                t = v1;  // W = 1
            } else {
                const float2 w = tw[Ns - 1 + m];
                t = cmul_v<INV, true>(v1, f2v{w.x, w.y});
            }
            y[d] = v0 + t;
            y[d + Ns] = v0 - t;
        }
#pragma unroll
        for (int q = 0; q < N; ++q) x[q] = y[q];
    }
    if constexpr (STAGE) {
        // every thread's own row only: the barrier orders the block's reads above before
        // any store below (in-place use is safe)
#pragma unroll
        for (int q = 0; q < H; ++q) st[threadIdx.x * ROW + q] = make_float4(x[2 * q].x, x[2 * q].y, x[2 * q + 1].x, x[2 * q + 1].y);
        __syncthreads();
        float4* dst = reinterpret_cast<float4*>(out + b0 * N);
#pragma unroll
        for (int q = 0; q < H; ++q) {
            const int e = threadIdx.x + 256 * q;
            if (e < nv * H) dst[e] = st[(e / H) * ROW + e % H];
        }
    } else if constexpr (N == 2) {
        out[b * 2] = make_float2(x[0].x, x[0].y);
        out[b * 2 + 1] = make_float2(x[1].x, x[1].y);
    } else {
        float4* dst = reinterpret_cast<float4*>(out + b * N);
#pragma unroll
        for (int q = 0; q < N / 2; ++q) dst[q] = make_float4(x[2 * q].x, x[2 * q].y, x[2 * q + 1].x, x[2 * q + 1].y);
    }
}


// N = 8 T (T = 4, 8): T lanes per transform, 8 points per lane, 64 / T transforms per wave.
// x[t + T p] -> lane t, point p.  X[k1 + 8 k2] = sum_t W_T^{t k2} W_N^{t k1} (sum_p W_8^{p k1}
// x[t + T p]): the inner 8-point DFT in the lane (dif_v3<8>: output bit-reversed), the
// twiddle (table tw of the radix-2 stages: W_N^e = tw[N/2 - 1 + e] for e < N/2, its negative
// above), the transpose through LDS (rows of T + 1 float2, wave-local: no barrier), and
// 8 / T T-point DFTs per lane (columns k1 = t + T j).  Unnormalised, conj twiddles for INV.
template <int N, bool INV>
__global__ __launch_bounds__(256) void k_fft_t8(const float2* __restrict__ in, float2* out,
                                                const float2* __restrict__ tw, int batch) {
    constexpr int T = N / 8, P = 8, NT = 256 / T, ROW = T + 1, J = P / T;
    static_assert(T == 4 || T == 8, "N = 32 or 64");
    __shared__ float2 xs[NT * P * ROW];
    __shared__ float2 twl[N / 2];
    const int tid = threadIdx.x;
    const int g = tid / T, t = tid % T;
    const long long b = (long long)blockIdx.x * NT + g;
    const bool live = b < batch;
    if (tid < N / 2) twl[tid] = tw[N / 2 - 1 + tid];
    f2v a[P];
    if (live) {
        const float2* src = in + b * N + t;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const float2 v = src[T * p];
            a[p] = f2v{v.x, v.y};
        }
    } else {
#pragma unroll
        for (int p = 0; p < P; ++p) a[p] = f2v{0.0f, 0.0f};
    }
    __syncthreads();  // twl
    dif_v3<P, INV>(a);  // a[bitrev3(k1)] = inner DFT k1
    float2* row = xs + g * P * ROW;
#pragma unroll
    for (int k1 = 0; k1 < P; ++k1) {
        f2v v = a[bitrevc(k1, 3)];
        if (k1 > 0) {
            const int e = t * k1;  // < N
            const float2 w = lds_ld(&twl[e & (N / 2 - 1)]);
            const f2v wv = (e & (N / 2)) ? f2v{-w.x, -w.y} : f2v{w.x, w.y};
            v = cmul_v<INV>(v, wv);
        }
        row[k1 * ROW + t] = make_float2(v.x, v.y);
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int k1 = t + T * j;
        f2v c[T];
#pragma unroll
        for (int s2 = 0; s2 < T; ++s2) {
            const float2 v = lds_ld(&row[k1 * ROW + s2]);
            c[s2] = f2v{v.x, v.y};
        }
        dif_v3<T, INV>(c);  // c[bitrev(k2)] = X[k1 + 8 k2]
        if (live) {
#pragma unroll
            for (int k2 = 0; k2 < T; ++k2) {
                const f2v v = c[bitrevc(k2, ilog2c(T))];
                out[b * N + k1 + P * k2] = make_float2(v.x, v.y);
            }
        }
    }
}

// N = 2048: two waves per transform (128 "lanes" x E = 16 points: the register budget of the
// N = 1024 kernel, which one wave holding 32 points per lane does not have — that form ran
// at 1 wave/SIMD, 3.5 TB/s).  Radix-16, 16, 8 Stockham passes, each pass's radix-2 stages in
// registers exactly as fft_pass (stage-major table twiddles W(m, Ns) = tw[Ns - 1 + m], W = 1 /
// -i in the first two stages), exchanges through one padded LDS tile per transform with a
// workgroup barrier (the two waves of a transform), the last pass's outputs stored straight
// from registers (for a fixed register they are 128 consecutive points: coalesced).
// A workgroup = 2 transforms x 2 waves.
constexpr int kF2L = 2048, kF2NL = 128, kF2E = kF2L / kF2NL;
__host__ __device__ constexpr int f2w_slot(int p) { return p + (p >> 4); }  // 1 pad per 16 points
constexpr int kF2Tile = f2w_slot(kF2L - 1) + 1;

template <int P, bool INV>
__device__ __forceinline__ void fft2w_pass(f2v (&a)[kF2E], const float2* tw, const float2 (&tw0)[16], int vl) {
    constexpr int L = kF2L, NL = kF2NL, E = kF2E;
    constexpr int S = 1 << (4 * P);
    constexpr int r = cmin(4, ilog2c(L) - 4 * P);
    constexpr int R = 1 << r;
    constexpr int NG = E / R;
#pragma unroll
    for (int st = 0; st < r; ++st) {
        const int Ns = S << st;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int jm = (vl + NL * g) & (S - 1);
            f2v b[R];
#pragma unroll
            for (int sb = 0; sb < R / 2; ++sb) {
                const int br = bitrevc(sb & ((1 << st) - 1), st);
                const f2v top = a[g * R + sb];
                const f2v bot = a[g * R + sb + R / 2];
                if (P == 0 && Ns == 2 && br != 0) {  // W = exactly -i (+i when INV)
                    b[2 * sb] = pk_add_swp<INV>(top, bot);
                    b[2 * sb + 1] = pk_add_swp<!INV>(top, bot);
                    continue;
                }
                f2v t;
                if (Ns == 1 || (P == 0 && Ns == 2)) {
                    t = bot;
                } else if constexpr (P == 0) {
                    const float2 w = tw0[(Ns - 1) + br];
                    t = cmul_v<INV, true>(bot, f2v{w.x, w.y});
                } else if constexpr (P == 1) {
                    const float2 w = lds_ld(&tw[(Ns - 1) + jm + S * br]);
                    t = cmul_v<INV, false>(bot, f2v{w.x, w.y});
                } else {  // pass 2: from the global table (L2), see k_fft2w
                    const float2 w = tw[(Ns - 1) + jm + S * br];
                    t = cmul_v<INV, false>(bot, f2v{w.x, w.y});
                }
                b[2 * sb] = top + t;
                b[2 * sb + 1] = top - t;
            }
#pragma unroll
            for (int q = 0; q < R; ++q) a[g * R + q] = b[q];
        }
    }
}

template <int P>
__device__ __forceinline__ void fft2w_store(const f2v (&a)[kF2E], float2* tile, int vl) {
    constexpr int L = kF2L, NL = kF2NL, E = kF2E;
    constexpr int S = 1 << (4 * P);
    constexpr int r = cmin(4, ilog2c(L) - 4 * P);
    constexpr int R = 1 << r;
#pragma unroll
    for (int g = 0; g < E / R; ++g) {
        const int j = vl + NL * g;
        const int J = (j / S) * R * S + (j & (S - 1));
#pragma unroll
        for (int f = 0; f < R; ++f) tile[f2w_slot(J + S * bitrevc(f, r))] = make_float2(a[g * R + f].x, a[g * R + f].y);
    }
}

template <int P>
__device__ __forceinline__ void fft2w_load(f2v (&a)[kF2E], const float2* tile, int vl) {
    constexpr int L = kF2L, NL = kF2NL, E = kF2E;
    constexpr int r = cmin(4, ilog2c(L) - 4 * P);
    constexpr int R = 1 << r;
#pragma unroll
    for (int g = 0; g < E / R; ++g)
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float2 v = lds_ld(&tile[f2w_slot(vl + NL * g + q * (L / R))]);
            a[g * R + q] = f2v{v.x, v.y};
        }
}

template <bool INV>
__global__ __launch_bounds__(256) void k_fft2w(const float2* __restrict__ in, float2* out,
                                                const float2* __restrict__ tw, int batch) {
    constexpr int L = kF2L, NL = kF2NL, E = kF2E;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // LDS: the stage-major entries of pass 1 (stages Ns = 16 .. 128: entries < 256) and one
    // tile per transform; pass 2's twiddles (Ns = 256 .. 1024) come from the global table
    // (L2-resident) so that 4 workgroups fit a CU (with the whole table in LDS: 3)
    float2* twl = reinterpret_cast<float2*>(smem);  // 256 stage-major twiddles
    float2* tiles = twl + 256;                      // 2 x kF2Tile
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tloc = w >> 1;                  // transform of the workgroup
    const int vl = ((w & 1) << 6) | (tid & 63);  // lane of the transform, 0..127
    const long long b = (long long)blockIdx.x * 2 + tloc;
    const bool live = b < batch;             // (no early return: the waves meet at barriers)
    f2v a[E];
    if (live) {
        const float2* src = in + b * L + vl;
#pragma unroll
        for (int q = 0; q < E; ++q) {
            const float2 v = src[NL * q];
            a[q] = f2v{v.x, v.y};
        }
    }
    float2 tw0[16];
#pragma unroll
    for (int i = 0; i < 15; ++i) tw0[i] = tw[i];
    tw0[15] = make_float2(1.0f, 0.0f);
    twl[tid] = tw[tid];  // entries 0 .. 255: pass 0 (tw0) and pass 1
    float2* tile = tiles + tloc * kF2Tile;
    __syncthreads();
    fft2w_pass<0, INV>(a, twl, tw0, vl);
    fft2w_store<0>(a, tile, vl);
    __syncthreads();
    fft2w_load<1>(a, tile, vl);
    fft2w_pass<1, INV>(a, twl, tw0, vl);
    __syncthreads();  // every pass-1 read of the tile before it is overwritten
    fft2w_store<1>(a, tile, vl);
    __syncthreads();
    fft2w_load<2>(a, tile, vl);
    fft2w_pass<2, INV>(a, tw, tw0, vl);
    // last pass (S = 256, R = 8): register g R + f holds point vl + 128 g + 256 bitrev3(f)
    if (live) {
        float2* dst = out + b * L + vl;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int f = 0; f < 8; ++f) dst[NL * g + 256 * bitrevc(f, 3)] = make_float2(a[g * 8 + f].x, a[g * 8 + f].y);
    }
}

hipError_t launch_fft(int n, int inverse, const float2* in, float2* out, const float2* tw, int batch,
                      hipStream_t s) {
    const dim3 grid((unsigned)((batch + 3) / 4)), block(256);
#define PV_FFT_L(LL_)                                                                             \
    {                                                                                             \
        const size_t lds = sizeof(float2) * (LL_ + 4 * Geo<LL_>::TILE);                           \
        if (inverse) hipLaunchKernelGGL((k_fft<LL_, true>), grid, block, lds, s, in, out, tw, batch); \
        else hipLaunchKernelGGL((k_fft<LL_, false>), grid, block, lds, s, in, out, tw, batch);     \
    }
    switch (n) {
        case 128: PV_FFT_L(128); break;
        case 256: PV_FFT_L(256); break;
        case 512: PV_FFT_L(512); break;
        case 1024: PV_FFT_L(1024); break;
        case 2048: {
            const dim3 g2((unsigned)((batch + 1) / 2));
            const size_t lds = sizeof(float2) * (256 + 2 * kF2Tile);
            if (inverse) hipLaunchKernelGGL((k_fft2w<true>), g2, block, lds, s, in, out, tw, batch);
            else hipLaunchKernelGGL((k_fft2w<false>), g2, block, lds, s, in, out, tw, batch);
            break;
        }
        case 32:
        case 64: {
            const dim3 g8((unsigned)((batch + 256 / (n / 8) - 1) / (256 / (n / 8))));
            if (n == 32) {
                if (inverse) hipLaunchKernelGGL((k_fft_t8<32, true>), g8, block, 0, s, in, out, tw, batch);
                else hipLaunchKernelGGL((k_fft_t8<32, false>), g8, block, 0, s, in, out, tw, batch);
            } else {
                if (inverse) hipLaunchKernelGGL((k_fft_t8<64, true>), g8, block, 0, s, in, out, tw, batch);
                else hipLaunchKernelGGL((k_fft_t8<64, false>), g8, block, 0, s, in, out, tw, batch);
            }
            break;
        }
        default: {
            if (n < 2 || n > 64 || (n & (n - 1))) return hipErrorInvalidValue;
            // in-place use reads each lane's transform completely before writing it: safe;
            // 16-byte vector access needs 16-byte aligned buffers (n >= 4)
            if (n >= 4 && ((((uintptr_t)in) | ((uintptr_t)out)) & 15)) {
                if (inverse) hipLaunchKernelGGL((k_fft_small<true>), grid, block, 0, s, in, out, tw, n, batch);
                else hipLaunchKernelGGL((k_fft_small<false>), grid, block, 0, s, in, out, tw, n, batch);
                break;
            }
            const dim3 g2((unsigned)((batch + 255) / 256));
#define PV_FFT_R(NN_)                                                                              \
    case NN_:                                                                                      \
        if (inverse) hipLaunchKernelGGL((k_fft_reg<NN_, true>), g2, block, 0, s, in, out, tw, batch); \
        else hipLaunchKernelGGL((k_fft_reg<NN_, false>), g2, block, 0, s, in, out, tw, batch);       \
        break;
            switch (n) { PV_FFT_R(2) PV_FFT_R(4) PV_FFT_R(8) PV_FFT_R(16) PV_FFT_R(32) PV_FFT_R(64) }
#undef PV_FFT_R
        }
    }
#undef PV_FFT_L
    return hipGetLastError();
}

}  // namespace pv
