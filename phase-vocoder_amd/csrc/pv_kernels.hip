// pv_kernels.hip — the phase-vocoder hot path as hand-written CDNA4 (gfx950) kernels.
//
// Pipeline, all channels x frames in one launch per stage:
//   K1  k_std_analysis / k_compat_analysis   frame -> window -> real FFT -> {mag, phase}
//         (+ per-run sums of the integer unwrap decisions, STANDARD)
//   K2  k_carry (+ k_runsum when the spectrum did not come from K1)
//         exclusive integer scan of the decisions over runs -> unwrap count at run start
//   K3  k_synthesis<MODE>   phase propagation -> polar->rect -> inverse real FFT ->
//         window -> overlap-add of the run in an LDS ring -> plain stores
//   K4  k_seam   adds each run's overlap tail into the next run's head
//
// Geometry: a workgroup = 4 waves owns a RUN of F consecutive frames of one channel;
// in each round the 4 waves transform 4 consecutive frames (one frame per wavefront).
#include "pv_device.hpp"
#include "pv_kernels.h"

namespace pv {

// ------------------------------------------------------------------ K1 STANDARD
template <int L>
__global__ __launch_bounds__(256) void k_std_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);
    float2* tiles = twl + L;
    float* phiring = reinterpret_cast<float*>(tiles + 4 * G_::TILE);
    const int BP = p.bins_pad;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int run = blockIdx.x, c = blockIdx.y;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    for (int i = tid; i < L; i += 256) twl[i] = p.tw[i];
    __syncthreads();

    float2* tile = tiles + w * G_::TILE;
    const float* xc = p.x + (long long)c * p.ldx;
    float2* specc = p.spec + (long long)c * p.ld_spec;
    int sacc[E + 1];
#pragma unroll
    for (int i = 0; i <= E; ++i) sacc[i] = 0;

    const int rounds = (nfr + 3) >> 2;
    for (int r = 0; r < rounds; ++r) {
        const int u = 4 * r + w;
        const bool valid = u < nfr;
        const int t = t0 + u;
        float phi[E + 1];
        if (valid) {
            float2 z[E];
            const long long base = (long long)t * p.hop;
            if (base + N <= p.n && p.aligned) {
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    const int i = lane + 64 * q;
                    const float2 xv = *reinterpret_cast<const float2*>(xc + base + 2 * i);
                    const float2 wv = *reinterpret_cast<const float2*>(p.win + 2 * i);
                    z[q].x = xv.x * wv.x;
                    z[q].y = xv.y * wv.y;
                }
            } else {
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    const int i = lane + 64 * q;
                    const long long s = base + 2 * i;
                    const float x0 = (s < p.n) ? xc[s] : 0.0f;
                    const float x1 = (s + 1 < p.n) ? xc[s + 1] : 0.0f;
                    z[q].x = x0 * p.win[2 * i];
                    z[q].y = x1 * p.win[2 * i + 1];
                }
            }
            fft_run<L, false>(z, tile, twl, lane);
            float2* srow = specc + (long long)t * p.spec_stride;
#pragma unroll
            for (int i = 0; i <= E; ++i) {
                if (i == E && lane != 0) break;
                const int k = (i == E) ? L : lane + 64 * i;
                const float2 A = tile[G_::pad(k & (L - 1))];
                const float2 Bz = tile[G_::pad((L - k) & (L - 1))];
                const float er = 0.5f * (A.x + Bz.x);
                const float ei = 0.5f * (A.y - Bz.y);
                const float orr = 0.5f * (A.y + Bz.y);
                const float oi = 0.5f * (Bz.x - A.x);
                const float2 tw = p.tws[k];
                float Xr = er + __builtin_fmaf(orr, tw.x, -(oi * tw.y));
                float Xi = ei + __builtin_fmaf(orr, tw.y, oi * tw.x);
                if (k == 0 || k == L) Xi = 0.0f;
                const float mag = __builtin_sqrtf(__builtin_fmaf(Xr, Xr, Xi * Xi));
                const float ph = atan2_pv(Xi, Xr);
                phi[i] = ph;
                srow[k] = make_float2(mag, ph);
                phiring[(u % 5) * BP + k] = ph;
            }
        }
        __syncthreads();
        if (valid && u > 0) {
            const float* prev = phiring + ((u + 4) % 5) * BP;
#pragma unroll
            for (int i = 0; i <= E; ++i) {
                if (i == E && lane != 0) break;
                const int k = (i == E) ? L : lane + 64 * i;
                sacc[i] += unwrap_count(phi[i], prev[k], p.ek[k]);
            }
        }
        __syncthreads();
    }
    if (p.runsum != nullptr) {
        int* sred = reinterpret_cast<int*>(tiles);  // tiles are free now
#pragma unroll
        for (int i = 0; i <= E; ++i) {
            if (i == E && lane != 0) break;
            const int k = (i == E) ? L : lane + 64 * i;
            sred[w * BP + k] = sacc[i];
        }
        __syncthreads();
        int* dst = p.runsum + ((long long)c * p.nruns + run) * BP;
        for (int k = tid; k <= L; k += 256)
            dst[k] = sred[k] + sred[BP + k] + sred[2 * BP + k] + sred[3 * BP + k];
    }
}

// ------------------------------------------------------------------ K1 REF_COMPAT
// kernel.cu:299-348: window (Hamming), zero-phase shift + zero pad to 2N, C2C 2N,
// (|X|, atanf(Im/Re)) for all 2N bins.  The 2N-point transform of the real padded frame
// is computed as an L = N point complex FFT + real split; bins > N by symmetry.
template <int L>
__global__ __launch_bounds__(256) void k_compat_analysis(AnaParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = L;  // window length
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);
    float2* tiles = twl + L;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int run = blockIdx.x, c = blockIdx.y;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    for (int i = tid; i < L; i += 256) twl[i] = p.tw[i];
    __syncthreads();
    float2* tile = tiles + w * G_::TILE;
    const float* xc = p.x + (long long)c * p.ldx;
    float2* specc = p.spec + (long long)c * p.ld_spec;

    for (int u = w; u < nfr; u += 4) {
        const int t = t0 + u;
        const long long base = (long long)t * p.hop;
        float2 z[E];
#pragma unroll
        for (int q = 0; q < E; ++q) {
            const int i = lane + 64 * q;
            // b[2i], b[2i+1] of the shifted/padded 2N buffer (kernel.cu:25-32)
            int src = -1;
            if (2 * i < N / 2) src = 2 * i + N / 2;
            else if (2 * i >= 3 * N / 2) src = 2 * i - 3 * N / 2;
            float b0 = 0.0f, b1 = 0.0f;
            if (src >= 0) {
                const long long s = base + src;
                const float x0 = (s < p.n) ? xc[s] : 0.0f;
                const float x1 = (s + 1 < p.n) ? xc[s + 1] : 0.0f;
                b0 = x0 * p.win[src];
                b1 = x1 * p.win[src + 1];
            }
            z[q] = make_float2(b0, b1);
        }
        fft_run<L, false>(z, tile, twl, lane);
        float2* srow = specc + (long long)t * p.spec_stride;
#pragma unroll
        for (int i = 0; i <= E; ++i) {
            if (i == E && lane != 0) break;
            const int k = (i == E) ? L : lane + 64 * i;
            const float2 A = tile[G_::pad(k & (L - 1))];
            const float2 Bz = tile[G_::pad((L - k) & (L - 1))];
            const float er = 0.5f * (A.x + Bz.x);
            const float ei = 0.5f * (A.y - Bz.y);
            const float orr = 0.5f * (A.y + Bz.y);
            const float oi = 0.5f * (Bz.x - A.x);
            const float2 tw = p.tws[k];
            const float Xr = er + __builtin_fmaf(orr, tw.x, -(oi * tw.y));
            float Xi = ei + __builtin_fmaf(orr, tw.y, oi * tw.x);
            if (k == 0 || k == L) Xi = 0.0f;
            const float mag = __builtin_sqrtf(Xr * Xr + Xi * Xi);
            float ph = atanf(Xi / Xr);
            if (Xr == 0.0f && Xi == 0.0f) ph = p.nan_faithful ? __builtin_nanf("") : 0.0f;
            srow[k] = make_float2(mag, ph);
            if (k != 0 && k != L) srow[2 * N - k] = make_float2(mag, -ph);
        }
    }
}

// ------------------------------------------------------------------ K2 scans
__global__ __launch_bounds__(256) void k_runsum(ScanParams p) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int run = blockIdx.y, c = blockIdx.z;
    if (k > p.L) return;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    const float2* s = p.spec + (long long)c * p.ld_spec + (long long)t0 * p.spec_stride + k;
    const float e = p.ek[k];
    float prev = s[0].y;
    int acc = 0;
    for (int u = 1; u < nfr; ++u) {
        const float ph = s[(long long)u * p.spec_stride].y;
        acc += unwrap_count(ph, prev, e);
        prev = ph;
    }
    p.runsum[((long long)c * p.nruns + run) * p.bins_pad + k] = acc;
}

__global__ __launch_bounds__(256) void k_carry(ScanParams p) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (k > p.L) return;
    const float2* s = p.spec + (long long)c * p.ld_spec + k;
    const float e = p.ek[k];
    const int* rs = p.runsum + (long long)c * p.nruns * p.bins_pad + k;
    int* cr = p.carry + (long long)c * p.nruns * p.bins_pad + k;
    int M = 0;
    for (int run = 0; run < p.nruns; ++run) {
        const long long t0 = (long long)run * p.F;
        const float ph0 = s[t0 * p.spec_stride].y;
        const float php = (t0 > 0) ? s[(t0 - 1) * p.spec_stride].y : 0.0f;
        M += unwrap_count(ph0, php, e);
        cr[(long long)run * p.bins_pad] = M;
        M += rs[(long long)run * p.bins_pad];
    }
}

// ------------------------------------------------------------------ K3 synthesis
// MODE 0: STANDARD — output phase rho*(phi + 2 pi (M_dec + (t+1) j_k)),
//         Hann synthesis window with overlap normalisation folded into gain[].
// MODE 1: REF_COMPAT — kernel.cu:352-432: x' = m cos(phi), y' = x' sin(phi), C2R N, /N,
//         swap halves (rot = N/2), Hamming window (gain = w/N), overlap-add at out_hop.
template <int L, int MODE>
__global__ __launch_bounds__(256) void k_synthesis(SynParams p) {
    using G_ = Geo<L>;
    constexpr int E = G_::E;
    constexpr int N = 2 * L;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* twl = reinterpret_cast<float2*>(smem);
    float2* tiles = twl + L;
    float* ring = reinterpret_cast<float*>(tiles + 4 * G_::TILE);
    float* phiring = ring + p.ring_size;         // 5 * BP   (MODE 0)
    int* Mbase = reinterpret_cast<int*>(phiring + 5 * p.bins_pad);  // BP
    int* mring = Mbase + p.bins_pad;                                 // 4 * BP
    const int BP = p.bins_pad;
    const int RMASK = p.ring_size - 1;
    const int hs = p.hs;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int run = blockIdx.x, c = blockIdx.y;
    const int t0 = run * p.F;
    const int nfr = min(p.F, p.frames - t0);
    for (int i = tid; i < L; i += 256) twl[i] = p.tw[i];
    for (int i = tid; i < p.ring_size; i += 256) ring[i] = 0.0f;
    if (MODE == 0) {
        const int* cr = p.carry + ((long long)c * p.nruns + run) * BP;
        for (int k = tid; k <= L; k += 256) Mbase[k] = cr[k];
    }
    __syncthreads();

    float2* tile = tiles + w * G_::TILE;
    const float2* specc = p.spec + (long long)c * p.ld_spec;
    float* outc = p.out + (long long)c * p.ldo;
    const long long obase = (long long)t0 * hs;

    const int rounds = (nfr + 3) >> 2;
    for (int r = 0; r < rounds; ++r) {
        const int u = 4 * r + w;
        const bool valid = u < nfr;
        const int t = t0 + u;
        float mag[E + 1], ph[E + 1];
        if (valid) {
            const float2* srow = specc + (long long)t * p.spec_stride;
#pragma unroll
            for (int i = 0; i <= E; ++i) {
                if (i == E && lane != 0) break;
                const int k = (i == E) ? L : lane + 64 * i;
                const float2 v = srow[k];
                mag[i] = v.x;
                ph[i] = v.y;
            }
        }
        float phc[E + 1];  // output phase (MODE 0) per analysis bin
        if (MODE == 0) {
            if (valid) {
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    phiring[(u % 5) * BP + k] = ph[i];
                }
            }
            __syncthreads();
            {
                const float* prev = phiring + ((u + 4) % 5) * BP;
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    const int m = (valid && u > 0) ? unwrap_count(ph[i], prev[k], p.ek[k]) : 0;
                    mring[w * BP + k] = m;
                }
            }
            __syncthreads();
            if (valid) {
                const unsigned tq = (unsigned)((long long)(t + 1) % p.q);
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    int Md = Mbase[k];
                    for (int ww = 0; ww <= w; ++ww) Md += mring[ww * BP + k];
                    // (p*M_tot) mod q with M_tot = M_dec + (t+1) j_k, all reduced mod q
                    int mdq;
                    if (p.q_pow2) {
                        mdq = Md & (int)(p.q - 1);  // two's complement: non-negative residue
                    } else {
                        mdq = Md % (int)p.q;
                        if (mdq < 0) mdq += (int)p.q;
                    }
                    const unsigned long long x =
                        (unsigned long long)p.p_mod * (unsigned long long)mdq +
                        (unsigned long long)tq * (unsigned long long)p.jk_mod[k];
                    const unsigned long long rr = p.q_pow2 ? (x & (unsigned long long)(p.q - 1))
                                                           : (x % (unsigned long long)p.q);
                    const float frac = (float)rr * p.inv_q;
                    phc[i] = __builtin_fmaf(p.rho, ph[i], kTwoPi * frac);
                }
            }
            __syncthreads();
            if (w == 0) {
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    Mbase[k] += mring[k] + mring[BP + k] + mring[2 * BP + k] + mring[3 * BP + k];
                }
            }
        }
        if (valid) {
            // polar -> rect into the tile (natural bin order, padded index)
            if (MODE == 0 && p.pitch) {
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    tile[G_::pad(k)] = make_float2(mag[i], phc[i]);
                }
                wave_lds_sync();
                float2 Y[E + 1];
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    const int s = p.src_first[k];
                    float ms = 0.0f, pc = 0.0f;
                    if (s >= 0) {
                        const int cnt = p.src_cnt[k];
                        pc = tile[G_::pad(s)].y;
                        for (int qq = 0; qq < cnt; ++qq) ms += tile[G_::pad(s + qq)].x;
                    }
                    float sn, cs;
                    __builtin_sincosf(pc, &sn, &cs);
                    Y[i] = make_float2(ms * cs, ms * sn);
                }
                wave_lds_sync();
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    float2 y = Y[i];
                    if (k == 0 || k == L) y.y = 0.0f;
                    tile[G_::pad(k)] = y;
                }
            } else {
#pragma unroll
                for (int i = 0; i <= E; ++i) {
                    if (i == E && lane != 0) break;
                    const int k = (i == E) ? L : lane + 64 * i;
                    float2 y;
                    if (MODE == 0) {
                        float sn, cs;
                        __builtin_sincosf(phc[i], &sn, &cs);
                        y = make_float2(mag[i] * cs, mag[i] * sn);
                    } else {
                        float sn, cs;
                        __builtin_sincosf(ph[i], &sn, &cs);
                        const float xr = mag[i] * cs;   // kernel.cu:127
                        y = make_float2(xr, xr * sn);   // kernel.cu:128 (uses updated x)
                    }
                    if (k == 0 || k == L) y.y = 0.0f;
                    tile[G_::pad(k)] = y;
                }
            }
            wave_lds_sync();
            // inverse real-FFT pre-step: Z[i] = Fe + i Fo, pass-0 layout i = lane + 64 q
            float2 z[E];
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int i = lane + 64 * q;
                const float2 A = tile[G_::pad(i)];
                const float2 Bc = tile[G_::pad(L - i)];
                const float fer = A.x + Bc.x, fei = A.y - Bc.y;    // A + conj(B)
                const float dr = A.x - Bc.x, di = A.y + Bc.y;      // A - conj(B)
                const float2 tw = p.tws[i];                        // e^{-2 pi i k/N}
                // Fo = (A - conj B) * conj(tw)
                const float For = __builtin_fmaf(dr, tw.x, di * tw.y);
                const float Foi = __builtin_fmaf(di, tw.x, -(dr * tw.y));
                z[q] = make_float2(fer - Foi, fei + For);
            }
            wave_lds_sync();
            fft_run<L, true>(z, tile, twl, lane);
        }
        __syncthreads();
        // overlap-add of this round's frames into the LDS ring (fixed frame order)
        {
            const int base = 4 * r * hs;
            const int span = 3 * hs + N;
            for (int pp = tid; pp < span; pp += 256) {
                const int pos = base + pp;
                float sum = 0.0f;
#pragma unroll
                for (int ww = 0; ww < 4; ++ww) {
                    const int uu = 4 * r + ww;
                    const int pl = pos - uu * hs;
                    if (uu < nfr && pl >= 0 && pl < N) {
                        const int nn = (pl + p.rot) & (N - 1);
                        const float* ty = reinterpret_cast<const float*>(tiles + ww * G_::TILE);
                        const float yv = ty[2 * G_::pad(nn >> 1) + (nn & 1)];
                        sum = __builtin_fmaf(yv, p.gain[pl], sum);
                    }
                }
                ring[pos & RMASK] += sum;
            }
        }
        __syncthreads();
        {
            const int f0 = 4 * r * hs;
            const int f1 = min(4 * r + 4, nfr) * hs;
            for (int pos = f0 + tid; pos < f1; pos += 256) {
                outc[obase + pos] = ring[pos & RMASK];
                ring[pos & RMASK] = 0.0f;
            }
        }
    }
    __syncthreads();
    // tail: [nfr*hs, nfr*hs + N - hs)
    {
        const int tl = N - hs;
        const bool last = (t0 + nfr >= p.frames);
        float* tdst = p.tails + ((long long)c * p.nruns + run) * p.tail_len;
        for (int j = tid; j < tl; j += 256) {
            const int pos = nfr * hs + j;
            const float v = ring[pos & RMASK];
            if (last) {
                if (obase + pos < p.out_len) outc[obase + pos] = v;
            } else {
                tdst[j] = v;
            }
        }
    }
}

// ------------------------------------------------------------------ K4 seam
__global__ __launch_bounds__(256) void k_seam(SeamParams p) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y, c = blockIdx.z;
    if (j >= p.tail_len) return;
    float* outc = p.out + (long long)c * p.ldo;
    if (b == 0) {
        if (p.ola_in != nullptr && j < p.out_len) outc[j] += p.ola_in[(long long)c * p.ld_ola + j];
    } else {
        const long long pos = (long long)b * p.F * p.hs + j;
        if (pos < p.out_len)
            outc[pos] += p.tails[((long long)c * p.nruns + (b - 1)) * p.tail_len + j];
    }
}

// ------------------------------------------------------------------ launchers
template <int L>
static size_t ana_lds_std(int bins_pad) {
    return sizeof(float2) * (L + 4 * Geo<L>::TILE) + sizeof(float) * 5 * bins_pad;
}
template <int L>
static size_t ana_lds_compat() {
    return sizeof(float2) * (L + 4 * Geo<L>::TILE);
}
template <int L>
static size_t syn_lds(int bins_pad, int ring) {
    return sizeof(float2) * (L + 4 * Geo<L>::TILE) + sizeof(float) * ring +
           sizeof(float) * 5 * bins_pad + sizeof(int) * 5 * bins_pad;
}

size_t synthesis_lds_bytes(int L, int bins_pad, int ring) {
    switch (L) {
        case 128: return syn_lds<128>(bins_pad, ring);
        case 256: return syn_lds<256>(bins_pad, ring);
        case 512: return syn_lds<512>(bins_pad, ring);
        case 1024: return syn_lds<1024>(bins_pad, ring);
        case 2048: return syn_lds<2048>(bins_pad, ring);
    }
    return 0;
}

#define PV_DISPATCH_L(L_, EXPR)                       \
    switch (L_) {                                     \
        case 128: { constexpr int LL = 128; EXPR; } break;   \
        case 256: { constexpr int LL = 256; EXPR; } break;   \
        case 512: { constexpr int LL = 512; EXPR; } break;   \
        case 1024: { constexpr int LL = 1024; EXPR; } break; \
        case 2048: { constexpr int LL = 2048; EXPR; } break; \
        default: return hipErrorInvalidValue;         \
    }

hipError_t launch_std_analysis(int L, int channels, const AnaParams& p, hipStream_t s) {
    dim3 grid(p.nruns, channels);
    PV_DISPATCH_L(L, {
        hipLaunchKernelGGL(k_std_analysis<LL>, grid, dim3(256), ana_lds_std<LL>(p.bins_pad), s, p);
    });
    return hipGetLastError();
}

hipError_t launch_compat_analysis(int L, int channels, const AnaParams& p, hipStream_t s) {
    dim3 grid(p.nruns, channels);
    PV_DISPATCH_L(L, {
        hipLaunchKernelGGL(k_compat_analysis<LL>, grid, dim3(256), ana_lds_compat<LL>(), s, p);
    });
    return hipGetLastError();
}

hipError_t launch_runsum(int channels, const ScanParams& p, hipStream_t s) {
    dim3 grid((p.L + 1 + 255) / 256, p.nruns, channels);
    hipLaunchKernelGGL(k_runsum, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_carry(int channels, const ScanParams& p, hipStream_t s) {
    dim3 grid((p.L + 1 + 255) / 256, channels);
    hipLaunchKernelGGL(k_carry, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_synthesis(int L, int mode, int channels, const SynParams& p, hipStream_t s) {
    dim3 grid(p.nruns, channels);
    if (mode == 0) {
        PV_DISPATCH_L(L, {
            hipLaunchKernelGGL((k_synthesis<LL, 0>), grid, dim3(256),
                               syn_lds<LL>(p.bins_pad, p.ring_size), s, p);
        });
    } else {
        PV_DISPATCH_L(L, {
            hipLaunchKernelGGL((k_synthesis<LL, 1>), grid, dim3(256),
                               syn_lds<LL>(p.bins_pad, p.ring_size), s, p);
        });
    }
    return hipGetLastError();
}

hipError_t launch_seam(int channels, const SeamParams& p, hipStream_t s) {
    dim3 grid((p.tail_len + 255) / 256, p.nruns, channels);
    hipLaunchKernelGGL(k_seam, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace pv
