// mix_probe — round 5: what sets the rate of the config-3 analysis byte mix (1 KiB of new
// input read + one 4 KiB packed row written per frame, non-temporal stores), with no
// arithmetic?  Diagnostic only (not part of libpv).  1024 channels x 1760 frames, random data.
//   hipcc -O3 --offload-arch=gfx950 -o mix_probe mix_probe.hip && ./mix_probe
//
// Variants (one JSON line each, two repetitions):
//   prod       wave = run of F = 88 frames, workgroup = 4 consecutive runs of a channel, 30 KB
//              LDS pad (5 workgroups per CU, as the product), input loaded at the top of the trip
//   prod_pf    the same with the input prefetched one frame ahead (the product's schedule)
//   prod_pf_occ8  prod_pf without the LDS pad (8 workgroups per CU)
//   prod_pf_x4 prod_pf with 16-byte-per-lane row stores (4 x 1 KiB instead of 8 x 512 B)
//   prod_pf_l2in  prod_pf with every frame re-reading the run's first frame (L2 hits)
//   ilv_pf     workgroup = one run of 4 x 22 frames of a channel, wave w takes frames
//              4 j + w: the 4 waves write 4 adjacent rows per step (each wave still reads
//              1 KiB of new input per frame)
//   stream     one frame per wave, frames in address order, 30 KB pad
//   stream_occ8  the same without the pad
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill(unsigned* p, long long n, unsigned seed) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = 0x3c000000u | (h & 0x007fffffu);
    }
}

constexpr int C = 1024, FRAMES = 1760, F = 88, NRUNS = FRAMES / F, S = 512;
constexpr long long LDX = (long long)FRAMES * 256 + 1024;

// PF: prefetch one frame ahead; X4: dwordx4 stores; L2IN: input of frame t0 only; PAD: 30 KB LDS
template <bool PF, bool X4, bool L2IN, bool PAD, bool ILV>
__global__ __launch_bounds__(256) void k_prod(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[PAD ? 7500 : 1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int c, t0, step, nfr;
    if (!ILV) { c = blockIdx.y; t0 = (blockIdx.x * 4 + w) * F; step = 1; nfr = F; }
    else { c = blockIdx.y; t0 = blockIdx.x * 4 * F + w; step = 4; nfr = F; }  // F frames per wave, stride 4
    const float* xc = x + c * LDX;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto src = [&](int u) { return xc + (long long)(L2IN ? t0 : t0 + u * step) * 256 + 768 + 2 * lane; };
    f2 a = *reinterpret_cast<const f2*>(src(0));
    f2 b = *reinterpret_cast<const f2*>(src(0) + 128);
    for (int u = 0; u < nfr; ++u) {
        const int t = t0 + u * step;
        f2 an, bn;
        if (PF) {
            const int un = u + 1 < nfr ? u + 1 : u;
            an = *reinterpret_cast<const f2*>(src(un));
            bn = *reinterpret_cast<const f2*>(src(un) + 128);
        }
        acc += a * b;
        f2* row = spec + ((long long)c * FRAMES + t) * S;
        if (X4) {
            f4 v = f4{acc.x, acc.y, acc.x + 1.0f, acc.y};
#pragma unroll
            for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(v + (float)i, reinterpret_cast<f4*>(&row[2 * lane + 128 * i]));
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        }
        if (PF) { a = an; b = bn; }
        else if (u + 1 < nfr) {
            a = *reinterpret_cast<const f2*>(src(u + 1));
            b = *reinterpret_cast<const f2*>(src(u + 1) + 128);
        }
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

template <bool PAD>
__global__ __launch_bounds__(256) void k_stream(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[PAD ? 7500 : 1];
    const int lane = threadIdx.x & 63;
    const long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);  // global frame
    const long long c = g / FRAMES, t = g % FRAMES;
    const float* s = x + c * LDX + t * 256 + 768 + 2 * lane;
    const f2 a = *reinterpret_cast<const f2*>(s);
    const f2 b = *reinterpret_cast<const f2*>(s + 128);
    const f2 acc = a * b;
    if (threadIdx.x == 0) pad[0] = acc.x;
    f2* row = spec + g * S;
#pragma unroll
    for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}


// reads only (the prod pattern's input, or one frame per wave in address order): the sum goes out once
template <bool STREAM>
__global__ __launch_bounds__(256) void k_rdonly(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    if (STREAM) {
        const long long g = (long long)blockIdx.x * 4 + w;
        const long long c = g / FRAMES, t = g % FRAMES;
        const float* s = x + c * LDX + t * 256 + 768 + 2 * lane;
        acc += *reinterpret_cast<const f2*>(s) * *reinterpret_cast<const f2*>(s + 128);
    } else {
        const int c = blockIdx.y, t0 = (blockIdx.x * 4 + w) * F;
        const float* xc = x + c * LDX;
        for (int u = 0; u < F; ++u) {
            const float* s = xc + (long long)(t0 + u) * 256 + 768 + 2 * lane;
            acc += *reinterpret_cast<const f2*>(s) * *reinterpret_cast<const f2*>(s + 128);
        }
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// prod with the input read 4 frames at a time (4 KiB contiguous per wave every 4 frames,
// the next chunk prefetched during the current 4 frames)
__global__ __launch_bounds__(256) void k_prod_chunk4(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y, t0 = (blockIdx.x * 4 + w) * F;
    const float* xc = x + c * LDX;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto ld = [&](int u, f2 (&v)[8]) {
        const float* s = xc + (long long)(t0 + u) * 256 + 768 + 2 * lane;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f2*>(s + 128 * i);
    };
    f2 cur[8], nxt[8];
    ld(0, cur);
    for (int u = 0; u < F; u += 4) {
        ld(u + 4 < F ? u + 4 : u, nxt);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc += cur[2 * j] * cur[2 * j + 1];
            f2* row = spec + ((long long)c * FRAMES + t0 + u + j) * S;
#pragma unroll
            for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// one frame per wave, consecutive waves = consecutive channels at the same frame (address
// order broken: each wave's input and row are a channel stride apart from its neighbour's)
__global__ __launch_bounds__(256) void k_stream_tc(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63;
    const long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long t = g / C, c = g % C;
    const float* s = x + c * LDX + t * 256 + 768 + 2 * lane;
    const f2 acc = *reinterpret_cast<const f2*>(s) * *reinterpret_cast<const f2*>(s + 128);
    if (threadIdx.x == 0) pad[0] = acc.x;
    f2* row = spec + (c * FRAMES + t) * S;
#pragma unroll
    for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// prod with runs of FF frames (F = 8: many short runs, fewer channels alive at once)
template <int FF>
__global__ __launch_bounds__(256) void k_prod_f(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y, t0 = (blockIdx.x * 4 + w) * FF;
    const float* xc = x + c * LDX;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto src = [&](int u) { return xc + (long long)(t0 + u) * 256 + 768 + 2 * lane; };
    f2 a = *reinterpret_cast<const f2*>(src(0)), b = *reinterpret_cast<const f2*>(src(0) + 128);
    for (int u = 0; u < FF; ++u) {
        const int un = u + 1 < FF ? u + 1 : u;
        const f2 an = *reinterpret_cast<const f2*>(src(un)), bn = *reinterpret_cast<const f2*>(src(un) + 128);
        acc += a * b;
        f2* row = spec + ((long long)c * FRAMES + t0 + u) * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        a = an; b = bn;
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// prod (F = 88, prefetch) with the address spans varied: MODE 1 every wave reads channel 0's
// input (read span 1.8 MB), 2 every wave writes channel 0's rows (write span 7 MB), 3 channel
// strides of input and rows padded by 28 KiB (no power-of-two channel aliasing), 4 channels in
// a scattered order (c = 613 y mod C)
template <int MODE>
__global__ __launch_bounds__(256) void k_prod_span(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = (MODE == 4) ? (int)((blockIdx.y * 613u) % C) : blockIdx.y;
    const int t0 = (blockIdx.x * 4 + w) * F;
    const long long ldx = (MODE == 3) ? LDX + 7 * 1024 : LDX;
    const long long lds = (MODE == 3) ? (long long)FRAMES * S + 7 * 512 : (long long)FRAMES * S;
    const float* xc = x + (MODE == 1 ? 0 : c) * ldx;
    f2* sc = spec + (MODE == 2 ? 0 : c) * lds;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto src = [&](int u) { return xc + (long long)(t0 + u) * 256 + 768 + 2 * lane; };
    f2 a = *reinterpret_cast<const f2*>(src(0)), b = *reinterpret_cast<const f2*>(src(0) + 128);
    for (int u = 0; u < F; ++u) {
        const int un = u + 1 < F ? u + 1 : u;
        const f2 an = *reinterpret_cast<const f2*>(src(un)), bn = *reinterpret_cast<const f2*>(src(un) + 128);
        acc += a * b;
        f2* row = sc + (long long)(t0 + u) * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        a = an; b = bn;
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// prod (F = 88, prefetch) with the channel of workgroup row y permuted (PM: see main)
__device__ __forceinline__ int perm_ch(int y, int pm) {
    switch (pm) {
        case 0: return y;
        case 1: return (int)((y * 613u) % C);
        case 2: return (y % 8) * (C / 8) + y / 8;
        case 3: return (y % 4) * (C / 4) + y / 4;
        case 4: return (y % 16) * (C / 16) + y / 16;
        case 5: return (y % 2) * (C / 2) + y / 2;
        case 6: return (int)(__brev((unsigned)y) >> 22);  // 10-bit reversal
        case 7: return (y % 32) * (C / 32) + y / 32;
        case 8: return (int)((y * 257u) % C);
        case 9: return (y % 64) * (C / 64) + y / 64;
        default: return y;
    }
}
__global__ __launch_bounds__(256) void k_prod_perm(const float* __restrict__ x, f2* __restrict__ spec, int pm) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = perm_ch(blockIdx.y, pm);
    const int t0 = (blockIdx.x * 4 + w) * F;
    const float* xc = x + c * LDX;
    f2* sc = spec + (long long)c * FRAMES * S;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto src = [&](int u) { return xc + (long long)(t0 + u) * 256 + 768 + 2 * lane; };
    f2 a = *reinterpret_cast<const f2*>(src(0)), b = *reinterpret_cast<const f2*>(src(0) + 128);
    for (int u = 0; u < F; ++u) {
        const int un = u + 1 < F ? u + 1 : u;
        const f2 an = *reinterpret_cast<const f2*>(src(un)), bn = *reinterpret_cast<const f2*>(src(un) + 128);
        acc += a * b;
        f2* row = sc + (long long)(t0 + u) * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        a = an; b = bn;
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}
// the synthesis byte mix (one 4 KiB row read, 512 B of output written per frame) with the
// same channel permutation
__global__ __launch_bounds__(256) void k_syn_perm(const f2* __restrict__ spec, float* __restrict__ y, int pm) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = perm_ch(blockIdx.y, pm);
    const int t0 = (blockIdx.x * 4 + w) * F;
    const long long ldy = (long long)FRAMES * 128 + 1024;
    float* yc = y + c * ldy;
    const f2* sc = spec + (long long)c * FRAMES * S;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    for (int u = 0; u < F; ++u) {
        const f2* row = sc + (long long)(t0 + u) * S;
        f2 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = __builtin_nontemporal_load(&row[lane + 64 * i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += v[i];
        __builtin_nontemporal_store(acc, reinterpret_cast<f2*>(yc + (long long)(t0 + u) * 128 + 2 * lane));
    }
    if (acc.x == -1.0f) y[0] = pad[lane];
}

// prod (F = 88, prefetch) with the cache policy of the row stores / input loads varied:
// ST 0 plain stores, 1 non-temporal; LDNT: non-temporal input loads
template <int ST, bool LDNT>
__global__ __launch_bounds__(256) void k_prod_pol(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y, t0 = (blockIdx.x * 4 + w) * F;
    const float* xc = x + c * LDX;
    f2* sc = spec + (long long)c * FRAMES * S;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto src = [&](int u) { return reinterpret_cast<const f2*>(xc + (long long)(t0 + u) * 256 + 768 + 2 * lane); };
    auto ld = [&](const f2* q) { return LDNT ? __builtin_nontemporal_load(q) : *q; };
    f2 a = ld(src(0)), b = ld(src(0) + 64);
    for (int u = 0; u < F; ++u) {
        const int un = u + 1 < F ? u + 1 : u;
        const f2 an = ld(src(un)), bn = ld(src(un) + 64);
        acc += a * b;
        f2* row = sc + (long long)(t0 + u) * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (ST == 1) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
            else row[lane + 64 * i] = acc + (float)i;
        }
        a = an; b = bn;
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// prod with synthetic VALU work per frame: K rounds of 16 independent v_fma_f32 chains
// (16 K fmas, ~2.25 cycles each per wave at high occupancy): does the 8-frame-run map keep
// its advantage when the frame also computes?
template <int FF, int K>
__global__ __launch_bounds__(256, 5) void k_prod_cmp(const float* __restrict__ x, f2* __restrict__ spec) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y, t0 = (blockIdx.x * 4 + w) * FF;
    const float* xc = x + c * LDX;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    auto src = [&](int u) { return xc + (long long)(t0 + u) * 256 + 768 + 2 * lane; };
    f2 a = *reinterpret_cast<const f2*>(src(0)), b = *reinterpret_cast<const f2*>(src(0) + 128);
    for (int u = 0; u < FF; ++u) {
        const int un = u + 1 < FF ? u + 1 : u;
        const f2 an = *reinterpret_cast<const f2*>(src(un)), bn = *reinterpret_cast<const f2*>(src(un) + 128);
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = a.x * (float)(i + 1) + b.y;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = __builtin_fmaf(v[i], 0.999f, b.x);
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) sum += v[i];
        acc += a * b + sum;
        f2* row = spec + ((long long)c * FRAMES + t0 + u) * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        a = an; b = bn;
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

template <typename Fn>
static double timeit(Fn f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int r = 0; r < 3; ++r) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    return ms / reps;
}

int main() {
    const long long spec_elems = (long long)C * (FRAMES * S + 7 * 512);
    float* x; f2* spec;
    CK(hipMalloc(&x, sizeof(float) * C * (LDX + 7 * 1024)));
    CK(hipMalloc(&spec, sizeof(f2) * spec_elems));
    k_fill<<<8192, 256>>>((unsigned*)x, C * LDX, 12345u);
    k_fill<<<8192, 256>>>((unsigned*)spec, spec_elems * 2, 777u);
    CK(hipDeviceSynchronize());
    const double frames = (double)C * FRAMES, BYTES = 1024.0 + 4096.0;
    auto rep = [&](const char* name, double ms) {
        printf("{\"probe\": \"ana_%s\", \"ms\": %.4f, \"GBps\": %.1f, \"frac_8TBps\": %.3f}\n", name, ms,
               frames * BYTES / ms / 1e6, frames * BYTES / ms / 1e6 / 8000.0);
        fflush(stdout);
    };
    const int R = 10;
    const dim3 gp(NRUNS / 4, C), gi(NRUNS / 4, C);
    const char* only = getenv("MIX_ONLY");
    if (only && only[0] == '5') {
        for (int r2 = 0; r2 < 2; ++r2) {
            rep("cmp0_F88", timeit([&] { k_prod_cmp<88, 0><<<gp, 256>>>(x, spec); }, R));
            rep("cmp0_F8", timeit([&] { k_prod_cmp<8, 0><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
            rep("cmp24_F88", timeit([&] { k_prod_cmp<88, 24><<<gp, 256>>>(x, spec); }, R));
            rep("cmp24_F8", timeit([&] { k_prod_cmp<8, 24><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
            rep("cmp44_F88", timeit([&] { k_prod_cmp<88, 44><<<gp, 256>>>(x, spec); }, R));
            rep("cmp44_F8", timeit([&] { k_prod_cmp<8, 44><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
            rep("cmp60_F88", timeit([&] { k_prod_cmp<88, 60><<<gp, 256>>>(x, spec); }, R));
            rep("cmp60_F8", timeit([&] { k_prod_cmp<8, 60><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
        }
        return 0;
    }
    if (only && only[0] == '4') {
        for (int r2 = 0; r2 < 2; ++r2) {
            rep("pol_st_nt", timeit([&] { k_prod_pol<1, false><<<gp, 256>>>(x, spec); }, R));
            rep("pol_st_plain", timeit([&] { k_prod_pol<0, false><<<gp, 256>>>(x, spec); }, R));
            rep("pol_st_nt_ldnt", timeit([&] { k_prod_pol<1, true><<<gp, 256>>>(x, spec); }, R));
            rep("pol_st_plain_ldnt", timeit([&] { k_prod_pol<0, true><<<gp, 256>>>(x, spec); }, R));
            rep("prod_F8", timeit([&] { k_prod_f<8><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
            rep("stream", timeit([&] { k_stream<true><<<C * FRAMES / 4, 256>>>(x, spec); }, R));
            rep("span_scatter", timeit([&] { k_prod_span<4><<<gp, 256>>>(x, spec); }, R));
        }
        return 0;
    }
    if (only && only[0] == '3') {
        float* yb;
        CK(hipMalloc(&yb, sizeof(float) * C * ((long long)FRAMES * 128 + 1024)));
        const double SYN = 4096.0 + 512.0;
        for (int r2 = 0; r2 < 2; ++r2) {
            for (int pm = 0; pm < 10; ++pm) {
                char nm[32];
                snprintf(nm, sizeof nm, "perm%d", pm);
                rep(nm, timeit([&] { k_prod_perm<<<gp, 256>>>(x, spec, pm); }, R));
            }
            for (int pm = 0; pm < 10; ++pm) {
                const double ms = timeit([&] { k_syn_perm<<<gp, 256>>>(spec, yb, pm); }, R);
                printf("{\"probe\": \"syn_perm%d\", \"ms\": %.4f, \"GBps\": %.1f}\n", pm, ms, frames * SYN / ms / 1e6);
                fflush(stdout);
            }
        }
        return 0;
    }
    if (only && only[0] == '2') {
        for (int r2 = 0; r2 < 2; ++r2) {
            rep("prod_pf", timeit([&] { k_prod<true, false, false, true, false><<<gp, 256>>>(x, spec); }, R));
            rep("span_rcompact", timeit([&] { k_prod_span<1><<<gp, 256>>>(x, spec); }, R));
            rep("span_wcompact", timeit([&] { k_prod_span<2><<<gp, 256>>>(x, spec); }, R));
            rep("span_skew28k", timeit([&] { k_prod_span<3><<<gp, 256>>>(x, spec); }, R));
            rep("span_scatter", timeit([&] { k_prod_span<4><<<gp, 256>>>(x, spec); }, R));
            rep("prod_F8", timeit([&] { k_prod_f<8><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
        }
        return 0;
    }
    for (int r2 = 0; r2 < 2; ++r2) {
        rep("prod", timeit([&] { k_prod<false, false, false, true, false><<<gp, 256>>>(x, spec); }, R));
        rep("prod_pf", timeit([&] { k_prod<true, false, false, true, false><<<gp, 256>>>(x, spec); }, R));
        rep("prod_pf_occ8", timeit([&] { k_prod<true, false, false, false, false><<<gp, 256>>>(x, spec); }, R));
        rep("prod_pf_x4", timeit([&] { k_prod<true, true, false, true, false><<<gp, 256>>>(x, spec); }, R));
        rep("prod_pf_l2in", timeit([&] { k_prod<true, false, true, true, false><<<gp, 256>>>(x, spec); }, R));
        rep("ilv_pf", timeit([&] { k_prod<true, false, false, true, true><<<gi, 256>>>(x, spec); }, R));
        rep("ilv_pf_x4", timeit([&] { k_prod<true, true, false, true, true><<<gi, 256>>>(x, spec); }, R));
        rep("stream", timeit([&] { k_stream<true><<<C * FRAMES / 4, 256>>>(x, spec); }, R));
        rep("stream_occ8", timeit([&] { k_stream<false><<<C * FRAMES / 4, 256>>>(x, spec); }, R));
        rep("prod_chunk4", timeit([&] { k_prod_chunk4<<<gp, 256>>>(x, spec); }, R));
        rep("prod_F8", timeit([&] { k_prod_f<8><<<dim3(FRAMES / 32, C), 256>>>(x, spec); }, R));
        rep("prod_F22", timeit([&] { k_prod_f<22><<<dim3(FRAMES / 88, C), 256>>>(x, spec); }, R));
        rep("stream_tc", timeit([&] { k_stream_tc<<<C * FRAMES / 4, 256>>>(x, spec); }, R));
    }
    // byte-normalised to the 1 KiB read per frame only
    for (int r2 = 0; r2 < 2; ++r2) {
        const double mp = timeit([&] { k_rdonly<false><<<gp, 256>>>(x, spec); }, R);
        const double ms = timeit([&] { k_rdonly<true><<<C * FRAMES / 4, 256>>>(x, spec); }, R);
        printf("{\"probe\": \"rd_prod\", \"ms\": %.4f, \"GBps\": %.1f}\n", mp, frames * 1024.0 / mp / 1e6);
        printf("{\"probe\": \"rd_stream\", \"ms\": %.4f, \"GBps\": %.1f}\n", ms, frames * 1024.0 / ms / 1e6);
        fflush(stdout);
    }
    return 0;
}
