// layout_probe — which spectrum row layout / wave mapping lets the analysis byte mix (1 KiB
// of new input read + one row written per frame) and the synthesis byte mix (one row read +
// 512 B of output written per frame) run near the HBM copy ceiling?  Diagnostic only (not
// part of libpv).  Config-3 geometry: 1024 channels x 1728 frames, runs of F = 48 frames
// per wave, non-temporal row stores / loads, random data.
//   hipcc -O3 --offload-arch=gfx950 -o layout_probe layout_probe.hip && ./layout_probe
//
// Row layouts (row index of frame t of channel c; nruns = frames / F):
//   LY 0  channel-major  c*frames + t                      (the product's [c][t][k])
//   LY 1  run-interleaved  c*frames + (t % F)*nruns + t/F  (waves of one channel alive at the
//                                                           same step write adjacent rows)
//   LY 2  time-major  t*C + c                               ([t][c][k])
//   LY 3  channel-major, each run's rows shifted by (run % 16) * 256 B (bank/channel skew)
// Wave mappings:
//   MP 0  workgroup = 4 consecutive runs of one channel, grid (nruns/4, C)  (the product)
//   MP 1  workgroup = one run of 4 consecutive channels, grid (C/4, nruns)
// Row stride S = 520 float2 with bin L written as an 8-byte partial store (the product), or
// 512 with no bin-L store (bin L packed into bin 0: both are real).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill(unsigned* p, long long n, unsigned seed) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = 0x3c000000u | (h & 0x007fffffu);
    }
}

constexpr int C = 1024, FRAMES = 1728, F = 48, NRUNS = FRAMES / F;

template <int LY, int S>
__device__ __forceinline__ long long row_off(int c, int t) {
    if (LY == 0) return ((long long)c * FRAMES + t) * S;
    if (LY == 1) return ((long long)c * FRAMES + (t % F) * NRUNS + t / F) * S;
    if (LY == 2) return ((long long)t * C + c) * S;
    return (long long)c * (FRAMES * S + 16 * 32) + (long long)t * S + ((t / F) % 16) * 32;
}

template <int MP>
__device__ __forceinline__ void wave_of(int& c, int& run) {
    const int w = threadIdx.x >> 6;
    if (MP == 0) { run = blockIdx.x * 4 + w; c = blockIdx.y; }
    else { c = blockIdx.x * 4 + w; run = blockIdx.y; }
}

template <int MP, int FF = F>
static dim3 grid_of() { return MP == 0 ? dim3(FRAMES / FF / 4, C) : dim3(C / 4, FRAMES / FF); }

// analysis byte mix: 1 KiB of input per frame (2 x 512 B), one row out
template <int LY, int MP, int S, bool BINL, int FF = F>
__global__ __launch_bounds__(256) void k_ana(const float* __restrict__ x, f2* __restrict__ spec, long long ldx) {
    __shared__ float pad[7500];  // 30 KB: occupancy like the product (5 workgroups per CU)
    const int lane = threadIdx.x & 63;
    int c, run;
    wave_of<MP>(c, run);
    const float* xc = x + c * ldx;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    for (int u = 0; u < FF; ++u) {
        const int t = run * FF + u;
        const f2 a = *reinterpret_cast<const f2*>(xc + (long long)t * 256 + 768 + 2 * lane);
        const f2 b = *reinterpret_cast<const f2*>(xc + (long long)t * 256 + 896 + 2 * lane);
        acc += a * b;
        f2* row = spec + row_off<LY, S>(c, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        if (BINL) __builtin_nontemporal_store(acc, &row[512]);
    }
    if (acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

// synthesis byte mix: one row in, 512 B of output (128 samples) per frame
template <int LY, int MP, int S, bool BINL, int FF = F>
__global__ __launch_bounds__(256) void k_syn(const f2* __restrict__ spec, float* __restrict__ y, long long ldy) {
    __shared__ float pad[7500];
    const int lane = threadIdx.x & 63;
    int c, run;
    wave_of<MP>(c, run);
    float* yc = y + c * ldy;
    f2 acc = f2((float)lane);
    if (threadIdx.x == 0) pad[0] = acc.x;
    for (int u = 0; u < FF; ++u) {
        const int t = run * FF + u;
        const f2* row = spec + row_off<LY, S>(c, t);
        f2 v[9];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = __builtin_nontemporal_load(&row[lane + 64 * i]);
        v[8] = BINL ? __builtin_nontemporal_load(&row[512]) : f2(0.0f);
#pragma unroll
        for (int i = 0; i < 9; ++i) acc += v[i];
        __builtin_nontemporal_store(acc, reinterpret_cast<f2*>(yc + (long long)t * 128 + 2 * lane));
    }
    if (acc.x == -1.0f) y[0] = pad[lane];
}

// ceilings: the same bytes as pure streams, one frame per wave in address order
template <int S, bool BINL>
__global__ __launch_bounds__(256) void k_ana_stream(const float* __restrict__ x, f2* __restrict__ spec) {
    const int lane = threadIdx.x & 63;
    const long long g = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);  // global frame
    const f2 a = *reinterpret_cast<const f2*>(x + g * 256 + 2 * lane);
    const f2 b = *reinterpret_cast<const f2*>(x + g * 256 + 128 + 2 * lane);
    const f2 acc = a * b;
    f2* row = spec + g * S;
#pragma unroll
    for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
    if (BINL) __builtin_nontemporal_store(acc, &row[512]);
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
    const long long ldx = (long long)FRAMES * 256 + 1024;
    const long long spec_elems = (long long)C * (FRAMES * 520 + 16 * 32);
    const long long ldy = (long long)FRAMES * 128 + 1024;
    float *x, *y; f2* spec;
    CK(hipMalloc(&x, sizeof(float) * C * ldx));
    CK(hipMalloc(&y, sizeof(float) * C * ldy));
    CK(hipMalloc(&spec, sizeof(f2) * spec_elems));
    k_fill<<<8192, 256>>>((unsigned*)x, C * ldx, 12345u);
    k_fill<<<8192, 256>>>((unsigned*)spec, spec_elems * 2, 777u);
    CK(hipDeviceSynchronize());
    const double frames = (double)C * FRAMES;
    auto rep = [&](const char* kind, const char* name, double alg_bytes_per_frame, double ms) {
        printf("{\"probe\": \"%s_%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", kind, name, ms,
               frames * alg_bytes_per_frame / ms / 1e6);
        fflush(stdout);
    };
    const int R = 10;
    const double ANA = 1024.0 + 4104.0, SYN = 4104.0 + 512.0;
#define ANA_RUN(LY, MP, S, BL, name) rep("ana", name, ANA, timeit([&] { k_ana<LY, MP, S, BL><<<grid_of<MP>(), 256>>>(x, spec, ldx); }, R))
#define SYN_RUN(LY, MP, S, BL, name) rep("syn", name, SYN, timeit([&] { k_syn<LY, MP, S, BL><<<grid_of<MP>(), 256>>>(spec, y, ldy); }, R))
#define ANA_RUNF(LY, MP, S, BL, FF, name) rep("ana", name, ANA, timeit([&] { k_ana<LY, MP, S, BL, FF><<<grid_of<MP, FF>(), 256>>>(x, spec, ldx); }, R))
#define SYN_RUNF(LY, MP, S, BL, FF, name) rep("syn", name, SYN, timeit([&] { k_syn<LY, MP, S, BL, FF><<<grid_of<MP, FF>(), 256>>>(spec, y, ldy); }, R))
    for (int rep2 = 0; rep2 < 2; ++rep2) {
        rep("ana", "stream_512", ANA, timeit([&] { k_ana_stream<512, false><<<C * FRAMES / 4, 256>>>(x, spec); }, R));
        ANA_RUN(0, 0, 512, false, "cmaj_product_512");
        ANA_RUN(2, 0, 512, false, "tmaj_product_512");
        ANA_RUN(2, 0, 520, true, "tmaj_product_520_L");
        ANA_RUNF(2, 0, 512, false, 24, "tmaj_product_512_F24");
        ANA_RUNF(2, 0, 512, false, 72, "tmaj_product_512_F72");
        ANA_RUNF(0, 0, 512, false, 72, "cmaj_product_512_F72");
        SYN_RUN(0, 0, 512, false, "cmaj_product_512");
        SYN_RUN(2, 0, 512, false, "tmaj_product_512");
        SYN_RUN(2, 1, 512, false, "tmaj_chgroup_512");
        SYN_RUNF(2, 0, 512, false, 72, "tmaj_product_512_F72");
    }
    return 0;
}
