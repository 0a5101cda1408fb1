// rowmap_probe — does writing the spectrum rows of many consecutive frames at once (a
// workgroup of W waves, wave w taking frame u*W + w, one barrier per step) let the analysis
// byte mix run closer to the contiguous-write ceiling than the product's mapping (each wave
// a run of F consecutive frames)?  Diagnostic only (not part of libpv).
//   hipcc -O3 --offload-arch=gfx950 -o rowmap_probe rowmap_probe.hip && ./rowmap_probe
// Config-3 geometry: 1024 channels x 1728 frames, 1 KiB of new input read and one
// 513-float2 row (stride 520) written per frame, non-temporal stores, random data.
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

constexpr int S = 520;  // row stride (float2)

// MAP 0: wave = run of F consecutive frames (4 waves per workgroup: 4 consecutive runs)
// MAP 1: workgroup of W waves walks W*F consecutive frames, wave w takes frame u*W + w,
//        one barrier per step (the phase exchange a frame-parallel analysis would need)
template <int W, int MAP, int LDSB>
__global__ __launch_bounds__(64 * W) void k_rows(const float* __restrict__ x, f2* __restrict__ spec, int F,
                                                 long long ch_samples, long long ch_spec) {
    __shared__ float pad[LDSB > 0 ? LDSB / 4 : 1];  // pins occupancy like the product's LDS
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y;
    const float* xc = x + c * ch_samples;
    f2* sc = spec + c * ch_spec;
    f2 acc = f2((float)lane);
    if (LDSB > 0 && threadIdx.x == 0) pad[0] = acc.x;
    for (int u = 0; u < F; ++u) {
        const long long fr = (MAP == 0) ? (long long)(blockIdx.x * W + w) * F + u
                                        : (long long)blockIdx.x * W * F + (long long)u * W + w;
        const f2 a = *reinterpret_cast<const f2*>(xc + fr * 256 + 2 * lane);
        const f2 b = *reinterpret_cast<const f2*>(xc + fr * 256 + 128 + 2 * lane);
        acc += a * b;
        f2* row = sc + fr * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
        __builtin_nontemporal_store(acc, &row[512]);
        if (MAP == 1) __syncthreads();
    }
    if (LDSB > 0 && acc.x == -1.0f) spec[0] = f2(pad[lane]);
}

__global__ __launch_bounds__(256) void k_contig(f2* __restrict__ y, long long n) {
    const long long i0 = (long long)blockIdx.x * 256 * 8 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (i0 + 256 * u < n) __builtin_nontemporal_store(f2{(float)threadIdx.x, (float)u}, &y[i0 + 256 * u]);
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
    const int C = 1024, frames = 1728;
    const long long ch_samples = (long long)frames * 256 + 1024, ch_spec = (long long)frames * S;
    float* x; f2* spec;
    CK(hipMalloc(&x, sizeof(float) * C * ch_samples));
    CK(hipMalloc(&spec, sizeof(f2) * C * ch_spec));
    k_fill<<<8192, 256>>>((unsigned*)x, C * ch_samples, 12345u);
    k_fill<<<8192, 256>>>((unsigned*)spec, C * ch_spec * 2, 777u);
    CK(hipDeviceSynchronize());
    const double bytes = (double)C * frames * (1024.0 + 4104.0);
    auto rep = [&](const char* name, double ms) {
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
        fflush(stdout);
    };
    const int R = 10;
    const long long nrow = (long long)C * frames * 513;
    rep("contig_same_bytes", timeit([&] { k_contig<<<(nrow + 2047) / 2048, 256>>>(spec, nrow); }, R) *
                                 1.0);
#define RUN(W, MAP, F, LDSB, name) rep(name, timeit([&] { k_rows<W, MAP, LDSB><<<dim3(frames / (W * F), C), 64 * W>>>(x, spec, F, ch_samples, ch_spec); }, R))
    RUN(4, 0, 48, 30000, "product_map_4x48");
    RUN(4, 1, 48, 30000, "wg4_interleaved_48");
    RUN(8, 1, 24, 60000, "wg8_interleaved_24");
    RUN(16, 1, 12, 120000, "wg16_interleaved_12");
    RUN(16, 1, 12, 0, "wg16_interleaved_12_freelds");
    RUN(16, 1, 36, 0, "wg16_interleaved_36_freelds");
    RUN(4, 0, 48, 30000, "product_map_4x48_again");
    return 0;
}
