// mall_probe — does a buffer written by one kernel come back faster than HBM when the next
// kernel reads it (L2 = 4 MB per XCD, Infinity Cache / MALL = 256 MB on the memory side)?
// Diagnostic only (not part of libpv).
//   hipcc -O3 --offload-arch=gfx950 -o mall_probe mall_probe.hip && ./mall_probe
// For S in 8 MB .. 2 GB: write S (temporal or non-temporal 16-byte stores of random-ish
// data), then read the same S at once ("hot"); separately read S after 4 GB of other
// traffic ("cold").  One JSON line per (S, store kind): read GB/s hot vs cold.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void k_write(f4* __restrict__ y, float salt) {
    f4* p = y + (long long)blockIdx.x * 256 * 8 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        unsigned h = (unsigned)(blockIdx.x * 2048 + threadIdx.x + 256 * u) * 2654435761u;
        const f4 v = {(float)(h & 0xffff) * salt, (float)(h >> 16), salt, (float)u};
        if (NT) __builtin_nontemporal_store(v, &p[256 * u]); else p[256 * u] = v;
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ x, float* sink) {
    const f4* p = x + (long long)blockIdx.x * 256 * 8 + threadIdx.x;
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = NT ? __builtin_nontemporal_load(&p[256 * u]) : p[256 * u];
    f4 acc = v[0];
#pragma unroll
    for (int u = 1; u < 8; ++u) acc += v[u];
    if (acc.x == -12345.0f) sink[0] = acc.y;
}

int main() {
    const long long big = 4LL << 30;
    char *buf, *flush; float* sink;
    CK(hipMalloc(&buf, 2LL << 30)); CK(hipMalloc(&flush, big)); CK(hipMalloc(&sink, 4));
    hipEvent_t ev[4];
    for (auto& x : ev) CK(hipEventCreate(&x));
    const long long sizes_mb[] = {8, 32, 64, 128, 192, 256, 384, 512, 2048};
    for (int nt = 0; nt < 2; ++nt) {
        for (long long mb : sizes_mb) {
            const long long bytes = mb << 20;
            const int grid = (int)(bytes / (256LL * 8 * 16));
            double hot = 0, cold = 0, wr = 0;
            const int R = 5;
            for (int r = 0; r < R + 1; ++r) {
                // cold read: touch 4 GB of other memory first
                k_write<false><<<(int)(big / (256LL * 8 * 16)), 256>>>((f4*)flush, 1.0f + r);
                CK(hipEventRecord(ev[0]));
                k_read<false><<<grid, 256>>>((const f4*)buf, sink);
                CK(hipEventRecord(ev[1]));
                // write then read at once
                k_write<false><<<(int)(big / (256LL * 8 * 16)), 256>>>((f4*)flush, 2.0f + r);
                CK(hipEventRecord(ev[2]));
                if (nt) k_write<true><<<grid, 256>>>((f4*)buf, 3.0f + r);
                else k_write<false><<<grid, 256>>>((f4*)buf, 3.0f + r);
                CK(hipEventRecord(ev[3]));
                hipEvent_t e4, e5;
                CK(hipEventCreate(&e4)); CK(hipEventCreate(&e5));
                k_read<false><<<grid, 256>>>((const f4*)buf, sink);
                CK(hipEventRecord(e4));
                CK(hipEventSynchronize(e4));
                float a, b, c;
                CK(hipEventElapsedTime(&a, ev[0], ev[1]));
                CK(hipEventElapsedTime(&b, ev[2], ev[3]));
                CK(hipEventElapsedTime(&c, ev[3], e4));
                if (r > 0) { cold += a; wr += b; hot += c; }
                CK(hipEventDestroy(e4)); CK(hipEventDestroy(e5));
            }
            printf("{\"MB\": %lld, \"store\": \"%s\", \"write_GBps\": %.1f, \"read_cold_GBps\": %.1f, \"read_after_write_GBps\": %.1f}\n",
                   mb, nt ? "nt" : "temporal", bytes * R / wr / 1e6, bytes * R / cold / 1e6, bytes * R / hot / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
