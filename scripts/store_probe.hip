// store_probe — which spectrum-row write shape lets the analysis byte mix run at the
// chip's write ceiling?  Diagnostic only (not part of libpv).
//   hipcc -O3 --offload-arch=gfx950 -o store_probe store_probe.hip && ./store_probe
//
// Same geometry as bw_probe's ana_* mix (config 3: 1024 channels x 1728 frames, 48 frames
// per wave, 4 waves per workgroup, 4 KiB input read + one 513-float2 row written per frame),
// random data, every variant timed back to back.  Knobs:
//   S     row stride in float2 (520 = the product's 64-byte padding, 528 / 576 / 1024)
//   MAP   0: wave = run of F consecutive rows (the product's mapping)
//         1: the 4 waves of a workgroup take rows 4u + w of 4F consecutive rows, so each
//            step of a workgroup writes 4 adjacent rows (16 KiB contiguous)
//   BL    bin L: 0 not written, 1 one 8-byte store (all lanes, one address), 2 a whole
//         64-byte segment (lanes 0..7, with the row's padding)
//   LDS   dynamic LDS per workgroup, to pin occupancy at the product's (~30 KiB -> 4-5
//         workgroups per CU) or leave it free (0)
//   NT    non-temporal row stores
// Output: one JSON line per variant {"probe", "ms", "GBps"} (5128 B per frame / time).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k_fill(unsigned* p, long long n, unsigned seed) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = 0x3c000000u | (h & 0x007fffffu);
    }
}

// cache-policy bits of the row stores: 0 plain / nt (per NT), 1 sc1, 2 sc0 sc1, 3 nt sc1,
// 4 nt sc0 sc1 (MI355X_MICROARCH.md: sc1 / sc0 sc1 stores drop the line from the XCD's L2)
template <int POL>
__device__ __forceinline__ void st_pol(f2* p, f2 v) {
    if constexpr (POL == 1) asm volatile("global_store_dwordx2 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx2 %0, %1, off nt sc1" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off nt sc0 sc1" :: "v"(p), "v"(v) : "memory");
}

template <int S, int MAP, int BL, bool NT, int POL = 0>
__global__ __launch_bounds__(256) void k_rows(const float* __restrict__ x, f2* __restrict__ spec, int F,
                                              long long ch_samples, long long ch_spec) {
    extern __shared__ float lds_pad[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y;
    const float* xc = x + c * ch_samples;
    f2* sc = spec + c * ch_spec;
    if (lane == 64) lds_pad[0] = 0.0f;  // keep the allocation
    f2 acc = f2((float)lane);
    for (int u = 0; u < F; ++u) {
        long long t;
        if (MAP == 0) t = (long long)(blockIdx.x * 4 + w) * F + u;
        else t = (long long)blockIdx.x * 4 * F + 4 * u + w;
        const f2 a = *reinterpret_cast<const f2*>(xc + t * 256 + 2 * lane);
        const f2 b = *reinterpret_cast<const f2*>(xc + t * 256 + 128 + 2 * lane);
        acc += a * b;
        f2* row = sc + t * S;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const f2 v = acc + (float)i;
            if (POL) st_pol<POL>(&row[lane + 64 * i], v);
            else if (NT) __builtin_nontemporal_store(v, &row[lane + 64 * i]); else row[lane + 64 * i] = v;
        }
        if (BL == 1) {
            if (POL) st_pol<POL>(&row[512], acc);
            else if (NT) __builtin_nontemporal_store(acc, &row[512]); else row[512] = acc;
        } else if (BL == 2 && lane < 8) {
            if (POL) st_pol<POL>(&row[512 + lane], acc);
            else if (NT) __builtin_nontemporal_store(acc, &row[512 + lane]); else row[512 + lane] = acc;
        }
    }
}

// input reads batched: every K frames a wave loads the K frames' new input (K KiB) at once,
// then writes the K rows (tests whether the read/write interleaving costs the mix)
template <int K>
__global__ __launch_bounds__(256) void k_rows_batched(const float* __restrict__ x, f2* __restrict__ spec, int F,
                                                      long long ch_samples, long long ch_spec) {
    extern __shared__ float lds_pad[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y;
    const float* xc = x + c * ch_samples;
    f2* sc = spec + c * ch_spec;
    if (lane == 64) lds_pad[0] = 0.0f;
    f2 acc = f2((float)lane);
    const long long r0 = (long long)(blockIdx.x * 4 + w) * F;
    for (int u0 = 0; u0 < F; u0 += K) {
        f2 a[K], b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            a[k] = *reinterpret_cast<const f2*>(xc + (r0 + u0 + k) * 256 + 2 * lane);
            b[k] = *reinterpret_cast<const f2*>(xc + (r0 + u0 + k) * 256 + 128 + 2 * lane);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc += a[k] * b[k];
            f2* row = sc + (r0 + u0 + k) * 520;
#pragma unroll
            for (int i = 0; i < 8; ++i) __builtin_nontemporal_store(acc + (float)i, &row[lane + 64 * i]);
            if (lane < 8) __builtin_nontemporal_store(acc, &row[512 + lane]);
        }
    }
}

// the reference point: plain contiguous writes of the same byte count (16 KiB per workgroup)
__global__ __launch_bounds__(256) void k_write(f2* __restrict__ y) {
    f2* p = y + (long long)blockIdx.x * 256 * 8 + threadIdx.x;
    const f2 v = f2((float)threadIdx.x * 1e-3f);
#pragma unroll
    for (int u = 0; u < 8; ++u) __builtin_nontemporal_store(v, &p[256 * u]);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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
    const int C = 1024, F = 48, frames = 1728, runs = frames / F;
    const long long ch_samples = (long long)frames * 256 + 1024;
    const long long xbytes = (long long)C * ch_samples * 4;
    const long long sbytes = (long long)C * frames * 1024 * 8;  // room for S <= 1024
    char *x, *y;
    CK(hipMalloc(&x, xbytes)); CK(hipMalloc(&y, sbytes));
    k_fill<<<8192, 256>>>((unsigned*)x, xbytes / 4, 12345u);
    k_fill<<<8192, 256>>>((unsigned*)y, sbytes / 4, 777u);
    CK(hipDeviceSynchronize());
    const double abytes = (double)C * frames * 5128.0;
    auto rep = [&](const char* name, double ms, double bytes) {
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
        fflush(stdout);
    };
    const int R = 20;
    dim3 grid(runs / 4, C);
#define ROWS(S_, MAP_, BL_, NT_, LDS_, name)                                                                  \
    rep(name, timeit([&] {                                                                                     \
        hipLaunchKernelGGL((k_rows<S_, MAP_, BL_, NT_>), grid, dim3(256), LDS_, 0, (const float*)x, (f2*)y, F, \
                           ch_samples, (long long)frames * S_);                                                \
    }, R), abytes)
    const long long wn = (long long)C * frames * 4104 / (256LL * 8 * 8);
    rep("write_contig_same_bytes", timeit([&] { k_write<<<wn, 256>>>((f2*)y); }, R), (double)wn * 256 * 8 * 8);
#define ROWSP(S_, BL_, POL_, name)                                                                      \
    rep(name, timeit([&] {                                                                               \
        hipLaunchKernelGGL((k_rows<S_, 0, BL_, true, POL_>), grid, dim3(256), 30000, 0, (const float*)x, \
                           (f2*)y, F, ch_samples, (long long)frames * S_);                               \
    }, R), abytes)
#define ROWSB(K_, name)                                                                                 \
    rep(name, timeit([&] {                                                                               \
        hipLaunchKernelGGL((k_rows_batched<K_>), grid, dim3(256), 30000, 0, (const float*)x, (f2*)y, F,  \
                           ch_samples, (long long)frames * 520);                                          \
    }, R), abytes)
    for (int pass = 0; pass < 2; ++pass) {
        ROWS(520, 0, 2, true, 30000, "s520_bl2_nt");
        ROWSB(1, "batched_K1");
        ROWSB(2, "batched_K2");
        ROWSB(4, "batched_K4");
        ROWSB(8, "batched_K8");
        ROWSB(16, "batched_K16");
    }
    for (int pass = 0; pass < 0; ++pass) {
        ROWS(520, 0, 1, true, 30000, "s520_bl1_nt (product)");
        ROWSP(520, 1, 1, "s520_bl1_sc1");
        ROWSP(520, 1, 2, "s520_bl1_sc0sc1");
        ROWSP(520, 1, 3, "s520_bl1_ntsc1");
        ROWSP(520, 1, 4, "s520_bl1_ntsc0sc1");
        ROWS(520, 0, 2, true, 30000, "s520_bl2_nt");
        ROWSP(520, 2, 1, "s520_bl2_sc1");
        ROWSP(520, 2, 2, "s520_bl2_sc0sc1");
        ROWSP(520, 2, 3, "s520_bl2_ntsc1");
    }
    for (int pass = 0; pass < 0; ++pass) {
        ROWS(520, 0, 1, true, 30000, "s520_map0_bl1_lds30k (product)");
        ROWS(520, 0, 1, true, 0, "s520_map0_bl1_lds0");
        ROWS(520, 0, 2, true, 30000, "s520_map0_bl2_lds30k");
        ROWS(520, 0, 0, true, 30000, "s520_map0_bl0_lds30k");
        ROWS(528, 0, 2, true, 30000, "s528_map0_bl2_lds30k");
        ROWS(576, 0, 2, true, 30000, "s576_map0_bl2_lds30k");
        ROWS(1024, 0, 2, true, 30000, "s1024_map0_bl2_lds30k");
        ROWS(520, 1, 1, true, 30000, "s520_map1_bl1_lds30k");
        ROWS(520, 1, 2, true, 30000, "s520_map1_bl2_lds30k");
        ROWS(528, 1, 2, true, 30000, "s528_map1_bl2_lds30k");
        ROWS(576, 1, 2, true, 30000, "s576_map1_bl2_lds30k");
        ROWS(520, 1, 2, false, 30000, "s520_map1_bl2_lds30k_temporal");
        ROWS(520, 0, 2, false, 30000, "s520_map0_bl2_lds30k_temporal");
        ROWS(520, 1, 2, true, 0, "s520_map1_bl2_lds0");
        ROWS(520, 1, 2, true, 50000, "s520_map1_bl2_lds50k");
        ROWS(520, 0, 2, true, 50000, "s520_map0_bl2_lds50k");
    }
    CK(hipFree(x)); CK(hipFree(y));
    return 0;
}
