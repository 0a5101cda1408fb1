// bw_probe — HBM bandwidth ceilings on the box for the access shapes of the phase-vocoder
// kernels: write-only, read-only and copy streams of 8 / 16 B per lane, default and
// non-temporal policy.  Diagnostic only (not part of libpv).
//   hipcc -O3 --offload-arch=gfx950 -o bw_probe bw_probe.hip && ./bw_probe [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ y, long long n) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
        T v = T(1.0f + (float)(i & 7));
        if (NT) __builtin_nontemporal_store(v, &y[i]); else y[i] = v;
    }
}
template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ x, long long n, float* sink) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    T acc = T(0.0f);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) acc += x[i];
    float s = acc.x;
    if (s == -12345.0f) sink[0] = s;  // never true: keeps the loads alive
}
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_copy(const T* __restrict__ x, T* __restrict__ y, long long n) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
        T v = x[i];
        if (NT) __builtin_nontemporal_store(v, &y[i]); else y[i] = v;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F>
static double timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const long long bytes = (long long)(gib * (1LL << 30));
    char *x, *y; float* sink;
    CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes)); CK(hipMalloc(&sink, 4));
    CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
    const int grid = 256 * 8 * 4;
    auto rep = [&](const char* name, double ms, double moved) {
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, moved / ms / 1e6);
    };
    const long long n2 = bytes / 8, n4 = bytes / 16;
    rep("write_b64", timeit([&] { k_write<f2, false><<<grid, 256>>>((f2*)y, n2); }, 10), bytes);
    rep("write_b64_nt", timeit([&] { k_write<f2, true><<<grid, 256>>>((f2*)y, n2); }, 10), bytes);
    rep("write_b128", timeit([&] { k_write<f4, false><<<grid, 256>>>((f4*)y, n4); }, 10), bytes);
    rep("write_b128_nt", timeit([&] { k_write<f4, true><<<grid, 256>>>((f4*)y, n4); }, 10), bytes);
    rep("read_b64", timeit([&] { k_read<f2><<<grid, 256>>>((const f2*)x, n2, sink); }, 10), bytes);
    rep("read_b128", timeit([&] { k_read<f4><<<grid, 256>>>((const f4*)x, n4, sink); }, 10), bytes);
    rep("copy_b64", timeit([&] { k_copy<f2, false><<<grid, 256>>>((const f2*)x, (f2*)y, n2); }, 10), 2.0 * bytes);
    rep("copy_b128", timeit([&] { k_copy<f4, false><<<grid, 256>>>((const f4*)x, (f4*)y, n4); }, 10), 2.0 * bytes);
    rep("copy_b128_nt", timeit([&] { k_copy<f4, true><<<grid, 256>>>((const f4*)x, (f4*)y, n4); }, 10), 2.0 * bytes);
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(sink));
    return 0;
}
