// bw_probe — HBM bandwidth ceilings of this MI355X for the access shapes of the
// phase-vocoder kernels.  Diagnostic only (not part of libpv).
//   hipcc -O3 --offload-arch=gfx950 -o bw_probe bw_probe.hip && ./bw_probe [GiB]
//
// Every probe runs on random data (a hash fill; zero-filled buffers let the chip hold a
// higher clock, MI355X_MICROARCH.md "DVFS give-back") and keeps U independent 16- or
// 8-byte accesses in flight per lane: each workgroup owns a contiguous tile of
// 256 lanes x U x width bytes and issues all of its loads before its stores (unlike a
// one-load-per-iteration grid-stride loop, which leaves the memory pipeline shallow).
//   read_*   sum of the tile (kept alive by an impossible compare)
//   write_*  store a lane-dependent value
//   copy_*   read tile, write it elsewhere
//   ana_*    the analysis kernel's byte mix and store shape: per "frame" a wave reads
//            1 KiB of input (2 x 8 B per lane) and writes one padded spectrum row of
//            513 float2 (8 x 512 B wave-stores + one 8-byte bin, row stride 520 float2),
//            48 frames per wave, 4 waves per workgroup — the same bytes per frame as
//            k_std_analysis<512,false,2> (4 hop + 8 (N/2+1) = 5128 B) without its ALU work.
//   syn_*    the synthesis kernel's mix: per frame a wave reads a 513-float2 row and
//            writes 128 output floats (hop_s = 128), 48 frames per wave.
// Output: one JSON line per probe {"probe", "ms", "GBps"} (bytes moved / time).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(unsigned* p, long long n, unsigned seed) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = 0x3c000000u | (h & 0x007fffffu);  // random mantissa, |v| in [2^-7, 2^-6)
    }
}

template <typename T, int U>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ x, float* sink) {
    const T* p = x + (long long)blockIdx.x * 256 * U + threadIdx.x;
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[256 * u];
    T acc = v[0];
#pragma unroll
    for (int u = 1; u < U; ++u) acc += v[u];
    if (acc.x == -12345.0f) sink[0] = acc.y;
}

template <typename T, int U, bool NT>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ y) {
    T* p = y + (long long)blockIdx.x * 256 * U + threadIdx.x;
    const T v = T((float)threadIdx.x * 1e-3f);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (NT) __builtin_nontemporal_store(v, &p[256 * u]); else p[256 * u] = v;
    }
}

template <typename T, int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const T* __restrict__ x, T* __restrict__ y) {
    const long long o = (long long)blockIdx.x * 256 * U + threadIdx.x;
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[o + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (NT) __builtin_nontemporal_store(v[u], &y[o + 256 * u]); else y[o + 256 * u] = v[u];
    }
}

// analysis byte mix: wave = run of F frames of one "channel"; input hop 256 floats.
// S: row stride (float2); BL: bin L as 0 = not stored, 1 = one 8-byte store (every lane,
// same address, as k_std_analysis), 2 = a whole 64-byte segment (lanes 0..7, with the
// padding); LD: read the input; W16: 16 bytes per lane (two bins per lane, 4 row stores)
template <bool NT, int S, int BL, bool LD, bool W16>
__global__ __launch_bounds__(256) void k_ana(const float* __restrict__ x, f2* __restrict__ spec, int F,
                                             long long ch_samples, long long ch_spec) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int run = blockIdx.x * 4 + w, c = blockIdx.y;
    const float* xc = x + c * ch_samples + (long long)run * F * 256;
    f2* sc = spec + c * ch_spec + (long long)run * F * S;
    f2 acc = f2((float)lane);
    for (int u = 0; u < F; ++u) {
        if (LD) {
            const f2 a = *reinterpret_cast<const f2*>(xc + u * 256 + 2 * lane);
            const f2 b = *reinterpret_cast<const f2*>(xc + u * 256 + 128 + 2 * lane);
            acc += a * b;
        } else {
            acc += 1.0f;
        }
        f2* row = sc + (long long)u * S;
        if (W16) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f4 v = {acc.x, acc.y, acc.x + (float)i, acc.y};
                f4* d = reinterpret_cast<f4*>(row + 2 * lane + 128 * i);
                if (NT) __builtin_nontemporal_store(v, d); else *d = v;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const f2 v = acc + (float)i;
                if (NT) __builtin_nontemporal_store(v, &row[lane + 64 * i]); else row[lane + 64 * i] = v;
            }
        }
        if (BL == 1) {
            if (NT) __builtin_nontemporal_store(acc, &row[512]); else row[512] = acc;
        } else if (BL == 2 && lane < 8) {
            if (NT) __builtin_nontemporal_store(acc, &row[512 + lane]); else row[512 + lane] = acc;
        }
    }
}

// synthesis byte mix: read a 513-float2 row, write hop_s = 128 floats per frame
__global__ __launch_bounds__(256) void k_syn(const f2* __restrict__ spec, float* __restrict__ out, int F,
                                             long long ch_spec, long long ch_out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int run = blockIdx.x * 4 + w, c = blockIdx.y;
    const f2* sc = spec + c * ch_spec + (long long)run * F * 520 + lane;
    float* oc = out + c * ch_out + (long long)run * F * 128 + 2 * lane;
    for (int u = 0; u < F; ++u) {
        const f2* row = sc + (long long)u * 520;
        f2 acc = __builtin_nontemporal_load(&row[512 - lane]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += __builtin_nontemporal_load(&row[64 * i]);
        __builtin_nontemporal_store(acc, reinterpret_cast<f2*>(oc + u * 128));
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F>
static double timeit(F f, int reps) {
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

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const long long bytes = (long long)(gib * (1LL << 30)) & ~((1LL << 20) - 1);
    char *x, *y; float* sink;
    CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes)); CK(hipMalloc(&sink, 4));
    k_fill<<<8192, 256>>>((unsigned*)x, bytes / 4, 12345u);
    k_fill<<<8192, 256>>>((unsigned*)y, bytes / 4, 777u);
    CK(hipDeviceSynchronize());
    auto rep = [&](const char* name, double ms, double moved) {
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, moved / ms / 1e6);
        fflush(stdout);
    };
    const int R = 20;
#define RD(T, U, name) rep(name, timeit([&] { k_read<T, U><<<bytes / (256LL * U * sizeof(T)), 256>>>((const T*)x, sink); }, R), (double)bytes)
#define WR(T, U, NT, name) rep(name, timeit([&] { k_write<T, U, NT><<<bytes / (256LL * U * sizeof(T)), 256>>>((T*)y); }, R), (double)bytes)
#define CP(T, U, NT, name) rep(name, timeit([&] { k_copy<T, U, NT><<<bytes / 2 / (256LL * U * sizeof(T)), 256>>>((const T*)x, (T*)y); }, R), (double)bytes)
    RD(f4, 1, "read_b128_u1");
    RD(f4, 4, "read_b128_u4");
    RD(f4, 8, "read_b128_u8");
    RD(f2, 8, "read_b64_u8");
    WR(f4, 4, false, "write_b128_u4");
    WR(f4, 8, false, "write_b128_u8");
    WR(f4, 8, true, "write_b128_u8_nt");
    WR(f2, 8, false, "write_b64_u8");
    WR(f2, 8, true, "write_b64_u8_nt");
    CP(f4, 4, false, "copy_b128_u4");
    CP(f4, 8, false, "copy_b128_u8");
    CP(f4, 8, true, "copy_b128_u8_nt");
    CP(f2, 8, false, "copy_b64_u8");
    // analysis / synthesis mixes over the config-3 geometry: C channels x 1722 frames
    {
        const int F = 48, frames = 1728, runs = frames / F;
        const long long ch_samples = (long long)frames * 256 + 1024, ch_spec = (long long)frames * 576;
        int C = (int)(bytes / (long long)(ch_spec * 8));
        if ((long long)C * ch_samples * 4 > bytes) C = (int)(bytes / (ch_samples * 4));
        if (C > 1024) C = 1024;
        const double abytes = (double)C * frames * (1024.0 + 4104.0);
        dim3 grid(runs / 4, C);
#define ANA(NT, S_, BL, LD, W16, name) rep(name, timeit([&] { k_ana<NT, S_, BL, LD, W16><<<grid, 256>>>((const float*)x, (f2*)y, F, ch_samples, (long long)frames * S_); }, R), abytes)
        ANA(true, 520, 1, true, false, "ana_mix_nt");
        ANA(false, 520, 1, true, false, "ana_mix");
        ANA(true, 520, 0, true, false, "ana_mix_nt_noL");
        ANA(true, 520, 2, true, false, "ana_mix_nt_Lseg");
        ANA(true, 576, 1, true, false, "ana_mix_nt_s576");
        ANA(true, 576, 2, true, false, "ana_mix_nt_s576_Lseg");
        ANA(true, 520, 1, false, false, "ana_mix_nt_noload");
        ANA(true, 520, 1, true, true, "ana_mix_nt_w16");
        ANA(true, 576, 2, true, true, "ana_mix_nt_w16_s576_Lseg");
        ANA(false, 576, 2, true, true, "ana_mix_w16_s576_Lseg");
        const long long ch_out = (long long)frames * 128 + 1024;
        const double sbytes = (double)C * frames * (4104.0 + 512.0);
        rep("syn_mix", timeit([&] { k_syn<<<grid, 256>>>((const f2*)y, (float*)x, F, ch_spec, ch_out); }, R), sbytes);
    }
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(sink));
    return 0;
}
