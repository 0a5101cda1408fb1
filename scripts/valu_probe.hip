// valu_probe — issue cost of the VALU instruction forms the analysis kernel is made of
// (diagnostic only, not part of libpv).  Every workgroup (256 lanes, 8 per CU... x4096)
// runs a long unrolled stream of independent instructions of one form on 8 accumulators;
// the result is cycles per wave-instruction per SIMD at the clock the chip holds
// (reported with the in-kernel clock, s_memtime / s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 -o valu_probe valu_probe.hip && ./valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int ITER = 2048;

template <int KIND>
__global__ __launch_bounds__(256) void k_valu(float* out, unsigned long long* clk, float seed) {
    float a[8];
    f2 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = seed + threadIdx.x * 1e-3f + j;
        p[j] = f2{a[j], a[j] + 0.5f};
    }
    const float c1 = seed * 0.999f, c2 = seed * 1e-3f;
    const f2 q1 = f2{c1, c1 * 0.5f}, q2 = f2{c2, c2 * 0.5f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
            if (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[j]) : "v"(q1), "v"(q2));
            if (KIND == 2) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[j]) : "v"(q2));
            if (KIND == 3) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[j]));
            if (KIND == 4) asm volatile("v_max3_f32 %0, |%0|, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
            if (KIND == 5) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c1));
            if (KIND == 6) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[j]) : "v"(q1));
            if (KIND == 7) asm volatile("v_sin_f32 %0, %0" : "+v"(a[j]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + p[j].x + p[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    const int grid = 256 * 8;  // 8 workgroups (32 waves) per CU: 8 waves per SIMD
    float* out; unsigned long long* clk;
    CK(hipMalloc(&out, sizeof(float) * grid * 256));
    CK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * grid));
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_sqrt_f32", "v_max3_f32",
                           "v_cndmask_b32", "v_pk_mul_f32", "v_sin_f32"};
    for (int kind = 0; kind < 8; ++kind) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        auto launch = [&] {
            switch (kind) {
                case 0: k_valu<0><<<grid, 256>>>(out, clk, 1.0f); break;
                case 1: k_valu<1><<<grid, 256>>>(out, clk, 1.0f); break;
                case 2: k_valu<2><<<grid, 256>>>(out, clk, 1.0f); break;
                case 3: k_valu<3><<<grid, 256>>>(out, clk, 1.0f); break;
                case 4: k_valu<4><<<grid, 256>>>(out, clk, 1.0f); break;
                case 5: k_valu<5><<<grid, 256>>>(out, clk, 1.0f); break;
                case 6: k_valu<6><<<grid, 256>>>(out, clk, 1.0f); break;
                case 7: k_valu<7><<<grid, 256>>>(out, clk, 1.0f); break;
            }
        };
        for (int r = 0; r < 3; ++r) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        const int R = 10;
        for (int r = 0; r < R; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        unsigned long long h[2];
        CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
        const double ghz = (double)h[0] / (double)h[1] * 0.1;
        // wave-instructions per SIMD: grid*4 waves / 1024 SIMDs * ITER * 8
        const double per_simd = (double)grid * 4 / 1024.0 * ITER * 8;
        const double cyc = ms * 1e-3 * ghz * 1e9 / per_simd;
        printf("{\"instr\": \"%s\", \"ms\": %.4f, \"clock_GHz\": %.3f, \"cycles_per_wave_instr_per_simd\": %.3f}\n",
               names[kind], ms, ghz, cyc);
        CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    }
    return 0;
}
