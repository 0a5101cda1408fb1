// valu_probe2 — issue cost (8 independent chains per wave) and dependent latency (1 chain)
// of the VALU forms the analysis / synthesis / fused kernels are made of, at 8 waves per
// SIMD and at 1 (diagnostic only, not part of libpv; extends valu_probe.hip, whose
// v_cndmask_b32 row read an undefined VCC).  Result: cycles per wave-instruction per SIMD at
// the clock the chip holds (in-kernel s_memtime / s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 -o valu_probe2 valu_probe2.hip && ./valu_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int ITER = 1024;
constexpr int NK = 20;
static const char* kNames[NK] = {"v_fma_f32", "v_pk_fma_f32", "v_add_f32", "v_mul_f32", "v_mov_b32",
                                 "v_cndmask_b32_e64(sgpr mask)", "v_cndmask_b32(vcc)", "v_cmp_gt_f32_e64(sgpr)",
                                 "v_bfi_b32", "v_rndne_f32", "v_min_f32_e64(abs)", "v_max3_f32(abs)",
                                 "v_add_u32", "v_sqrt_f32", "v_sin_f32", "v_fract_f32",
                                 "v_cndmask_b32_e64(vcc)", "v_cmp_gt_f32_e32(vcc)+v_cndmask_b32(vcc)",
                                 "v_cmp_gt_f32_e64(sgpr)+v_cndmask_b32_e64(sgpr)", "v_sub_f32(literal)"};

template <int KIND, int CHAINS>
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
    unsigned long long cm = 0;
    const unsigned m32 = __builtin_amdgcn_readfirstlane(0x55555555u ^ (unsigned)(seed > 2.0f));
    const unsigned long long mask = ((unsigned long long)m32 << 32) | m32;
    asm volatile("s_mov_b32 vcc_lo, %0\n\ts_mov_b32 vcc_hi, %0" :: "s"(m32) : "vcc");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int j = 0; j < CHAINS; ++j) {
                if (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
                if (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[j]) : "v"(q1), "v"(q2));
                if (KIND == 2) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(c2));
                if (KIND == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(c1));
                if (KIND == 4) asm volatile("v_mov_b32 %0, %0" : "+v"(a[j]));
                if (KIND == 5) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c1), "s"(mask));
                if (KIND == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c1));
                if (KIND == 7) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(cm) : "v"(a[j]), "v"(c1));
                if (KIND == 8) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[j]) : "v"(0x7fffffff), "v"(c1));
                if (KIND == 9) asm volatile("v_rndne_f32 %0, %0" : "+v"(a[j]));
                if (KIND == 10) asm volatile("v_min_f32_e64 %0, |%0|, |%1|" : "+v"(a[j]) : "v"(c1));
                if (KIND == 11) asm volatile("v_max3_f32 %0, |%0|, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
                if (KIND == 12) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(c1));
                if (KIND == 13) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[j]));
                if (KIND == 14) asm volatile("v_sin_f32 %0, %0" : "+v"(a[j]));
                if (KIND == 15) asm volatile("v_fract_f32 %0, %0" : "+v"(a[j]));
                if (KIND == 16) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c1));
                if (KIND == 17)  // counted as two instructions (the pair)
                    asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c1) : "vcc");
                if (KIND == 18) {
                    unsigned long long mm;
                    asm volatile("v_cmp_gt_f32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(a[j]), "=&s"(mm) : "v"(c1));
                }
                if (KIND == 19) asm volatile("v_sub_f32 %0, 0x3fc90fdb, %0" : "+v"(a[j]));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = (float)(cm & 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + p[j].x + p[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int KIND, int CHAINS>
static double run(int wg_per_cu, float* out, unsigned long long* clk) {
    const int grid = 256 * wg_per_cu;
    for (int r = 0; r < 2; ++r) k_valu<KIND, CHAINS><<<grid, 256>>>(out, clk, 1.0f);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    const int R = 5;
    for (int r = 0; r < R; ++r) k_valu<KIND, CHAINS><<<grid, 256>>>(out, clk, 1.0f);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= R;
    unsigned long long h[2];
    CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / (double)h[1] * 0.1;
    // wave-instructions per SIMD: grid * 4 waves / 1024 SIMDs * ITER * 8 * CHAINS
    const double per_simd = (double)grid * 4 / 1024.0 * ITER * 8 * CHAINS * ((KIND == 17 || KIND == 18) ? 2 : 1);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e-3 * ghz * 1e9 / per_simd;
}

template <int KIND>
static void row(float* out, unsigned long long* clk) {
    const double thr8 = run<KIND, 8>(8, out, clk);   // 8 waves/SIMD, 8 independent chains
    const double thr1 = run<KIND, 8>(1, out, clk);   // 1 wave/SIMD, 8 independent chains
    const double lat1 = run<KIND, 1>(1, out, clk);   // 1 wave/SIMD, one dependent chain
    printf("{\"instr\": \"%s\", \"issue_cyc_8waves\": %.2f, \"issue_cyc_1wave\": %.2f, \"dep_chain_cyc_1wave\": %.2f}\n",
           kNames[KIND], thr8, thr1, lat1);
}

template <int... K>
static void all(float* out, unsigned long long* clk, std::integer_sequence<int, K...>) {
    (row<K>(out, clk), ...);
}

int main() {
    float* out;
    unsigned long long* clk;
    CK(hipMalloc(&out, sizeof(float) * 256 * 8 * 256));
    CK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * 256 * 8));
    all(out, clk, std::make_integer_sequence<int, NK>{});
    return 0;
}
