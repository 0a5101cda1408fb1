// valu_probe3 — issue cost of more gfx950 VALU forms (diagnostic only, not part of libpv):
// the integer / bitwise ops, e32 vs e64 encodings, source modifiers, selects with a
// loop-invariant mask (VCC or SGPR pair), per-chain compares, packed forms and DPP moves.
// Same harness as valu_probe2.hip: 8 independent chains per wave at 8 waves per SIMD
// (issue cost) and one dependent chain at 1 wave per SIMD (latency); cycles per
// wave-instruction per SIMD at the clock the chip holds (s_memtime / s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 -o valu_probe3 valu_probe3.hip && ./valu_probe3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <utility>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int ITER = 1024;
constexpr int NK = 33;
static const char* kNames[NK] = {
    "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshlrev_b32", "v_ashrrev_i32",
    "v_and_or_b32", "v_or3_b32", "v_max_f32_e32", "v_min_f32_e32", "v_max_f32_e64(abs)",
    "v_sub_f32_e64(abs,abs)", "v_mul_f32_e64(abs)", "v_fma_f32(neg)", "v_cndmask_b32_e32(vcc, invariant)",
    "v_cndmask_b32_e64(sgpr, invariant)", "v_cmp_gt_f32_e64(own sgpr pair per chain)", "v_rcp_f32",
    "v_cvt_f32_i32", "v_cvt_i32_f32", "v_ldexp_f32", "v_med3_f32", "v_bfe_u32", "v_perm_b32",
    "v_add3_u32", "v_mul_u32_u24", "v_pk_add_f32", "v_pk_mul_f32", "v_mov_b32_dpp(row_mirror)",
    "v_fmac_f32_e32", "v_mul_f32_e64(omod div:2)", "v_xad_u32", "v_lshl_or_b32", "v_max3_f32(no mods)"};

template <int KIND, int CHAINS>
__global__ __launch_bounds__(256) void k_valu(float* out, unsigned long long* clk, float seed) {
    float a[8];
    f2 p[8];
    unsigned long long cm[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = seed + threadIdx.x * 1e-3f + j;
        p[j] = f2{a[j], a[j] + 0.5f};
        cm[j] = 0;
    }
    const float c1 = seed * 0.999f, c2 = seed * 1e-3f;
    const unsigned u1 = 0x3f800000u ^ (unsigned)(seed > 2.0f), u2 = 0x80000000u | (unsigned)(seed > 3.0f);
    const f2 q1 = f2{c1, c1 * 0.5f};
    // a loop-invariant lane mask, made by a compare the compiler sees (lane parity)
    unsigned long long mask;
    asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(mask) : "v"((float)(threadIdx.x & 1)), "v"(0.5f));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (KIND == 13) asm volatile("s_mov_b64 vcc, %0" :: "s"(mask) : "vcc");
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int j = 0; j < CHAINS; ++j) {
                if (KIND == 0) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[j]) : "v"(u1));
                if (KIND == 1) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[j]) : "v"(u1));
                if (KIND == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(u1));
                if (KIND == 3) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a[j]));
                if (KIND == 4) asm volatile("v_ashrrev_i32 %0, 1, %0" : "+v"(a[j]));
                if (KIND == 5) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(u2), "v"(u1));
                if (KIND == 6) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(u2), "v"(u1));
                if (KIND == 7) asm volatile("v_max_f32_e32 %0, %0, %1" : "+v"(a[j]) : "v"(c1));
                if (KIND == 8) asm volatile("v_min_f32_e32 %0, %0, %1" : "+v"(a[j]) : "v"(c1));
                if (KIND == 9) asm volatile("v_max_f32_e64 %0, |%0|, |%1|" : "+v"(a[j]) : "v"(c1));
                if (KIND == 10) asm volatile("v_sub_f32_e64 %0, |%0|, |%1|" : "+v"(a[j]) : "v"(c1));
                if (KIND == 11) asm volatile("v_mul_f32_e64 %0, |%0|, %1" : "+v"(a[j]) : "v"(c1));
                if (KIND == 12) asm volatile("v_fma_f32 %0, -%0, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
                if (KIND == 13) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c1));
                if (KIND == 14) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c1), "s"(mask));
                if (KIND == 15) asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(cm[j]) : "v"(a[j]), "v"(c1));
                if (KIND == 16) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[j]));
                if (KIND == 17) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(a[j]));
                if (KIND == 18) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a[j]));
                if (KIND == 19) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(a[j]) : "v"(1));
                if (KIND == 20) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
                if (KIND == 21) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(a[j]));
                if (KIND == 22) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(u1), "v"(0x05040100u));
                if (KIND == 23) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(u1), "v"(u2));
                if (KIND == 24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(u1));
                if (KIND == 25) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[j]) : "v"(q1));
                if (KIND == 26) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[j]) : "v"(q1));
                if (KIND == 27) asm volatile("v_mov_b32_dpp %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(a[j]));
                if (KIND == 28) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
                if (KIND == 29) asm volatile("v_mul_f32_e64 %0, %0, %1 div:2" : "+v"(a[j]) : "v"(c1));
                if (KIND == 30) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(u1), "v"(u2));
                if (KIND == 31) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a[j]) : "v"(u1));
                if (KIND == 32) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c1), "v"(c2));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + p[j].x + p[j].y + (float)(cm[j] & 1);
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
    const double per_simd = (double)grid * 4 / 1024.0 * ITER * 8 * CHAINS;
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e-3 * ghz * 1e9 / per_simd;
}

template <int KIND>
static void row(float* out, unsigned long long* clk) {
    const double thr8 = run<KIND, 8>(8, out, clk);
    const double thr1 = run<KIND, 8>(1, out, clk);
    const double lat1 = run<KIND, 1>(1, out, clk);
    printf("{\"instr\": \"%s\", \"issue_cyc_8waves\": %.2f, \"issue_cyc_1wave\": %.2f, \"dep_chain_cyc_1wave\": %.2f}\n",
           kNames[KIND], thr8, thr1, lat1);
    fflush(stdout);
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
