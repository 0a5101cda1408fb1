// pv_device.hpp — CDNA4 device building blocks of the phase-vocoder hot path.
//
// One frame per wavefront: the L complex points of a frame's FFT live in the 64 lanes'
// registers (E = L/64 per lane) and in one per-wave LDS tile between passes.  Each pass
// performs log2(E) radix-2 Stockham stages entirely in registers; a pass is exactly the
// composition of the radix-2 stages of hpfft.cu:145-167 (same butterfly, same tabled
// twiddle per butterfly), so the result is bit-identical to the oracle's radix-2
// restatement (oracle/pvref.c pvr_fft_c32) — only the LDS round trips are removed.
//
// Compiled with -ffp-contract=off: every fp32 operation below is the one written, and
// fmaf() marks the fused operations of the numerical contract.
#pragma once
#include <hip/hip_runtime.h>

namespace pv {

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }
constexpr int bitrevc(int v, int bits) {
    int r = 0;
    for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
    return r;
}
constexpr int cmin(int a, int b) { return a < b ? a : b; }

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1 (register-array
// indices that must fold to constants, where #pragma unroll may give up on a large body)
template <int I>
struct IC {
    static constexpr int value = I;
};
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(IC<B>{});
        static_for<B + 1, E>(f);
    }
}

// ------------------------------------------------------------------ fp32 contract
constexpr float kHalfPi = 0x1.921fb6p+0f;
constexpr float kPi = 0x1.921fb6p+1f;
constexpr float kTwoPi = 0x1.921fb6p+2f;
constexpr float kInv2Pi = 0x1.45f306p-3f;

// native 2-vector: arithmetic on it selects the packed fp32 VALU ops (v_pk_mul/add/fma_f32)
typedef float f2v __attribute__((ext_vector_type(2)));

// cmul() with packed ops, two VOP3P instructions whose modifiers do the swizzles:
//   p = (b.y * -w.y, b.y * w.x)     v_pk_mul_f32 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]
//   t = (fma(b.x, w.x, p.x), fma(b.x, w.y, p.y))   v_pk_fma_f32 op_sel_hi:[0,1,1]
// (-(b.y w.y) = b.y (-w.y) exactly), i.e. the same roundings as cmul().  CONJ uses
// conj(w) = (w.x, -w.y) through the neg modifiers instead of a register copy.
// Plain C++ vector code makes the compiler materialise the negated / swapped twiddle
// with extra moves, hence the asm.  WS: the twiddle lives in SGPRs (pass 0, tw0).
template <bool CONJ, bool WS = false>
__device__ __forceinline__ f2v cmul_v(f2v b, f2v w) {
    f2v p, t;
    if constexpr (!CONJ) {
        if constexpr (WS) {
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(p) : "v"(b), "s"(w));
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(b), "s"(w), "v"(p));
        } else {
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(p) : "v"(b), "v"(w));
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(b), "v"(w), "v"(p));
        }
    } else {
        // w' = (w.x, -w.y): p = (b.y w.y, b.y w.x), t = (fma(b.x, w.x, p.x), fma(b.x, -w.y, p.y))
        if constexpr (WS) {
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(p) : "v"(b), "s"(w));
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(t) : "v"(b), "s"(w), "v"(p));
        } else {
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(p) : "v"(b), "v"(w));
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(t) : "v"(b), "v"(w), "v"(p));
        }
    }
    return t;
}

// top + (bot.y, -bot.x) [NEG = false] or top - (bot.y, -bot.x) = top + (-bot.y, bot.x)
// [NEG = true]: the -i (or +i) butterfly of stage Ns = 2 with the swap and sign in the
// VOP3P modifiers; each lane op is the single rounding of the scalar form.
template <bool NEG>
__device__ __forceinline__ f2v pk_add_swp(f2v top, f2v bot) {
    f2v r;
    if constexpr (!NEG)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(top), "v"(bot));
    else
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(top), "v"(bot));
    return r;
}

// LDS loads the compiler must not pair into ds_read2_b32/_b64: a paired read costs 4x the
// LDS cycles of the same bytes as ds_read_b64 (MI355X_MICROARCH.md §LDS).  Volatile
// accesses are never merged; they still schedule freely against non-volatile code.
#define PV_LDS __attribute__((address_space(3)))
__device__ __forceinline__ float2 lds_ld(const float2* p) {
    const f2v v = *(const volatile PV_LDS f2v*)(p);  // explicit LDS: volatile blocks the
    return make_float2(v.x, v.y);                      // generic->LDS address-space inference
}
__device__ __forceinline__ float lds_ld(const float* p) { return *(const volatile PV_LDS float*)(p); }
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) { return *(const volatile PV_LDS unsigned*)(p); }
__device__ __forceinline__ int lds_ld(const int* p) { return *(const volatile PV_LDS int*)(p); }
typedef int i2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i2v lds_ld2i(const int* p) {  // 8-byte aligned pair
    return *(const volatile PV_LDS i2v*)(p);
}

// ---------------------------------------------------------------------------
// Self-tracked prefetch.  vmcnt counts loads and stores together in issue order and the
// compiler's wait insertion merges paths conservatively, which in a frame loop turns
// "wait for the prefetched samples" into "drain the previous frame's stores too".  These
// loads are invisible to the compiler's wait insertion; the caller issues them, then
// exactly K unconditional stores, then vm_wait<K>, all within one loop trip (so the
// registers are never copied or spilled while the loads are in flight; check
// "VGPRs Spill: 0" in the resource-usage report).
template <int E, bool NT = false>
__device__ __forceinline__ void gload_pairs(f2v (&xr)[E], const float* src) {
#pragma unroll
    for (int q = 0; q < E; ++q) {
        const float* pq = src + 1024 * (q >> 3);  // 13-bit signed immediate offsets
        if constexpr (NT)
            asm volatile("global_load_dwordx2 %0, %1, off offset:%2 nt"
                         : "=v"(xr[q]) : "v"(pq), "n"(512 * (q & 7)) : "memory");
        else
            asm volatile("global_load_dwordx2 %0, %1, off offset:%2"
                         : "=v"(xr[q]) : "v"(pq), "n"(512 * (q & 7)) : "memory");
    }
}
// the last D pairs of gload_pairs<E>: registers q = E-D .. E-1 (plain loads: non-temporal
// ones measured +0.1 %, noise)
template <int D, int E>
__device__ __forceinline__ void gload_tail(f2v (&xr)[D], const float* src) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
        constexpr int Q0 = E - D;
        const int q = Q0 + j;
        const float* pq = src + 1024 * (q >> 3);
        asm volatile("global_load_dwordx2 %0, %1, off offset:%2"
                     : "=v"(xr[j]) : "v"(pq), "n"(512 * (q & 7)) : "memory");
    }
}
// one spectrum row: bins lane + 64 q (q < E) from rowlane = row + lane, and (bin_l) bin L
// (the same address on every lane) from rowL.  Rows are read exactly once: NT streams them
// past the caches (measured +0.4 % on config 3).
template <int E, bool NT = true>
__device__ __forceinline__ void gload_row(f2v (&v)[E + 1], const float2* rowlane, const float2* rowL,
                                          bool bin_l = true) {
    f2v (&head)[E] = *reinterpret_cast<f2v(*)[E]>(&v[0]);
    gload_pairs<E, NT>(head, reinterpret_cast<const float*>(rowlane));
    if (bin_l) {
        if constexpr (NT)
            asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(v[E]) : "v"(rowL) : "memory");
        else
            asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v[E]) : "v"(rowL) : "memory");
    }
}

// PV_SPEC_PACKED slot value of a real bin (bins 0 and L: Im = +0, so the contract's phase is
// +0 or pi): the magnitude with the sign bit set for phase pi
__device__ __forceinline__ float pack_real_bin(float mag, float ph) { return ph > 0.0f ? -mag : mag; }
// slot 0 {s0, sL} -> {mag, phase} of bins 0 and L: the magnitude is the sign-free value, the
// phase +0 or pi by the sign bit (exactly the analysis's phases)
__device__ __forceinline__ void unpack_real_bins(float2 s, float2& b0, float2& bL) {
    constexpr float pi = 0x1.921fb6p+1f;  // kPi (declared below)
    const float p0 = (__float_as_uint(s.x) >> 31) ? pi : 0.0f;
    const float pL = (__float_as_uint(s.y) >> 31) ? pi : 0.0f;
    b0 = make_float2(__builtin_fabsf(s.x), p0);
    bL = make_float2(__builtin_fabsf(s.y), pL);
}
template <int K, int E>
__device__ __forceinline__ void vm_wait(f2v (&xr)[E]) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(K) : "memory");
#pragma unroll
    for (int q = 0; q < E; ++q) asm volatile("" : "+v"(xr[q]));  // uses stay after the wait
}

// Lane 0 only: (bx, by) <- (ax, ay) by two v_mov_b32 under exec & 1 (the lane-0 partner fix-up
// of the real-FFT splits, whose partner bins are lane 0's own registers).  A v_mov issues at
// the full VALU rate, a v_cndmask_b32 select at half (profiles/r04_valu_probe3.jsonl: 2.25 vs
// 4.15 cycles per wave-instruction); exec is restored, and lane 0 is only written if active.
__device__ __forceinline__ void lane0_mov2(float& bx, float& by, float ax, float ay) {
#ifndef PV_LANE0_SELECT  // (A/B build: the select form)
    unsigned long long saved;
    asm("s_mov_b64 %2, exec\n\t"
        "s_and_b64 exec, exec, 1\n\t"
        "v_mov_b32 %0, %3\n\t"
        "v_mov_b32 %1, %4\n\t"
        "s_mov_b64 exec, %2"
        : "+v"(bx), "+v"(by), "=&s"(saved) : "v"(ax), "v"(ay) : "scc");  // s_and_b64 writes SCC
#else
    const bool l0 = __lane_id() == 0;
    bx = l0 ? ax : bx;
    by = l0 ? ay : by;
#endif
}

__device__ __forceinline__ float2 cmul(float2 b, float2 w) {
    float2 t;
    t.x = __builtin_fmaf(b.x, w.x, -(b.y * w.y));
    t.y = __builtin_fmaf(b.x, w.y, b.y * w.x);
    return t;
}

// atan2 of the contract (oracle pvr_atan2f); atan(a) = a*P(a^2), |err| <= 2.7e-7 rad.
// Zero bins: +-0 (the sign of y); y = -0 gives -phase like C's atan2.
__device__ __forceinline__ float atan2_pv(float y, float x) {
    float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
    // max/min of |x|, |y| as single instructions with abs modifiers (fmaxf/fminf make
    // the compiler canonicalise operands it cannot prove canonical, e.g. asm results);
    // identical values for non-NaN inputs
// mx is floored at FLT_MIN (contract): an all-zero bin gets a = 0 and phase +-0 with
    // no special case
    float mx, mn;
    asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(mx) : "v"(x), "v"(y), "s"(0x1p-126f));
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(mn) : "v"(x), "v"(y));
    // a = mn / mx by the contract's division-free reciprocal (oracle pvr_atan2f): integer
    // seed + a cubic and a Newton fmaf step + one product (7 VALU, no v_rcp / div_scale chain)
    float r = __uint_as_float(0x7EF311C3u - __float_as_uint(mx));
    float e = __builtin_fmaf(-mx, r, 1.0f);  // contract v3: a cubic step, then a Newton step
    const float e2 = __builtin_fmaf(e, e, e);
    r = __builtin_fmaf(r, e2, r);
    e = __builtin_fmaf(-mx, r, 1.0f);
    r = __builtin_fmaf(r, e, r);
    // contract v4: a = clamp(mn r, 0, 1) by the output modifier (DX10 clamp: NaN -> 0, the
    // kernels' default mode), so the phase is finite for any input: no unwrap decision of a
    // non-finite bin corrupts the channel's run sums
    float a;
    asm("v_mul_f32_e64 %0, %1, %2 clamp" : "=v"(a) : "v"(mn), "v"(r));
    float s = a * a;
    float p = -0x1.8ba68ap-10f;
    p = __builtin_fmaf(p, s, 0x1.398008p-7f);
    p = __builtin_fmaf(p, s, -0x1.d2ca58p-6f);
    p = __builtin_fmaf(p, s, 0x1.c2c9f4p-5f);
    p = __builtin_fmaf(p, s, -0x1.506f6cp-4f);
    p = __builtin_fmaf(p, s, 0x1.bd9028p-4f);
    p = __builtin_fmaf(p, s, -0x1.23c87ap-3f);
    p = __builtin_fmaf(p, s, 0x1.9986ecp-3f);
    p = __builtin_fmaf(p, s, -0x1.5554eep-2f);
    p = __builtin_fmaf(p, s, 0x1.000000p+0f);
    float rr = a * p;
    if (ay > ax) rr = kHalfPi - rr;
    if (x < 0.0f) rr = kPi - rr;
    return __builtin_copysignf(rr, y);  // rr >= 0 here: the sign of y (v_bfi_b32)
}

// atan2_pv of two bins at once: the same operations on each half of a register pair, the
// Newton steps and the polynomial as v_pk_fma_f32 / v_pk_mul_f32 (each half rounds exactly
// like the scalar op, so both results are atan2_pv's bit for bit): 18 VALU fewer per pair.
// The min/max, the seeds and the octant fix-ups stay scalar on the halves (no packed forms;
// they read and write the pair's registers directly, no moves).
__device__ __forceinline__ f2v atan2_pv2(float y0, float x0, float y1, float x1) {
    f2v mx, mn, r;
    float t0, t1, u0, u1;
    asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(t0) : "v"(x0), "v"(y0), "s"(0x1p-126f));
    asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(t1) : "v"(x1), "v"(y1), "s"(0x1p-126f));
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(u0) : "v"(x0), "v"(y0));
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(u1) : "v"(x1), "v"(y1));
    mx = f2v{t0, t1};
    mn = f2v{u0, u1};
    r = f2v{__uint_as_float(0x7EF311C3u - __float_as_uint(t0)), __uint_as_float(0x7EF311C3u - __float_as_uint(t1))};
    const f2v one = f2v{1.0f, 1.0f};
    f2v e = __builtin_elementwise_fma(-mx, r, one);  // contract v3: cubic step + Newton step
    const f2v e2 = __builtin_elementwise_fma(e, e, e);
    r = __builtin_elementwise_fma(r, e2, r);
    e = __builtin_elementwise_fma(-mx, r, one);
    r = __builtin_elementwise_fma(r, e, r);
    f2v a;  // contract v4: clamp(mn r, 0, 1), NaN -> 0 (atan2_pv)
    asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(a) : "v"(mn), "v"(r));
    const f2v sq = a * a;
    auto c = [](float v) { return f2v{v, v}; };
    f2v p = c(-0x1.8ba68ap-10f);
    p = __builtin_elementwise_fma(p, sq, c(0x1.398008p-7f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.d2ca58p-6f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.c2c9f4p-5f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.506f6cp-4f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.bd9028p-4f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.23c87ap-3f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.9986ecp-3f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.5554eep-2f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.000000p+0f));
    const f2v rr = a * p;
    float r0 = rr.x, r1 = rr.y;
    if (__builtin_fabsf(y0) > __builtin_fabsf(x0)) r0 = kHalfPi - r0;
    if (__builtin_fabsf(y1) > __builtin_fabsf(x1)) r1 = kHalfPi - r1;
    if (x0 < 0.0f) r0 = kPi - r0;
    if (x1 < 0.0f) r1 = kPi - r1;
    return f2v{__builtin_copysignf(r0, y0), __builtin_copysignf(r1, y1)};
}

// REF_COMPAT's atanf(y / x) (kernel.cu:101-109, range (-pi/2, pi/2]: the quadrant is lost)
// without the division, for a pair of bins: atan2_pv2's reduction and polynomial without
// its x < 0 fix-up, signed by sign(x) * sign(y) (y / x of signed zeros and infinities
// included: 0 / -0 -> -0 ... and +-y / 0 -> +-pi/2 with the signs of the quotient).
// Within 2.7e-7 rad of atanf; REF_COMPAT parity is tolerance based.  x = y = 0 gives +-0
// (the caller substitutes the reference's NaN when asked).
__device__ __forceinline__ f2v atan_ratio_pv2(float y0, float x0, float y1, float x1) {
    f2v mx, mn, r;
    float t0, t1, u0, u1;
    asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(t0) : "v"(x0), "v"(y0), "s"(0x1p-126f));
    asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(t1) : "v"(x1), "v"(y1), "s"(0x1p-126f));
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(u0) : "v"(x0), "v"(y0));
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(u1) : "v"(x1), "v"(y1));
    mx = f2v{t0, t1};
    mn = f2v{u0, u1};
    r = f2v{__uint_as_float(0x7EF311C3u - __float_as_uint(t0)), __uint_as_float(0x7EF311C3u - __float_as_uint(t1))};
    const f2v one = f2v{1.0f, 1.0f};
    f2v e = __builtin_elementwise_fma(-mx, r, one);  // contract v3: cubic step + Newton step
    const f2v e2 = __builtin_elementwise_fma(e, e, e);
    r = __builtin_elementwise_fma(r, e2, r);
    e = __builtin_elementwise_fma(-mx, r, one);
    r = __builtin_elementwise_fma(r, e, r);
    const f2v a = mn * r;
    const f2v sq = a * a;
    auto c = [](float v) { return f2v{v, v}; };
    f2v p = c(-0x1.8ba68ap-10f);
    p = __builtin_elementwise_fma(p, sq, c(0x1.398008p-7f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.d2ca58p-6f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.c2c9f4p-5f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.506f6cp-4f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.bd9028p-4f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.23c87ap-3f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.9986ecp-3f));
    p = __builtin_elementwise_fma(p, sq, c(-0x1.5554eep-2f));
    p = __builtin_elementwise_fma(p, sq, c(0x1.000000p+0f));
    const f2v rr = a * p;
    float r0 = rr.x, r1 = rr.y;
    if (__builtin_fabsf(y0) > __builtin_fabsf(x0)) r0 = kHalfPi - r0;
    if (__builtin_fabsf(y1) > __builtin_fabsf(x1)) r1 = kHalfPi - r1;
    // sign of y / x: sign bit of y XOR sign bit of x
    const unsigned s0 = (__float_as_uint(y0) ^ __float_as_uint(x0)) & 0x80000000u;
    const unsigned s1 = (__float_as_uint(y1) ^ __float_as_uint(x1)) & 0x80000000u;
    return f2v{__uint_as_float(__float_as_uint(r0) | s0), __uint_as_float(__float_as_uint(r1) | s1)};
}

// sin/cos of 2 pi rev: the hardware v_sin_f32 / v_cos_f32 (inputs in revolutions,
// quarter-rate transcendental; they reduce their input themselves over [-256, 256]
// revolutions, and every caller passes |rev| < 4: output phases are carried reduced;
// measured: synthesis -2.5 % against an explicit rev - rint(rev)).  Synthesis parity is
// tolerance based; the GPU tests bound the end-to-end error.
__device__ __forceinline__ void sincos_rev(float rev, float* sn, float* cs) {
    *sn = __builtin_amdgcn_sinf(rev);
    *cs = __builtin_amdgcn_cosf(rev);
}

// |X| from |2X|^2 = fma(2X.re, 2X.re, (2X.im)^2) (the analysis' doubled split): hardware
// v_sqrt_f32 (<= 1 ulp), halved exactly
__device__ __forceinline__ float half_sqrt(float s2) { return 0.5f * __builtin_amdgcn_sqrtf(s2); }

// unwrap decision of the contract (oracle pvr_unwrap_count, contract v2): the exact product
// d * (1/2pi) rounded once onto the integer grid of [2^23, 2^24) by an fma with the magic
// 1.5 * 2^23 (ties to even, as rint: the magic is even); t - magic is then exact.  Two fast
// VALU operations instead of a multiply and a (quarter-rate) v_rndne.
constexpr float kRintMagic = 0x1.8p23f;
constexpr unsigned kRintMagicBits = 0x4B400000u;
// t = magic + rint(d / 2pi): the decision's bits (m = -(bits(t) - kRintMagicBits))
__device__ __forceinline__ float unwrap_t(float phi, float phi_prev, float e) {
    const float d = (phi - phi_prev) - e;
    return __builtin_fmaf(d, kInv2Pi, kRintMagic);
}
// rint of the scaled deviation as a float: m = -unwrap_round(...) (exact small integer)
__device__ __forceinline__ float unwrap_round(float phi, float phi_prev, float e) {
    return unwrap_t(phi, phi_prev, e) - kRintMagic;
}
__device__ __forceinline__ int unwrap_count(float phi, float phi_prev, float e) {
    return -(int)(__float_as_uint(unwrap_t(phi, phi_prev, e)) - kRintMagicBits);
}

// ------------------------------------------------------------------ wave-local LDS sync
// A frame's LDS tile is private to one wave and the LDS executes one wave's DS
// instructions in issue order, so a cross-lane exchange (ds_write by lane a, later
// ds_read by lane b) needs no s_waitcnt: only the compiler must keep program order,
// which the memory clobber enforces.
// s_waitcnt immediate for vmcnt(0) alone (gfx9 encoding: vmcnt [3:0] and [15:14] = 0,
// expcnt [6:4] = 7 and lgkmcnt [11:8] = 15 mean "no wait"); as a builtin, unlike inline asm,
// the compiler's wait insertion sees it
constexpr int kVmcnt0 = 0x0F70;

__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------ FFT geometry
// LDS tile layouts.  A frame's tile carries NPASS - 1 inter-pass exchanges (pass P stores,
// pass P + 1 loads) and the final natural-order image (last pass stores; the real split,
// the synthesis' time samples and the FFT op read it).  Each has its own layout, chosen by
// a bank-conflict model of its exact access shapes (MI355X_MICROARCH.md §LDS: ds_read_b64
// in 2 x 32 lanes over 64 banks, ds_write_b64 in 4 x 16 lanes over 32 banks):
//   exchange X: slot(p) = p + XC * (p >> XS)   (XC pad slots every 2^XS points)
//   final image: slot(p) = p                   (contiguous and mirrored 32-lane reads and
//                                               the last pass's contiguous stores are all
//                                               conflict-free unpadded)
// At L = 512 this is 176 LDS-array cycles per frame-transform instead of 256 with one pad
// every E points for every image.  Every access is still one per-lane base plus
// compile-time offsets: slot(a + c) = slot(a) + slot(c) for all (a, c) the passes use.
constexpr int lay_c(int L, int X) {
    return L == 128 ? (X == 0 ? 1 : X == 1 ? 2 : X == 2 ? 4 : X == 3 ? 8 : 0)
         : L == 256 ? (X == 0 ? 1 : X == 1 ? 4 : 0)
         : L == 512 ? (X == 0 ? 1 : X == 1 ? 8 : 0)
         : L == 1024 ? (X == 0 ? 1 : 0)
         : (X == 0 ? 1 : 0);
}
constexpr int lay_s(int L, int X) {
    return L == 512 && X == 1 ? 6 : L == 2048 ? 5 : 4;
}
constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <int L_>
struct Geo {
    static constexpr int L = L_;
    static constexpr int LOG2L = ilog2c(L);
    static constexpr int E = L / 64;                 // complex points per lane
    static constexpr int RLOG = ilog2c(E);           // stages per full pass
    static constexpr int NPASS = (LOG2L + RLOG - 1) / RLOG;
    static_assert(L >= 128 && L <= 2048, "one frame per wave: L in [128, 2048]");
    // exchange X's slot of point p (constexpr: offsets fold into the instruction)
    template <int X>
    __host__ __device__ static constexpr int xslot(int p) {
        return p + lay_c(L, X) * (p >> lay_s(L, X));
    }
    static constexpr int xsize(int X) { return (L - 1) + lay_c(L, X) * ((L - 1) >> lay_s(L, X)) + 1; }
    static constexpr int max_xsize() {
        int m = L;
        for (int X = 0; X + 1 < NPASS; ++X) m = cmax(m, xsize(X));
        return m;
    }
    static constexpr int TILE = max_xsize() + 2;  // LDS tile (float2), +bin L
    // every exchange layout must keep "per-lane base + compile-time offset" exact for the
    // address pairs pass_store / pass_load form (checked at compile time below)
    static constexpr bool layouts_affine() {
        for (int P = 0; P + 1 < NPASS; ++P) {
            const int S = 1 << (P * RLOG);
            const int r = cmin(RLOG, LOG2L - P * RLOG), R = 1 << r;
            const int r2 = cmin(RLOG, LOG2L - (P + 1) * RLOG), R2 = 1 << r2;
            const int c = lay_c(L, P), s = lay_s(L, P);
            auto sl = [&](int p) { return p + c * (p >> s); };
            for (int j = 0; j < L / R; ++j) {
                const int J = (j / S) * R * S + (j & (S - 1));
                for (int f = 0; f < R; ++f) {
                    const int off = S * bitrevc(f, r);
                    if (sl(J + off) != sl(J) + sl(off)) return false;
                }
            }
            for (int lane = 0; lane < 64; ++lane)
                for (int g = 0; g < E / R2; ++g)
                    for (int q = 0; q < R2; ++q) {
                        const int off = 64 * g + q * (L / R2);
                        if (sl(lane + off) != sl(lane) + sl(off)) return false;
                    }
        }
        return true;
    }

    // final natural-order image: unpadded
    __device__ static __forceinline__ int pad(int p) { return p; }
    static constexpr int padc(int c) { return c; }
};
static_assert(Geo<128>::layouts_affine() && Geo<256>::layouts_affine() && Geo<512>::layouts_affine() &&
                  Geo<1024>::layouts_affine() && Geo<2048>::layouts_affine(),
              "tile layout breaks base + offset addressing");

// Stage-major twiddle table: stage Ns occupies [Ns-1, 2Ns-1), entry idx = e^{-i pi idx/Ns}
// (the values of the oracle's master table tw[idx*L/(2Ns)], copied, so bit-identical).

// One register pass: P-th pass, INV selects conjugated twiddles.
// Input layout : v[g*R + q] = x[j + q*L/R],   j = lane + 64 g
// Output layout: v[g*R + f] = y[(j/S)*R*S + j%S + S*bitrev_r(f)]
// TWS_MIN > 0: stages Ns >= TWS_MIN read W(m, Ns) = e^{-2 pi i m / 2Ns} from the split
// table tws (e^{-2 pi i k / 2L}, k <= L) at k = m L / Ns instead of the stage-major table:
// both are tw_entry() of the same double angle (2 pi m / 2Ns and 2 pi (m L/Ns) / 2L differ
// by a power-of-two scaling of numerator and denominator, exact), so the values are the
// same bits and the stage-major table only needs its first TWS_MIN - 1 entries in LDS.
template <int L, int P, bool INV, int TWS_MIN = 0>
__device__ __forceinline__ void fft_pass(float2 (&v)[Geo<L>::E], const float2* tw,
                                         const float2 (&tw0)[Geo<L>::E], int lane,
                                         const float2* tws = nullptr) {
    using G_ = Geo<L>;
    constexpr int S = 1 << (P * G_::RLOG);
    constexpr int r = cmin(G_::RLOG, G_::LOG2L - P * G_::RLOG);
    constexpr int R = 1 << r;
    constexpr int NG = G_::E / R;
    constexpr int E = G_::E;
    // the stages run on native 2-vectors (64-bit register pairs), so the packed operations
    // need no register moves to assemble their operands.  Stage-major over the NG groups of
    // R points: a stage's LDS twiddles for every group (2^st distinct per group: R / 2
    // butterflies share them) are read once, as one batch, before its butterflies — at most
    // 8 per batch, else group by group.  The LDS loads are volatile, so per-butterfly reads
    // were never merged (at L = 1024: 32 serialized round trips in pass 1 and 8 in pass 2
    // instead of 4 and 2 batched ones).  Each group's operations are unchanged.
    f2v a[E];
#pragma unroll
    for (int q = 0; q < E; ++q) a[q] = f2v{v[q].x, v[q].y};
#pragma unroll
    for (int st = 0; st < r; ++st) {
        const int Ns = S << st;
        const bool lds_tw = (P > 0) && Ns > 2;
        const bool batch_all = NG * (1 << st) <= 8;
        float2 wst[NG][R / 2];
        auto load_tw = [&](int g) {
            const int jm = (lane + 64 * g) & (S - 1);
#pragma unroll
            for (int bb = 0; bb < (1 << st); ++bb)
                wst[g][bb] = (TWS_MIN > 0 && Ns >= TWS_MIN) ? lds_ld(&tws[(jm + S * bb) * (L / Ns)])
                                                             : lds_ld(&tw[(Ns - 1) + jm + S * bb]);
        };
        if (lds_tw && batch_all) {
#pragma unroll
            for (int g = 0; g < NG; ++g) load_tw(g);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int jm = (lane + 64 * g) & (S - 1);
            if (lds_tw && !batch_all) load_tw(g);
            f2v b[R];
#pragma unroll
            for (int s = 0; s < R / 2; ++s) {
                const int br = bitrevc(s & ((1 << st) - 1), st);
                // pass 0: jm = 0, S = 1: compile-time index into the hoisted tw0 (SGPRs)
                // packed (v_pk_*) form of cmul + butterfly, same roundings as cmul();
                // INV multiplies by conj(w)
                const f2v top = a[g * R + s];
                const f2v bot = a[g * R + s + R / 2];
                if (P == 0 && Ns == 2 && br != 0) {  // compile-time in pass 0
                    // W = exactly -i (+i when INV): top +- (bot.y, -bot.x) as two packed adds
                    // whose op_sel / neg modifiers swap and negate bot (no register moves)
                    if constexpr (!INV) {
                        b[2 * s] = pk_add_swp<false>(top, bot);
                        b[2 * s + 1] = pk_add_swp<true>(top, bot);
                    } else {
                        b[2 * s] = pk_add_swp<true>(top, bot);
                        b[2 * s + 1] = pk_add_swp<false>(top, bot);
                    }
                    continue;
                }
                f2v t;
                if (Ns == 1 || (P == 0 && Ns == 2)) {
                    t = bot;  // W = 1 exactly (fp32 contract)
                } else if (Ns == 2) {
                    // later pass (L = 128): W = 1 or exactly -i (+i when INV) by lane
                    const f2v rr = INV ? f2v{-bot.y, bot.x} : f2v{bot.y, -bot.x};
                    t = (jm != 0) ? rr : bot;
                } else if constexpr (P == 0) {
                    const float2 w = tw0[(Ns - 1) + br];
                    t = cmul_v<INV, true>(bot, f2v{w.x, w.y});
                } else {
                    const float2 w = wst[g][br];
                    t = cmul_v<INV, false>(bot, f2v{w.x, w.y});
                }
                b[2 * s] = top + t;
                b[2 * s + 1] = top - t;
            }
#pragma unroll
            for (int q = 0; q < R; ++q) a[g * R + q] = b[q];
        }
    }
#pragma unroll
    for (int q = 0; q < E; ++q) v[q] = make_float2(a[q].x, a[q].y);
}

template <int L, int P>
__device__ __forceinline__ void pass_store(const float2 (&v)[Geo<L>::E], float2* tile, int lane) {
    using G_ = Geo<L>;
    constexpr int S = 1 << (P * G_::RLOG);
    constexpr int r = cmin(G_::RLOG, G_::LOG2L - P * G_::RLOG);
    constexpr int R = 1 << r;
    constexpr int NG = G_::E / R;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int j = lane + 64 * g;
        const int J = (j / S) * R * S + (j & (S - 1));
        // inter-pass exchange P, or the final image after the last pass
        constexpr bool FIN = (P + 1 == G_::NPASS);
        float2* base = tile + (FIN ? J : G_::template xslot<(FIN ? 0 : P)>(J));
#pragma unroll
        for (int f = 0; f < R; ++f) {
            const int off = S * bitrevc(f, r);
            base[FIN ? off : G_::template xslot<(FIN ? 0 : P)>(off)] = v[g * R + f];
        }
    }
}

template <int L, int P>
__device__ __forceinline__ void pass_load(float2 (&v)[Geo<L>::E], const float2* tile, int lane) {
    using G_ = Geo<L>;
    constexpr int r = cmin(G_::RLOG, G_::LOG2L - P * G_::RLOG);
    constexpr int R = 1 << r;
    constexpr int NG = G_::E / R;
    static_assert(P >= 1, "pass 0 reads registers");
    const float2* base = tile + G_::template xslot<P - 1>(lane);  // exchange P - 1
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
        for (int q = 0; q < R; ++q) v[g * R + q] = lds_ld(&base[G_::template xslot<P - 1>(64 * g + q * (L / R))]);
    }
}

// Pass-0 twiddles (stage-major entries 0..E-2): wave-uniform, loaded once per kernel from
// global memory so they live in SGPRs (s_load) instead of costing LDS reads every frame.
template <int L>
__device__ __forceinline__ void load_tw0(float2 (&tw0)[Geo<L>::E], const float2* __restrict__ tw) {
#pragma unroll
    for (int i = 0; i + 1 < Geo<L>::E; ++i) tw0[i] = tw[i];
    tw0[Geo<L>::E - 1] = make_float2(1.0f, 0.0f);
}

// Full FFT: v holds the pass-0 input layout (x[lane + 64 q], since R0 = E).  With
// STORE_LAST the result is left in `tile` in natural order (padded indexing); without it
// the last pass's output stays in v, where register v[g*R + f] holds point
// lane + 64 g + S_last * bitrev_r(f)  (= lane + 64 c, see last_slot()).
// ------------------------------------------------------------------ FFT contract v3
// For L in [128, 512] (E = L/64 <= 8) a pass is one twiddle-first radix-R Stockham step per
// group (oracle pvr_fft_c32_v3): the R points a_q (q >= 1) are multiplied by the pass-table
// twiddles T_P[m][q] = e^{-+2 pi i m q/(R S)}, m = j mod S (none in pass 0), then an R-point
// DIF whose internal twiddles are compile-time: 1, -i (a swapped, negated difference: the
// op_sel / neg modifiers of one v_pk_add), W8 and W8^3 (a swizzled v_pk_add and a v_pk_mul by
// 1/sqrt 2).  Register f ends up holding y_{bitrev(f)}: the same output layout as the radix-2
// stages (pass_store / last_slot unchanged).  Per L = 512 transform: 112 packed operations
// instead of 128 (radix-2 stages: a table twiddle per butterfly).  (Folding the analysis
// window into pass 0's first stage saves 4 more but holds the window pairs in 9 more VGPRs:
// the analysis drops to 4 waves/SIMD, measured slower.)  L >= 1024 keeps the radix-2 stages:
// its last pass would need an S (R - 1) ~ L-entry table, which costs the analysis a workgroup
// per CU of LDS.
// X: also at L = 1024 (radices 16, 16, 4; the batched synthesis's inverse transform, which no
// contract binds — its table is pv_api.cpp's second d_tw_syn block)
template <int L, bool X = false>
constexpr bool fft_v3() { return (L >= 128 && L <= 512) || (X && L == 1024); }
// pass table offset of pass P >= 1: sum over 1 <= P' < P of S_P' (R_P' - 1)
template <int L>
constexpr int v3_off(int P) {
    int off = 0;
    for (int p = 1; p < P; ++p) {
        const int S = 1 << (p * Geo<L>::RLOG);
        const int R = 1 << cmin(Geo<L>::RLOG, Geo<L>::LOG2L - p * Geo<L>::RLOG);
        off += S * (R - 1);
    }
    return off;
}
constexpr float kW8c = 0x1.6a09e6p-1f;  // (float)(1/sqrt 2), oracle PVR_W8C

// (u - v) * (-i) (forward) or * (+i) (inverse): one v_pk_add, each half a single rounding
template <bool INV>
__device__ __forceinline__ f2v pk_rot_sub(f2v u, f2v v) {
    f2v d;
    if constexpr (!INV)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[0,1] neg_hi:[1,0]" : "=v"(d) : "v"(u), "v"(v));
    else
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(u), "v"(v));
    return d;
}
// e * W8 (W8 = e^{-i pi/4}; conj when INV) or e * W8^3: the swizzled sum s of the oracle's
// dif_v3, then s * (1/sqrt 2)
template <bool W83, bool INV>
__device__ __forceinline__ f2v pk_w8(f2v e) {
    f2v sw, d;
    if constexpr (!W83 && !INV)  // (e.x + e.y, e.y - e.x)
        asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(sw) : "v"(e));
    else if constexpr (!W83 && INV)  // (e.x - e.y, e.x + e.y)
        asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1] neg_lo:[0,1]" : "=v"(sw) : "v"(e));
    else if constexpr (W83 && !INV)  // (e.y - e.x, -e.x - e.y)
        asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(sw) : "v"(e));
    else  // (-e.x - e.y, e.x - e.y)
        asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1] neg_lo:[1,1] neg_hi:[0,1]" : "=v"(sw) : "v"(e));
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(sw), "s"(f2v{kW8c, kW8c}));
    return d;
}

// The R-point DIF of contract v3 on t[0..R-1] (oracle dif_v3)
// e * W16^i, i odd (R = 16 only, outside the contract: W16^{1,3,5,7} = c - i s, s - i c,
// -s - i c, -c - i s with c = cos(pi/8), s = sin(pi/8)); conj when INV
template <int I, bool INV>
__device__ __forceinline__ f2v w16_odd(f2v e) {
    constexpr float c = 0x1.d906bcp-1f, sn = 0x1.87de2ap-2f;
    constexpr float wr = (I == 1) ? c : (I == 3) ? sn : (I == 5) ? -sn : -c;
    constexpr float wi = (I == 1) ? -sn : (I == 3) ? -c : (I == 5) ? -c : -sn;
    return cmul_v<INV, true>(e, f2v{wr, wi});
}

template <int R, bool INV>
__device__ __forceinline__ void dif_v3(f2v* t) {
    static_assert(R == 2 || R == 4 || R == 8 || R == 16, "v3 radices");
    static_for<0, ilog2c(R)>([&](auto sc) {
        constexpr int st = decltype(sc)::value;
        constexpr int h = R >> (st + 1);
        static_for<0, R / 2>([&](auto bc) {
            constexpr int bi = decltype(bc)::value;
            constexpr int b = (bi / h) * 2 * h, i = bi % h;
            const f2v u = t[b + i], v = t[b + i + h];
            f2v d;
            if constexpr (i > 0 && 2 * i == h) {
                d = pk_rot_sub<INV>(u, v);
            } else {
                const f2v e = u - v;
                if constexpr (i == 0) d = e;
                else if constexpr (h == 8 && (i & 1)) d = w16_odd<i, INV>(e);
                else d = pk_w8<(4 * i == 3 * h), INV>(e);
            }
            t[b + i] = u + v;
            t[b + i + h] = d;
        });
    });
}

template <int L, int P, bool INV>
__device__ __forceinline__ void fft_pass_v3(float2 (&v)[Geo<L>::E], const float2* tw, int lane) {
    using G_ = Geo<L>;
    constexpr int S = 1 << (P * G_::RLOG);
    constexpr int r = cmin(G_::RLOG, G_::LOG2L - P * G_::RLOG);
    constexpr int R = 1 << r;
    constexpr int NG = G_::E / R;
    constexpr int E = G_::E;
    f2v a[E];
#pragma unroll
    for (int q = 0; q < E; ++q) a[q] = f2v{v[q].x, v[q].y};
    if constexpr (P > 0) {
        // the pass's (R - 1) NG table twiddles as one batch of LDS reads (volatile: not paired)
        float2 w[NG][R - 1];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int m = (lane + 64 * g) & (S - 1);
            const float2* row = tw + v3_off<L>(P) + m * (R - 1);
#pragma unroll
            for (int q = 1; q < R; ++q) w[g][q - 1] = lds_ld(&row[q - 1]);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int q = 1; q < R; ++q) a[g * R + q] = cmul_v<INV>(a[g * R + q], f2v{w[g][q - 1].x, w[g][q - 1].y});
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) dif_v3<R, INV>(&a[g * R]);
#pragma unroll
    for (int q = 0; q < E; ++q) v[q] = make_float2(a[q].x, a[q].y);
}

template <int L, bool INV, bool STORE_LAST = true, int P = 0, int TWS_MIN = 0, bool V3X = false>
__device__ __forceinline__ void fft_run(float2 (&v)[Geo<L>::E], float2* tile, const float2* tw,
                                        const float2 (&tw0)[Geo<L>::E], int lane,
                                        const float2* tws = nullptr) {
    if constexpr (fft_v3<L, V3X>()) {
        (void)tw0;
        (void)tws;
        fft_pass_v3<L, P, INV>(v, tw, lane);
    } else {
        fft_pass<L, P, INV, TWS_MIN>(v, tw, tw0, lane, tws);
    }
    if constexpr (P + 1 < Geo<L>::NPASS) {
        pass_store<L, P>(v, tile, lane);
        wave_lds_sync();
        pass_load<L, P + 1>(v, tile, lane);
        wave_lds_sync();
        fft_run<L, INV, STORE_LAST, P + 1, TWS_MIN, V3X>(v, tile, tw, tw0, lane, tws);
    } else if constexpr (STORE_LAST) {
        pass_store<L, P>(v, tile, lane);
        wave_lds_sync();
    }
}

// slot c of register idx after the last pass: point = lane + 64 * last_slot(idx)
template <int L>
constexpr int last_slot(int idx) {
    using G_ = Geo<L>;
    constexpr int P = G_::NPASS - 1;
    constexpr int S = 1 << (P * G_::RLOG);
    constexpr int r = G_::LOG2L - P * G_::RLOG;
    constexpr int R = 1 << r;
    const int g = idx / R, f = idx % R;
    return g + (S / 64) * bitrevc(f, r);
}

}  // namespace pv
