/*
 * pvref.c — CPU ORACLE (test infrastructure only; see pvref.h for the contract).
 *
 * Build: oracle/Makefile (gcc, -ffp-contract=off so that every fp32 operation is the one
 * written here; fmaf() is used exactly where the contract says "fused").
 */
#define _GNU_SOURCE
#include "pvref.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PVR_PI_D 3.14159265358979323846

/* fp32 constants of the contract (exact hex values) */
#define PVR_HALF_PI_F 0x1.921fb6p+0f
#define PVR_PI_F 0x1.921fb6p+1f
#define PVR_INV_2PI_F 0x1.45f306p-3f

/* atan(a) = a * P(a^2) on [0,1]; minimax-fitted, |err| <= 2.7e-7 rad */
static const float PVR_ATAN_C[10] = {
    0x1.000000p+0f,  -0x1.5554eep-2f, 0x1.9986ecp-3f,  -0x1.23c87ap-3f, 0x1.bd9028p-4f,
    -0x1.506f6cp-4f, 0x1.c2c9f4p-5f,  -0x1.d2ca58p-6f, 0x1.398008p-7f,  -0x1.8ba68ap-10f};

int pvr_contract_version(void) { return PVR_CONTRACT_VERSION; }

/* ------------------------------------------------------------------ tables */

void pvr_hann_periodic(int N, float* w) {
    /* PV_STANDARD analysis/synthesis window: periodic Hann, as the reference's 1-arg
     * constructor (phaseVocoder.h:64-66) and cudaWindow_HanRT (kernel.cu:85-91) intend;
     * evaluated in double and rounded once. */
    for (int n = 0; n < N; ++n)
        w[n] = (float)(0.5 - 0.5 * cos(2.0 * PVR_PI_D * (double)n / (double)N));
}

void pvr_hamming_ref(int N, float* w) {
    /* phaseVocoder.h:85-89: float omega = 2.f*M_PI/(samples-1);
     * imp[i] = 0.54f - 0.46f*cos(omega*(i));  -- float argument, float overload of cos. */
    float omega = (float)(2.0 * PVR_PI_D / (double)(N - 1));
    for (int i = 0; i < N; ++i) {
        float arg = omega * (float)i;
        w[i] = 0.54f - 0.46f * cosf(arg);
    }
}

void pvr_hann_ref(int N, float* w) {
    /* phaseVocoder.h:64-66, PhaseVocoder(int samples):
     * imp[i] = 0.5f * (1.f - cosf(2.f*M_PI*i / samples));  -- 2.f*M_PI is double, so the
     * argument is evaluated in double and converted to float for cosf. */
    for (int i = 0; i < N; ++i)
        w[i] = 0.5f * (1.f - cosf((float)(2.0 * PVR_PI_D * (double)i / (double)N)));
}

void pvr_fft_twiddles(int L, pvr_c32* tw) {
    for (int m = 0; m < L / 2; ++m) {
        double a = 2.0 * PVR_PI_D * (double)m / (double)L;
        tw[m].x = (float)cos(a);
        tw[m].y = (float)(-sin(a));
    }
}

void pvr_split_twiddles(int N, pvr_c32* tws) {
    for (int k = 0; k <= N / 2; ++k) {
        double a = 2.0 * PVR_PI_D * (double)k / (double)N;
        tws[k].x = (float)cos(a);
        tws[k].y = (float)(-sin(a));
    }
}

void pvr_expected_advance(int N, int hop, float* e, int* j) {
    /* omega_k * hop = 2 pi (k*hop)/N = 2 pi j_k + e_k,  e_k in (-pi, pi] */
    for (int k = 0; k <= N / 2; ++k) {
        long long kh = (long long)k * hop;
        long long r = kh % N;
        long long rr = (r > N / 2) ? r - N : r;
        if (e) e[k] = (float)(2.0 * PVR_PI_D * (double)rr / (double)N);
        if (j) j[k] = (int)((kh - rr) / N);
    }
}

/* ------------------------------------------------------------------ fp32 contract */

float pvr_atan2f(float y, float x) {
    float ax = fabsf(x), ay = fabsf(y);
    /* IEEE maxNum / minNum (a NaN operand yields the other), as the GPU's v_max3_f32 /
     * v_min_f32 in IEEE mode; mx floored at FLT_MIN: an all-zero bin gets a = 0 and the
     * phase +-0 (the sign of y), without a special case.  (Contract v4: a bin whose
     * components are both NaN — a frame with a non-finite sample — gets a = 0, phase +-0.) */
    float mx = fmaxf(fmaxf(ax, ay), 0x1p-126f);
    float mn = fminf(ax, ay);
    /* a = mn / mx without a division: reciprocal of mx from an integer seed (relative
     * error <= 5.1e-2), a cubic and a Newton step (below), then one product; <= 6e-8
     * relative for normal mx (audio spectra are far from the fp32 range ends).  The GPU
     * (pv_device.hpp atan2_pv / atan2_pv2) performs the same operations. */
    uint32_t mb;
    memcpy(&mb, &mx, sizeof mb);
    mb = 0x7EF311C3u - mb;
    float r0;
    memcpy(&r0, &mb, sizeof r0);
    /* contract v3: one cubic step r (1 + e + e^2) (|e| <= 5.1e-2 -> 1.3e-4) and one Newton
     * step (-> ~2e-8): five fmaf instead of the three Newton steps' six */
    float e = fmaf(-mx, r0, 1.0f);
    float e2 = fmaf(e, e, e);
    r0 = fmaf(r0, e2, r0);
    e = fmaf(-mx, r0, 1.0f);
    r0 = fmaf(r0, e, r0);
    /* contract v4: the ratio clamped to [0, 1], NaN -> 0 (the GPU's clamp modifier with
     * DX10 clamping): the phase of a non-finite bin is finite, so no decision explodes */
    float a = mn * r0;
    a = (a >= 0.0f) ? ((a <= 1.0f) ? a : 1.0f) : 0.0f;
    float s = a * a;
    float p = PVR_ATAN_C[9];
    for (int i = 8; i >= 0; --i) p = fmaf(p, s, PVR_ATAN_C[i]);
    float r = a * p;
    if (ay > ax) r = PVR_HALF_PI_F - r;
    if (x < 0.0f) r = PVR_PI_F - r;
    return copysignf(r, y); /* r >= 0: the sign of y (y = -0 gives -r, like C atan2) */
}

static inline pvr_c32 cmul_c(pvr_c32 b, pvr_c32 w) {
    pvr_c32 t;
    t.x = fmaf(b.x, w.x, -(b.y * w.y));
    t.y = fmaf(b.x, w.y, b.y * w.x);
    return t;
}

void pvr_fft_c32(pvr_c32* data, pvr_c32* tmp, int L, const pvr_c32* tw, int inverse) {
    /* Stockham autosort radix-2, the stage structure of hpfft.cu:145-167 (FftIteration:
     * v1 = in[j+L/2]*W(j%Ns), out[expand(j,Ns,2)+{0,Ns}] = v0 +- v1), with the twiddle
     * W(idx,Ns) = e^{-i pi idx/Ns} taken from the table tw[idx*L/(2Ns)] instead of being
     * recomputed with cos/sin per butterfly.  The top element is never multiplied; the
     * bottom one is, except in the first two stages where W is exactly 1 (Ns = 1, and
     * Ns = 2, idx = 0: t = b) or -i (Ns = 2, idx = 1: t = (b.y, -b.x); +i when inverse). */
    pvr_c32* in = data;
    pvr_c32* out = tmp;
    const int half = L / 2;
    for (int Ns = 1; Ns < L; Ns <<= 1) {
        const int tstride = L / (2 * Ns);
        for (int j = 0; j < half; ++j) {
            pvr_c32 a = in[j], b = in[j + half];
            int idx = j & (Ns - 1);
            pvr_c32 w = tw[idx * tstride];
            if (inverse) w.y = -w.y;
            pvr_c32 t;
            if (Ns == 1 || (Ns == 2 && idx == 0)) {
                t = b;
            } else if (Ns == 2) {
                t.x = inverse ? -b.y : b.y;
                t.y = inverse ? b.x : -b.x;
            } else {
                t = cmul_c(b, w);
            }
            int pos = (j / Ns) * 2 * Ns + idx;
            out[pos].x = a.x + t.x;
            out[pos].y = a.y + t.y;
            out[pos + Ns].x = a.x - t.x;
            out[pos + Ns].y = a.y - t.y;
        }
        pvr_c32* s = in; in = out; out = s;
    }
    if (in != data) memcpy(data, in, sizeof(pvr_c32) * (size_t)L);
}

/* ---- contract v3 FFT (L = N/2 in [128, 512], E = L/64 points per GPU lane) ----
 * A Stockham FFT of twiddle-first radix-R passes: pass P has span S = E^P and radix
 * R = min(E, L/S); for every j < L/R (m = j mod S) the R points a_q = in[j + q L/R] are
 * multiplied by the table twiddles T_P[m][q] = e^{-2 pi i m q/(R S)} (q >= 1; none in pass 0,
 * where m = 0), transformed by the R-point DIF below (compile-time internal twiddles: 1, -i,
 * W8 = e^{-i pi/4}, W8^3) and written to out[(j/S) R S + m + S k] (register f of the GPU
 * holds y_k for k = bitrev(f), DIF order).  Exactly the operations of pv_device.hpp
 * fft_pass_v3. */
#define PVR_W8C 0x1.6a09e6p-1f /* (float)(1/sqrt 2) */

static inline int ilog2i(int v) { int r = 0; while ((1 << r) < v) ++r; return r; }
static inline int bitrevi(int v, int bits) {
    int r = 0;
    for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
    return r;
}

int pvr_fft_v3_applies(int L) { return L >= 128 && L <= 512; }

int pvr_fft_v3_table_size(int L) {
    const int E = L / 64;
    int n = 0;
    for (int S = E; S < L; S *= (E < L / S ? E : L / S)) n += S * ((E < L / S ? E : L / S) - 1);
    return n;
}

void pvr_fft_v3_table(int L, pvr_c32* t) {
    const int E = L / 64;
    int off = 0;
    for (int S = E; S < L;) {
        const int R = E < L / S ? E : L / S;
        for (int m = 0; m < S; ++m)
            for (int q = 1; q < R; ++q) {
                /* e^{-2 pi i m q/(R S)} = the L-point master entry (m q L/(R S)) mod L */
                const long idx = ((long)m * q * (L / (R * S))) % L;
                const double a = 2.0 * PVR_PI_D * (double)idx / (double)L;
                t[off + m * (R - 1) + (q - 1)].x = (float)cos(a);
                t[off + m * (R - 1) + (q - 1)].y = (float)(-sin(a));
            }
        off += S * (R - 1);
        S *= R;
    }
}

/* the R-point DIF of contract v3 on t[0..R-1] (R in {2, 4, 8}) */
static void dif_v3(pvr_c32* t, int R, int inverse) {
    const float c = PVR_W8C;
    for (int h = R / 2; h >= 1; h /= 2)
        for (int b = 0; b < R; b += 2 * h)
            for (int i = 0; i < h; ++i) {
                const pvr_c32 u = t[b + i], v = t[b + i + h];
                pvr_c32 d;
                if (i > 0 && 2 * i == h) {        /* -i (forward) / +i (inverse) rotation */
                    if (!inverse) { d.x = u.y - v.y; d.y = v.x - u.x; }
                    else { d.x = v.y - u.y; d.y = u.x - v.x; }
                } else {
                    const pvr_c32 e = {u.x - v.x, u.y - v.y};
                    if (i == 0) {
                        d = e;
                    } else {
                        pvr_c32 s;
                        if (4 * i == h) {         /* W8^1 = (c, -c); inverse (c, c) */
                            if (!inverse) { s.x = e.x + e.y; s.y = e.y - e.x; }
                            else { s.x = e.x - e.y; s.y = e.x + e.y; }
                        } else {                  /* 4i == 3h: W8^3 = (-c, -c); inverse (-c, c) */
                            if (!inverse) { s.x = e.y - e.x; s.y = -e.x - e.y; }
                            else { s.x = -e.x - e.y; s.y = e.x - e.y; }
                        }
                        d.x = s.x * c;
                        d.y = s.y * c;
                    }
                }
                t[b + i].x = u.x + v.x;
                t[b + i].y = u.y + v.y;
                t[b + i + h] = d;
            }
}

void pvr_fft_c32_v3(pvr_c32* data, pvr_c32* tmp, int L, const pvr_c32* ptab, int inverse) {
    const int E = L / 64;
    pvr_c32* in = data;
    pvr_c32* out = tmp;
    int off = 0;
    for (int S = 1, P = 0; S < L; ++P) {
        const int R = E < L / S ? E : L / S;
        const int r = ilog2i(R);
        for (int j = 0; j < L / R; ++j) {
            const int m = j % S;
            pvr_c32 t[8];
            for (int q = 0; q < R; ++q) t[q] = in[j + q * (L / R)];
            if (P > 0)
                for (int q = 1; q < R; ++q) {
                    pvr_c32 tw = ptab[off + m * (R - 1) + (q - 1)];
                    if (inverse) tw.y = -tw.y;
                    t[q] = cmul_c(t[q], tw);
                }
            dif_v3(t, R, inverse);
            for (int f = 0; f < R; ++f) out[(j / S) * R * S + m + S * bitrevi(f, r)] = t[f];
        }
        if (P > 0) off += S * (R - 1);
        pvr_c32* sw = in; in = out; out = sw;
        S *= R;
    }
    if (in != data) memcpy(data, in, sizeof(pvr_c32) * (size_t)L);
}

/* the contract's real FFT of N raw samples x with the analysis window w: x * w rounded, then
 * pvr_rfft_c32 */
void pvr_rfft_win_c32(const float* x, const float* w, int N, const pvr_c32* tw, const pvr_c32* tws,
                      pvr_c32* X, pvr_c32* work) {
    float* xw = (float*)malloc(sizeof(float) * N);
    for (int i = 0; i < N; ++i) xw[i] = x[i] * w[i];
    pvr_rfft_c32(xw, N, tw, tws, X, work);
    free(xw);
}

void pvr_rfft_c32(const float* xw, int N, const pvr_c32* tw, const pvr_c32* tws,
                  pvr_c32* X, pvr_c32* work) {
    const int L = N / 2;
    pvr_c32* z = work;
    pvr_c32* tmp = work + L;
    for (int n = 0; n < L; ++n) { z[n].x = xw[2 * n]; z[n].y = xw[2 * n + 1]; }
    if (pvr_fft_v3_applies(L)) pvr_fft_c32_v3(z, tmp, L, tw, 0);
    else pvr_fft_c32(z, tmp, L, tw, 0);
    pvr_split_c32(z, L, tws, X);
}

void pvr_split_c32(const pvr_c32* z, int L, const pvr_c32* tws, pvr_c32* X) {
    for (int k = 0; k <= L; ++k) {
        pvr_c32 A = z[k % L], B = z[(L - k) % L];
        float er = 0.5f * (A.x + B.x);
        float ei = 0.5f * (A.y - B.y);
        float orr = 0.5f * (A.y + B.y);
        float oi = 0.5f * (B.x - A.x);
        pvr_c32 w = tws[k];
        /* contract v2: the odd part's twiddle product accumulated onto the even part with
         * two fused operations per component (one rounding each), as the GPU's
         * split_chunk / split_chunk_bp / real_split / bin_l_real */
        X[k].x = fmaf(orr, w.x, fmaf(-oi, w.y, er));
        X[k].y = fmaf(orr, w.y, fmaf(oi, w.x, ei));
    }
    X[0].y = 0.0f;
    X[L].y = 0.0f;
}

/* contract v2: m = -RN_int(d * (1/2pi)) with ONE rounding: fmaf(d, 1/2pi, 1.5 * 2^23) rounds
 * the exact product onto the integer grid of [2^23, 2^24) (ties to even, as rintf, since the
 * magic is even); subtracting the magic back is exact (|d| < 3 pi).  The GPU
 * (pv_device.hpp unwrap_round / unwrap_count) performs the same two operations. */
#define PVR_RINT_MAGIC 0x1.8p23f
int pvr_unwrap_count(float phi, float phi_prev, float e) {
    float d = (phi - phi_prev) - e;
    float t = fmaf(d, PVR_INV_2PI_F, PVR_RINT_MAGIC);
    return -(int)(t - PVR_RINT_MAGIC);
}

/* ------------------------------------------------------------------ geometry */

int pvr_num_frames(long n, int hop) {
    /* main.cpp:231: for (i = 0; i < numSamples - hopSize; i += hopSize) */
    long span = n - hop;
    if (span <= 0) return 0;
    return (int)((span + hop - 1) / hop);
}

int pvr_out_hop(int N, int hop_div, int effect, float scale) {
    int hop = N / hop_div; /* phaseVocoder.h:79 hopSize(samples/hop) */
    if (effect == PVR_TIME_SHIFT) {
        float f = scale * (float)hop; /* phaseVocoder.h:104 outHopSize = scaleFactor*hopSize */
        return (int)f;
    }
    return hop; /* PITCH_SHIFT: the build's definition (reference leaves it unset) */
}

/* ------------------------------------------------------------------ fp64 FFT */

static void fft_c64_tab(pvr_c64* a, int L, int inverse, const pvr_c64* tab) {
    /* iterative radix-2 DIT with bit reversal; tab[m] = e^{-2 pi i m/L}, m < L/2 */
    for (int i = 1, j = 0; i < L; ++i) {
        int bit = L >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { pvr_c64 t = a[i]; a[i] = a[j]; a[j] = t; }
    }
    for (int len = 2; len <= L; len <<= 1) {
        int h = len / 2, step = L / len;
        for (int k = 0; k < h; ++k) {
            double wr = tab[k * step].x, wi = inverse ? -tab[k * step].y : tab[k * step].y;
            for (int i = 0; i < L; i += len) {
                pvr_c64 u = a[i + k], v = a[i + k + h];
                double tr = v.x * wr - v.y * wi, ti = v.x * wi + v.y * wr;
                a[i + k].x = u.x + tr; a[i + k].y = u.y + ti;
                a[i + k + h].x = u.x - tr; a[i + k + h].y = u.y - ti;
            }
        }
    }
}

static pvr_c64* c64_table(int L) {
    pvr_c64* t = (pvr_c64*)malloc(sizeof(pvr_c64) * (L / 2 + 1));
    for (int m = 0; m < L / 2; ++m) {
        double a = -2.0 * PVR_PI_D * (double)m / (double)L;
        t[m].x = cos(a);
        t[m].y = sin(a);
    }
    return t;
}

void pvr_fft_c64(pvr_c64* a, int L, int inverse) {
    pvr_c64* t = c64_table(L);
    fft_c64_tab(a, L, inverse, t);
    free(t);
}

/* C2R of size N from N/2+1 bins (Im of DC and Nyquist ignored), unnormalised */
static void irfft_c64(const pvr_c64* Y, int N, pvr_c64* work, double* y, const pvr_c64* tab) {
    const int L = N / 2;
    for (int k = 0; k <= L; ++k) work[k] = Y[k];
    work[0].y = 0.0;
    work[L].y = 0.0;
    for (int k = 1; k < L; ++k) { work[N - k].x = Y[k].x; work[N - k].y = -Y[k].y; }
    fft_c64_tab(work, N, 1, tab);
    for (int n = 0; n < N; ++n) y[n] = work[n].x;
}

/* ------------------------------------------------------------------ PV_STANDARD */

typedef struct {
    int N, L, B, hop;
    float* w;
    pvr_c32 *tw, *tws, *work, *X;
    float* xw;
} std_ana_ctx;

static void std_ana_init(std_ana_ctx* c, int N, int hop) {
    c->N = N; c->L = N / 2; c->B = N / 2 + 1; c->hop = hop;
    c->w = (float*)malloc(sizeof(float) * N);
    c->xw = (float*)malloc(sizeof(float) * N);
    c->tw = (pvr_c32*)malloc(sizeof(pvr_c32) * (N / 2 + 1));
    c->tws = (pvr_c32*)malloc(sizeof(pvr_c32) * c->B);
    c->work = (pvr_c32*)malloc(sizeof(pvr_c32) * N);
    c->X = (pvr_c32*)malloc(sizeof(pvr_c32) * c->B);
    pvr_hann_periodic(N, c->w);
    /* the FFT's table: contract v3 pass table (L <= 512) or the radix-2 master table */
    if (pvr_fft_v3_applies(c->L)) pvr_fft_v3_table(c->L, c->tw);
    else pvr_fft_twiddles(c->L, c->tw);
    pvr_split_twiddles(N, c->tws);
}

static void std_ana_free(std_ana_ctx* c) {
    free(c->w); free(c->xw); free(c->tw); free(c->tws); free(c->work); free(c->X);
}

/* one frame of the fp32 contract: mag/phase of frame starting at x[start] */
static void std_ana_frame(std_ana_ctx* c, const float* x, long n, long start, float* mag,
                          float* phase) {
    for (int i = 0; i < c->N; ++i) {
        long idx = start + i;
        c->xw[i] = (idx < n) ? x[idx] : 0.0f; /* defined deviation: OOB samples read as 0 */
    }
    /* the raw frame: the window is applied inside (contract v3: folded into the FFT) */
    pvr_rfft_win_c32(c->xw, c->w, c->N, c->tw, c->tws, c->X, c->work);
    for (int k = 0; k < c->B; ++k) {
        float re = c->X[k].x, im = c->X[k].y;
        mag[k] = sqrtf(fmaf(re, re, im * im));
        phase[k] = pvr_atan2f(im, re);
    }
}

void pvr_std_analysis(const float* x, long n, int N, int hop, int frames, pvr_c32* spec) {
    std_ana_ctx c;
    std_ana_init(&c, N, hop);
    float* mag = (float*)malloc(sizeof(float) * c.B);
    float* ph = (float*)malloc(sizeof(float) * c.B);
    for (int t = 0; t < frames; ++t) {
        std_ana_frame(&c, x, n, (long)t * hop, mag, ph);
        for (int k = 0; k < c.B; ++k) {
            spec[(size_t)t * c.B + k].x = mag[k];
            spec[(size_t)t * c.B + k].y = ph[k];
        }
    }
    free(mag); free(ph);
    std_ana_free(&c);
}

int pvr_std_process(const float* x, long n, int N, int hop_div, int effect, float scale,
                    int frames, double* out) {
    const int hop_a = N / hop_div;
    const int hop_s = pvr_out_hop(N, hop_div, effect, scale);
    const int L = N / 2, B = L + 1;
    const double TWO_PI = 2.0 * PVR_PI_D;
    std_ana_ctx c;
    std_ana_init(&c, N, hop_a);

    float* mag = (float*)malloc(sizeof(float) * B);
    float* ph = (float*)malloc(sizeof(float) * B);
    float* ph_prev = (float*)calloc(B, sizeof(float));
    float* ek = (float*)malloc(sizeof(float) * B);
    int* jk = (int*)malloc(sizeof(int) * B);
    double* omega_true = (double*)malloc(sizeof(double) * B);
    double* acc = (double*)calloc(B, sizeof(double));
    int* first = (int*)malloc(sizeof(int) * B);
    int* cnt = (int*)calloc(B, sizeof(int));
    pvr_c64* Y = (pvr_c64*)malloc(sizeof(pvr_c64) * B);
    pvr_c64* cw = (pvr_c64*)malloc(sizeof(pvr_c64) * N);
    double* y = (double*)malloc(sizeof(double) * N);
    double* g = (double*)malloc(sizeof(double) * N);
    pvr_expected_advance(N, hop_a, ek, jk);
    pvr_c64* ctab = c64_table(N);

    /* synthesis gain: periodic Hann (double) * hop_s / sum(w^2) / N   */
    double sw2 = 0.0;
    for (int i = 0; i < N; ++i) {
        double wd = 0.5 - 0.5 * cos(TWO_PI * (double)i / (double)N);
        g[i] = wd;
        sw2 += wd * wd;
    }
    for (int i = 0; i < N; ++i) g[i] = g[i] * ((double)hop_s / sw2) / (double)N;

    /* pitch bin map: k' = floor(beta*k + 0.5); magnitude summed, phase from smallest k */
    const double beta = (double)scale;
    for (int k = 0; k < B; ++k) first[k] = -1;
    if (effect == PVR_PITCH_SHIFT) {
        for (int k = 0; k < B; ++k) {
            long kp = (long)floor(beta * (double)k + 0.5);
            if (kp < 0 || kp >= B) continue;
            if (first[kp] < 0) first[kp] = k;
            cnt[kp]++;
        }
    }

    const long out_len = (long)frames * hop_s + (N - hop_s);
    for (long i = 0; i < out_len; ++i) out[i] = 0.0;

    for (int t = 0; t < frames; ++t) {
        std_ana_frame(&c, x, n, (long)t * hop_a, mag, ph);
        for (int k = 0; k < B; ++k) {
            /* textbook (milestone1_565.pdf p.2): delta = princarg(phi - phi_prev - w_k*hop);
             * the princarg branch is the fp32 integer decision m (+ j_k, which turns the
             * decision relative to the wrapped advance e_k into one relative to w_k*hop). */
            int m = pvr_unwrap_count(ph[k], ph_prev[k], ek[k]);
            double wk = TWO_PI * (double)k / (double)N;
            double delta = ((double)ph[k] - (double)ph_prev[k] - wk * (double)hop_a) +
                           TWO_PI * (double)(m + jk[k]);
            omega_true[k] = wk + delta / (double)hop_a;
            ph_prev[k] = ph[k];
        }
        if (effect == PVR_PITCH_SHIFT) {
            for (int kp = 0; kp < B; ++kp) {
                if (cnt[kp] == 0) { Y[kp].x = 0.0; Y[kp].y = 0.0; continue; }
                int s = first[kp];
                acc[kp] = fmod(acc[kp] + (double)hop_a * beta * omega_true[s], TWO_PI);
                double msum = 0.0;
                for (int q = 0; q < cnt[kp]; ++q) msum += (double)mag[s + q];
                Y[kp].x = msum * cos(acc[kp]);
                Y[kp].y = msum * sin(acc[kp]);
            }
        } else {
            for (int k = 0; k < B; ++k) {
                acc[k] = fmod(acc[k] + (double)hop_s * omega_true[k], TWO_PI);
                Y[k].x = (double)mag[k] * cos(acc[k]);
                Y[k].y = (double)mag[k] * sin(acc[k]);
            }
        }
        irfft_c64(Y, N, cw, y, ctab);
        double* o = out + (long)t * hop_s;
        for (int i = 0; i < N; ++i) o[i] += y[i] * g[i];
    }

    free(mag); free(ph); free(ph_prev); free(ek); free(jk); free(omega_true); free(acc);
    free(first); free(cnt); free(Y); free(cw); free(y); free(g); free(ctab);
    std_ana_free(&c);
    return hop_s;
}

int pvr_std_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                          int effect, float scale, int frames, float* out, long ldo,
                          int threads) {
    const int hop_s = pvr_out_hop(N, hop_div, effect, scale);
    const long out_len = (long)frames * hop_s + (N - hop_s);
    int used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
        double* buf = (double*)malloc(sizeof(double) * (size_t)out_len);
#pragma omp for schedule(dynamic, 1)
        for (int ch = 0; ch < C; ++ch) {
            pvr_std_process(x + (size_t)ch * ldx, n, N, hop_div, effect, scale, frames, buf);
            for (long i = 0; i < out_len; ++i) out[(size_t)ch * ldo + i] = (float)buf[i];
        }
        free(buf);
    }
#else
    (void)threads;
    double* buf = (double*)malloc(sizeof(double) * (size_t)out_len);
    for (int ch = 0; ch < C; ++ch) {
        pvr_std_process(x + (size_t)ch * ldx, n, N, hop_div, effect, scale, frames, buf);
        for (long i = 0; i < out_len; ++i) out[(size_t)ch * ldo + i] = (float)buf[i];
    }
    free(buf);
#endif
    return used;
}

int pvr_compat_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                             int frames, float* out, long ldo, int threads) {
    const int hop = N / hop_div;
    const long out_len = (long)frames * hop + (N - hop);
    int used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
        double* buf = (double*)malloc(sizeof(double) * (size_t)out_len);
#pragma omp for schedule(dynamic, 1)
        for (int ch = 0; ch < C; ++ch) {
            pvr_compat_process(x + (size_t)ch * ldx, n, N, hop_div, frames, buf);
            for (long i = 0; i < out_len; ++i) out[(size_t)ch * ldo + i] = (float)buf[i];
        }
        free(buf);
    }
#else
    (void)threads;
    double* buf = (double*)malloc(sizeof(double) * (size_t)out_len);
    for (int ch = 0; ch < C; ++ch) {
        pvr_compat_process(x + (size_t)ch * ldx, n, N, hop_div, frames, buf);
        for (long i = 0; i < out_len; ++i) out[(size_t)ch * ldo + i] = (float)buf[i];
    }
    free(buf);
#endif
    return used;
}

/* ------------------------------------------------------------------ REF_COMPAT */

void pvr_compat_analysis_frame(const float* frame, int N, const float* win, pvr_c64* b,
                               int nan_faithful) {
    const int N2 = 2 * N;
    /* cudaWindow (kernel.cu:68-74): interm[k] = in[k]*win[k] (exact in double) */
    /* cufftShiftPadZeros (kernel.cu:25-32) into a pre-zeroed 2N buffer (main.cpp:216) */
    for (int k = 0; k < N2; ++k) { b[k].x = 0.0; b[k].y = 0.0; }
    for (int k = 0; k < N / 2; ++k) {
        b[k].x = (double)frame[k + N / 2] * (double)win[k + N / 2];
        b[k + N / 2 + N].x = (double)frame[k] * (double)win[k];
    }
    /* cufftExecC2C FORWARD, size 2N, unnormalised (kernel.cu:324-336) */
    pvr_fft_c64(b, N2, 0);
    /* cudaMagFreq (kernel.cu:101-109): (sqrt(x^2+y^2), atanf(y/x)) */
    for (int k = 0; k < N2; ++k) {
        double re = b[k].x, im = b[k].y;
        double mag = sqrt(re * re + im * im);
        double ph;
        if (re == 0.0 && im == 0.0)
            ph = nan_faithful ? NAN : 0.0; /* defined deviation (4), SURVEY.md §8c */
        else
            ph = atan(im / re);
        b[k].x = mag;
        b[k].y = ph;
    }
}

void pvr_compat_resynth_frame(const pvr_c64* spec, int N, const float* win, double* y) {
    const int L = N / 2;
    pvr_c64* Z = (pvr_c64*)malloc(sizeof(pvr_c64) * (L + 1));
    pvr_c64* work = (pvr_c64*)malloc(sizeof(pvr_c64) * N);
    double* r = (double*)malloc(sizeof(double) * N);
    /* cudaTimeScale (kernel.cu:121-129), timeScale = 1: x' = m cos(phi); y' = x' sin(phi)
     * (the y-bug: uses the updated x).  Only bins 0..N/2 are read by the C2R below. */
    for (int k = 0; k <= L; ++k) {
        double m = spec[k].x, ph = spec[k].y;
        double xr = m * cos(ph);
        double yi = xr * sin(ph);
        Z[k].x = xr;
        Z[k].y = yi;
    }
    /* cufftExecC2R size N on the first N/2+1 bins (kernel.cu:363-368) */
    pvr_c64* tab = c64_table(N);
    irfft_c64(Z, N, work, r, tab);
    free(tab);
    /* cudaDivVec /N (kernel.cu:380), cufftShift swap halves (kernel.cu:393),
     * cudaWindow (kernel.cu:406) */
    for (int k = 0; k < N; ++k) {
        double v = r[(k + L) % N] / (double)N;
        y[k] = v * (double)win[k];
    }
    free(Z); free(work); free(r);
}

int pvr_compat_process(const float* x, long n, int N, int hop_div, int frames, double* out) {
    return pvr_compat_process_ex(x, n, N, hop_div, frames, NULL, 0, out);
}

int pvr_compat_process_ex(const float* x, long n, int N, int hop_div, int frames,
                          const float* window, int nan_faithful, double* out) {
    return pvr_compat_process_hs(x, n, N, hop_div, N / hop_div, frames, window, nan_faithful, out);
}

/* out hop hs = (int)(timeScale * hop) (phaseVocoder.h:74): the reference passes outHopSize to
 * resynthesis_CUFFT (phaseVocoder.cpp:68) while cudaTimeScale's factor is hard-coded 1
 * (kernel.cu:354), so a time scale only moves the overlap-add hop and the emitted block
 * (main.cpp:266-287: frame i lands at i * outHopSize).  out: frames * hs + (N - hs). */
int pvr_compat_process_hs(const float* x, long n, int N, int hop_div, int hs, int frames,
                          const float* window, int nan_faithful, double* out) {
    const int hop = N / hop_div;
    float* win = (float*)malloc(sizeof(float) * N);
    float* frame = (float*)malloc(sizeof(float) * N);
    pvr_c64* spec = (pvr_c64*)malloc(sizeof(pvr_c64) * 2 * N);
    double* front = (double*)malloc(sizeof(double) * N);
    double* back = (double*)calloc(N, sizeof(double));
    if (window) memcpy(win, window, sizeof(float) * N);  /* the caller's imp (kernel.cu:301, :406) */
    else pvr_hamming_ref(N, win);
    for (int i = 0; i < frames; ++i) {
        long start = (long)i * hop;
        for (int k = 0; k < N; ++k) frame[k] = (start + k < n) ? x[start + k] : 0.0f;
        pvr_compat_analysis_frame(frame, N, win, spec, nan_faithful);
        pvr_compat_resynth_frame(spec, N, win, front);
        /* cudaOverlapAdd (kernel.cu:111-119): front[k-hop] += back[k], k in [hop, N);
         * then main.cpp:279 backFrame <- final_output; emit backFrame[0..hop) */
        for (int k = hs; k < N; ++k) front[k - hs] += back[k];
        for (int j = 0; j < hs; ++j) out[(long)i * hs + j] = front[j];
        memcpy(back, front, sizeof(double) * N);
    }
    /* remaining tail of the running accumulator (frames >= A carry zero spectra) */
    for (int k = hs; k < N; ++k) out[(long)frames * hs + (k - hs)] = back[k];
    free(win); free(frame); free(spec); free(front); free(back);
    return hs;
}
