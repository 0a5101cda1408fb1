/*
 * pvport.c — fp32 CPU PORT of the PV_STANDARD path (test infrastructure: bench.py's
 * cpu_baseline leg only; never linked into or called by the product).
 *
 * What bench.py times as the CPU baseline: the same algorithm the GPU runs, in fp32 end to
 * end, the way a CPU port of the reference path (kernel.cu:299-348 analysis, kernel.cu:352-432
 * resynthesis — fp32 throughout) would be written:
 *   analysis   the fp32 contract of pvref.c (window, contract-v3 FFT, split, sqrtf, atan2,
 *              unwrap decision) — the phases and decisions are the oracle's bit for bit;
 *   synthesis  the exact integer phase scan of DESIGN.md §3.3 (phi_s = rho (phi + 2 pi
 *              (M + (t+1) j_k)), the 2 pi multiple reduced mod q in integers), fp32 sin/cos,
 *              an fp32 inverse real FFT (an L-point complex FFT + the real split), fp32 gain
 *              and overlap-add — no fp64 anywhere in the frame loop;
 *   OpenMP over channels.
 * pvref.c's pvr_std_process stays the checker (fp64 textbook recurrence and fp64 FFT);
 * tests/test_oracle.py pins this port to it (<= 1e-6 RMS per sample).
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "pvref.h"

#define PORT_PI_D 3.14159265358979323846

static long gcd_l(long a, long b) {
    while (b) { long t = a % b; a = b; b = t; }
    return a < 0 ? -a : a;
}

/* rho = p / q exactly: stretch hop_s / hop_a; pitch the float scale (a dyadic rational) */
static void port_ratio(int effect, float scale, int hop_a, int hop_s, long* p, long* q) {
    if (effect == PVR_PITCH_SHIFT) {
        int e = 0;
        double m = frexp((double)scale, &e); /* scale = m 2^e, m in [0.5, 1): 24 bits */
        long num = (long)ldexp(m, 24);
        long den = 1L << 24;
        if (e >= 0) num <<= e; else den <<= -e;
        long g = gcd_l(num, den);
        *p = num / g; *q = den / g;
    } else {
        long g = gcd_l(hop_s, hop_a);
        *p = hop_s / g; *q = hop_a / g;
    }
}

typedef struct {
    int N, L, B, hop_a, hop_s, effect;
    long p, q;
    float rho_rev; /* rho / 2pi */
    float *w, *g, *xw, *mag, *ph, *php, *y;
    int *jk, *first, *cnt;
    long long* M; /* running unwrap count per bin */
    float* ek;
    pvr_c32 *tw, *tws, *work, *X, *Z, *twi, *tws_s;
} port_ctx;

static void port_init(port_ctx* c, int N, int hop_div, int effect, float scale) {
    const double TWO_PI = 2.0 * PORT_PI_D;
    c->N = N; c->L = N / 2; c->B = N / 2 + 1; c->hop_a = N / hop_div;
    c->hop_s = pvr_out_hop(N, hop_div, effect, scale);
    c->effect = effect;
    port_ratio(effect, scale, c->hop_a, c->hop_s, &c->p, &c->q);
    c->rho_rev = (float)((double)c->p / (double)c->q / TWO_PI);
    const int L = c->L, B = c->B;
    c->w = malloc(sizeof(float) * N); c->g = malloc(sizeof(float) * N);
    c->xw = malloc(sizeof(float) * N); c->y = malloc(sizeof(float) * N);
    c->mag = malloc(sizeof(float) * B); c->ph = malloc(sizeof(float) * B);
    c->php = calloc(B, sizeof(float)); c->ek = malloc(sizeof(float) * B);
    c->jk = malloc(sizeof(int) * B); c->first = malloc(sizeof(int) * B); c->cnt = calloc(B, sizeof(int));
    c->M = calloc(B, sizeof(long long));
    c->tw = malloc(sizeof(pvr_c32) * (L + 1)); c->tws = malloc(sizeof(pvr_c32) * B);
    c->twi = malloc(sizeof(pvr_c32) * (L + 1)); c->tws_s = malloc(sizeof(pvr_c32) * B);
    c->work = malloc(sizeof(pvr_c32) * N); c->X = malloc(sizeof(pvr_c32) * B);
    c->Z = malloc(sizeof(pvr_c32) * L);
    pvr_hann_periodic(N, c->w);
    if (pvr_fft_v3_applies(L)) pvr_fft_v3_table(L, c->tw); else pvr_fft_twiddles(L, c->tw);
    pvr_fft_twiddles(L, c->twi); /* radix-2 table for the inverse transform */
    pvr_split_twiddles(N, c->tws);
    memcpy(c->tws_s, c->tws, sizeof(pvr_c32) * B);
    pvr_expected_advance(N, c->hop_a, c->ek, c->jk);
    double sw2 = 0.0;
    for (int i = 0; i < N; ++i) {
        double wd = 0.5 - 0.5 * cos(TWO_PI * (double)i / (double)N);
        sw2 += wd * wd;
    }
    for (int i = 0; i < N; ++i) {
        double wd = 0.5 - 0.5 * cos(TWO_PI * (double)i / (double)N);
        c->g[i] = (float)(wd * ((double)c->hop_s / sw2) / (double)N);
    }
    for (int k = 0; k < B; ++k) c->first[k] = -1;
    if (effect == PVR_PITCH_SHIFT) {
        for (int k = 0; k < B; ++k) {
            long kp = (long)floor((double)scale * (double)k + 0.5);
            if (kp < 0 || kp >= B) continue;
            if (c->first[kp] < 0) c->first[kp] = k;
            c->cnt[kp]++;
        }
    }
}

static void port_free(port_ctx* c) {
    free(c->w); free(c->g); free(c->xw); free(c->y); free(c->mag); free(c->ph); free(c->php);
    free(c->ek); free(c->jk); free(c->first); free(c->cnt); free(c->M); free(c->tw); free(c->tws);
    free(c->twi); free(c->tws_s); free(c->work); free(c->X); free(c->Z);
}

/* fp32 sin/cos of 2 pi rev, rev reduced to [-1/2, 1/2] first */
static inline void sincos_rev(float rev, float* s, float* co) {
    const float r = rev - rintf(rev);
    const float a = r * 6.28318530717958647692f;
    *s = sinf(a);
    *co = cosf(a);
}

/* y[0..N) = unnormalised C2R of the N/2+1 bins Y (Im of DC / Nyquist ignored): an L-point
 * complex inverse FFT of Z[k] = Fe + i Fo, Fe = Y[k] + conj Y[L-k], Fo = (Y[k] - conj Y[L-k])
 * e^{+2 pi i k / N}; y[2n] + i y[2n+1] = z[n] */
static void port_irfft(port_ctx* c, const pvr_c32* Y, float* y) {
    const int L = c->L;
    for (int k = 0; k < L; ++k) {
        pvr_c32 A = Y[k], Bc = Y[L - k];
        if (k == 0) { A.y = 0.0f; Bc.y = 0.0f; }
        Bc.y = -Bc.y;
        const float fer = A.x + Bc.x, fei = A.y + Bc.y;
        const float dr = A.x - Bc.x, di = A.y - Bc.y;
        const pvr_c32 w = c->tws_s[k]; /* e^{-2 pi i k/N}: conj for the inverse */
        const float for_ = dr * w.x + di * w.y, foi = di * w.x - dr * w.y;
        c->Z[k].x = fer - foi;
        c->Z[k].y = fei + for_;
    }
    pvr_fft_c32(c->Z, c->work, L, c->twi, 1);
    for (int n = 0; n < L; ++n) { y[2 * n] = c->Z[n].x; y[2 * n + 1] = c->Z[n].y; }
}

static void port_channel(port_ctx* c, const float* x, long n, int frames, float* out) {
    const int N = c->N, B = c->B, hop_a = c->hop_a, hop_s = c->hop_s;
    const long q = c->q, p = c->p;
    const float inv_q = 1.0f / (float)q;
    pvr_c32* Y = c->X; /* reused after the analysis of the frame */
    memset(c->php, 0, sizeof(float) * B);
    memset(c->M, 0, sizeof(long long) * B);
    const long out_len = (long)frames * hop_s + (N - hop_s);
    memset(out, 0, sizeof(float) * (size_t)out_len);
    for (int t = 0; t < frames; ++t) {
        const long start = (long)t * hop_a;
        for (int i = 0; i < N; ++i) {
            const long idx = start + i;
            c->xw[i] = ((idx < n) ? x[idx] : 0.0f) * c->w[i];
        }
        pvr_rfft_c32(c->xw, N, c->tw, c->tws, c->X, c->work);
        for (int k = 0; k < B; ++k) {
            const float re = c->X[k].x, im = c->X[k].y;
            c->mag[k] = sqrtf(fmaf(re, re, im * im));
            c->ph[k] = pvr_atan2f(im, re);
            c->M[k] += pvr_unwrap_count(c->ph[k], c->php[k], c->ek[k]);
            c->php[k] = c->ph[k];
        }
        /* output phase in revolutions: rho phi / 2pi + ((p (M + (t+1) j_k)) mod q) / q */
        for (int kp = 0; kp < B; ++kp) {
            int s = kp;
            float m = c->mag[kp];
            if (c->effect == PVR_PITCH_SHIFT) {
                if (c->cnt[kp] == 0) { Y[kp].x = 0.0f; Y[kp].y = 0.0f; continue; }
                s = c->first[kp];
                m = 0.0f;
                for (int j = 0; j < c->cnt[kp]; ++j) m += c->mag[s + j];
            }
            long long r = (c->M[s] + (long long)(t + 1) * c->jk[s]) % q;
            if (r < 0) r += q;
            const float frac = (float)((p % q) * r % q) * inv_q;
            float sn, cs;
            sincos_rev(c->rho_rev * c->ph[s] + frac, &sn, &cs);
            Y[kp].x = m * cs;
            Y[kp].y = m * sn;
        }
        port_irfft(c, Y, c->y);
        float* o = out + (long)t * hop_s;
        for (int i = 0; i < N; ++i) o[i] += c->y[i] * c->g[i];
    }
}

int pvr_port_std_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                               int effect, float scale, int frames, float* out, long ldo,
                               int threads) {
    int used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
        port_ctx c;
        port_init(&c, N, hop_div, effect, scale);
#pragma omp for schedule(dynamic, 1)
        for (int ch = 0; ch < C; ++ch) port_channel(&c, x + (size_t)ch * ldx, n, frames, out + (size_t)ch * ldo);
        port_free(&c);
    }
#else
    (void)threads;
    port_ctx c;
    port_init(&c, N, hop_div, effect, scale);
    for (int ch = 0; ch < C; ++ch) port_channel(&c, x + (size_t)ch * ldx, n, frames, out + (size_t)ch * ldo);
    port_free(&c);
#endif
    return used;
}

/* ------------------------------------------------------------------ REF_COMPAT, fp32
 * The reference's own path (kernel.cu:299-348 analysis, kernel.cu:352-432 resynthesis, the
 * main.cpp:228-297 offline loop) as an fp32 CPU port — kernel.cu is fp32 throughout — timed
 * as the REF_COMPAT line's cpu_baseline; pvref.c's pvr_compat_process (fp64) stays the
 * checker and tests/test_oracle.py pins this port to it (<= 1e-6 RMS per sample):
 *   cudaWindow (Hamming, phaseVocoder.h:85-89) + cufftShiftPadZeros (kernel.cu:25-32) into a
 *   2N real frame; C2C 2N (kernel.cu:324-336) as the 2N-point real FFT (an N-point complex
 *   FFT + split: the input is real) with bins N+1 .. 2N-1 the conjugate mirror; cudaMagFreq
 *   (kernel.cu:101-109) sqrtf and atanf(y / x) over all 2N bins (the GPU computes and stores
 *   them all too); cudaTimeScale's y-bug (kernel.cu:121-129); C2R N on bins 0 .. N/2
 *   (kernel.cu:363-368) as an N/2-point complex inverse FFT; /N, swap halves, window
 *   (kernel.cu:380, 393, 406); the running overlap-add (kernel.cu:111-119, main.cpp:279). */
typedef struct {
    int N, hop;
    float *w, *fr, *xw, *y, *front, *back;
    pvr_c32 *tw2, *tws2, *twi, *tws_s, *work, *X, *S, *Z;
} cport_ctx;

static void cport_init(cport_ctx* c, int N, int hop_div) {
    const int L2 = N;       /* complex points of the 2N-point real FFT */
    const int L = N / 2;    /* complex points of the N-point C2R */
    c->N = N;
    c->hop = N / hop_div;
    c->w = (float*)malloc(sizeof(float) * N);
    pvr_hamming_ref(N, c->w);
    c->fr = (float*)malloc(sizeof(float) * N);
    c->xw = (float*)calloc(2 * (size_t)N, sizeof(float));
    c->y = (float*)malloc(sizeof(float) * N);
    c->front = (float*)malloc(sizeof(float) * N);
    c->back = (float*)calloc(N, sizeof(float));
    const int t2 = pvr_fft_v3_applies(L2) ? pvr_fft_v3_table_size(L2) : L2 / 2;
    c->tw2 = (pvr_c32*)malloc(sizeof(pvr_c32) * (size_t)(t2 > 1 ? t2 : 1));
    if (pvr_fft_v3_applies(L2)) pvr_fft_v3_table(L2, c->tw2);
    else pvr_fft_twiddles(L2, c->tw2);
    c->tws2 = (pvr_c32*)malloc(sizeof(pvr_c32) * (L2 + 1));
    pvr_split_twiddles(2 * N, c->tws2);
    c->twi = (pvr_c32*)malloc(sizeof(pvr_c32) * (L / 2 > 1 ? L / 2 : 1));
    pvr_fft_twiddles(L, c->twi);
    c->tws_s = (pvr_c32*)malloc(sizeof(pvr_c32) * (L + 1));
    pvr_split_twiddles(N, c->tws_s);
    c->work = (pvr_c32*)malloc(sizeof(pvr_c32) * 2 * (size_t)L2);
    c->X = (pvr_c32*)malloc(sizeof(pvr_c32) * (L2 + 1));
    c->S = (pvr_c32*)malloc(sizeof(pvr_c32) * 2 * (size_t)N);  /* the 2N-bin {mag, phase} row */
    c->Z = (pvr_c32*)malloc(sizeof(pvr_c32) * (L + 1));
}

static void cport_free(cport_ctx* c) {
    free(c->w); free(c->fr); free(c->xw); free(c->y); free(c->front); free(c->back);
    free(c->tw2); free(c->tws2); free(c->twi); free(c->tws_s); free(c->work); free(c->X);
    free(c->S); free(c->Z);
}

static void cport_channel(cport_ctx* c, const float* x, long n, int frames, float* out) {
    const int N = c->N, L = N / 2, hop = c->hop;
    memset(c->back, 0, sizeof(float) * N);
    for (int t = 0; t < frames; ++t) {
        const long start = (long)t * hop;
        for (int k = 0; k < N; ++k) c->fr[k] = (start + k < n) ? x[start + k] : 0.0f;
        /* window + shift + zero pad (2N real samples, the middle N zeros stay zero) */
        for (int k = 0; k < N / 2; ++k) {
            c->xw[k] = c->fr[k + N / 2] * c->w[k + N / 2];
            c->xw[k + N / 2 + N] = c->fr[k] * c->w[k];
        }
        pvr_rfft_c32(c->xw, 2 * N, c->tw2, c->tws2, c->X, c->work);
        /* magnitude and atanf(y / x) of bins 0 .. N; bins N+1 .. 2N-1 mirror them */
        for (int k = 0; k <= N; ++k) {
            const float re = c->X[k].x, im = c->X[k].y;
            c->S[k].x = sqrtf(re * re + im * im);
            c->S[k].y = atanf(im / re);
        }
        for (int k = N + 1; k < 2 * N; ++k) { c->S[k].x = c->S[2 * N - k].x; c->S[k].y = -c->S[2 * N - k].y; }
        /* cudaTimeScale (timeScale 1): x' = m cos(phi), y' = x' sin(phi); bins 0 .. N/2 */
        for (int k = 0; k <= L; ++k) {
            const float xr = c->S[k].x * cosf(c->S[k].y);
            c->X[k].x = xr;
            c->X[k].y = xr * sinf(c->S[k].y);
        }
        /* C2R N (Im of DC and Nyquist ignored): Z[k] = Fe + i Fo, L-point inverse FFT */
        for (int k = 0; k < L; ++k) {
            pvr_c32 A = c->X[k], Bc = c->X[L - k];
            if (k == 0) { A.y = 0.0f; Bc.y = 0.0f; }
            Bc.y = -Bc.y;
            const float fer = A.x + Bc.x, fei = A.y + Bc.y;
            const float dr = A.x - Bc.x, di = A.y - Bc.y;
            const pvr_c32 tw = c->tws_s[k];
            const float for_ = dr * tw.x + di * tw.y, foi = di * tw.x - dr * tw.y;
            c->Z[k].x = fer - foi;
            c->Z[k].y = fei + for_;
        }
        pvr_fft_c32(c->Z, c->work, L, c->twi, 1);
        for (int m = 0; m < L; ++m) { c->y[2 * m] = c->Z[m].x; c->y[2 * m + 1] = c->Z[m].y; }
        /* /N, swap halves, window; overlap-add with the running back frame, emit hop */
        const float invN = 1.0f / (float)N;
        for (int k = 0; k < N; ++k) c->front[k] = c->y[(k + L) % N] * invN * c->w[k];
        for (int k = hop; k < N; ++k) c->front[k - hop] += c->back[k];
        for (int j = 0; j < hop; ++j) out[start + j] = c->front[j];
        memcpy(c->back, c->front, sizeof(float) * N);
    }
    for (int k = hop; k < N; ++k) out[(long)frames * hop + (k - hop)] = c->back[k];
}

int pvr_port_compat_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                                  int frames, float* out, long ldo, int threads) {
    int used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
        cport_ctx c;
        cport_init(&c, N, hop_div);
#pragma omp for schedule(dynamic, 1)
        for (int ch = 0; ch < C; ++ch) cport_channel(&c, x + (size_t)ch * ldx, n, frames, out + (size_t)ch * ldo);
        cport_free(&c);
    }
#else
    (void)threads;
    cport_ctx c;
    cport_init(&c, N, hop_div);
    for (int ch = 0; ch < C; ++ch) cport_channel(&c, x + (size_t)ch * ldx, n, frames, out + (size_t)ch * ldo);
    cport_free(&c);
#endif
    return used;
}
