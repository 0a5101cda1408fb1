/*
 * pvref.h — CPU ORACLE for the phase-vocoder hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (phase-vocoder_amd/, include/)
 * may include, link or call this code.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker / CPU baseline.
 *
 * Parity status:
 *   - REF_COMPAT: a literal fp64 restatement of the reference's active path
 *     (karnel/kernel.cu:299-348 analysis, kernel.cu:352-432 resynthesis, main.cpp:228-297
 *     framing/running OLA).  The reference itself cannot be built here (needs nvcc +
 *     cuFFT), so the oracle is pinned to the DFT contract cuFFT implements
 *     through numpy/pocketfft golden vectors generated from the reference's own input
 *     fixtures (tests/golden/make_golden.py) and to the spectral signature of the
 *     reference's own output artifact output/1000hzout.wav.  => "pinned (DFT contract +
 *     spectral signature)", not bit-pinned to a reference binary.
 *   - PV_STANDARD: the reference never implemented it (phaseVocoder.h:107-110,
 *     main.cpp:301-303 are empty).  The algorithm is the textbook phase vocoder of the
 *     reference's milestone slides.  Pinned only by this oracle and by
 *     numpy fp64 cross-checks on well-conditioned inputs.
 *
 * Numerical contract (shared, by specification, with the GPU path; version
 * PVR_CONTRACT_VERSION, reported by the GPU library as pv_contract_version()):
 *   PV_STANDARD analysis is defined as an exact sequence of IEEE fp32 operations
 *   (radix-2 Stockham FFT of hpfft.cu:145-203 with tabled twiddles, the real-FFT split,
 *   sqrtf, the polynomial atan2 below, the unwrap decision).  Version 2 (round 4): the
 *   split accumulates the odd part's twiddle product with two fused operations per
 *   component, and the decision rounds the exact product d * (1/2pi) once (fmaf onto the
 *   1.5*2^23 integer grid) instead of rounding the product and then rintf.  Version 3:
 *   for L = N/2 in [128, 512] the FFT is a Stockham FFT of twiddle-first radix-(L/64) passes
 *   with R-point DIF butterflies (pvr_fft_c32_v3); L >= 1024 keeps the radix-2 Stockham
 *   stages.  Version 4 (round 5): atan2's ratio is clamped, a = min(max(mn * r, 0), 1)
 *   with NaN -> 0 (the GPU's clamp output modifier), so every phase is finite: a
 *   non-finite input sample makes the magnitudes of the frames that contain it NaN, but no
 *   unwrap decision becomes a huge integer that would shift the channel's output phase for
 *   the rest of the stream (later frames recover).  The GPU must reproduce these bit-for-bit, because
 *   the phase-unwrap decision (round((dphi - e_k)/2pi)) is discontinuous: any ulp of
 *   difference in a noise bin can flip it and change the output phase by 2*pi*rho.
 *   Everything downstream of the integer decisions is well-conditioned and is computed
 *   here in fp64 (the textbook recurrence), the GPU in fp32: parity there is tolerance
 *   based (<= 1e-5 RMS per sample, BASELINE.json north_star).
 */
#ifndef PVREF_H
#define PVREF_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PVR_CONTRACT_VERSION 4
int pvr_contract_version(void);

typedef struct { float x, y; } pvr_c32;
typedef struct { double x, y; } pvr_c64;

enum { PVR_TIME_SHIFT = 't', PVR_PITCH_SHIFT = 'p' };

/* ---------------- tables (double -> float recipes) ---------------- */
void pvr_hann_periodic(int N, float* w);                 /* 0.5-0.5cos(2 pi n/N)       */
void pvr_hamming_ref(int N, float* w);                   /* phaseVocoder.h:85-89        */
void pvr_hann_ref(int N, float* w);                      /* phaseVocoder.h:64-66 (1-arg)*/
void pvr_fft_twiddles(int L, pvr_c32* tw);               /* L/2 entries e^{-2 pi i m/L} */
void pvr_split_twiddles(int N, pvr_c32* tws);            /* N/2+1 entries e^{-2pi i k/N}*/
void pvr_expected_advance(int N, int hop, float* e, int* j); /* N/2+1: e_k, j_k        */

/* ---------------- fp32 contract primitives ---------------- */
float pvr_atan2f(float y, float x);
/* radix-2 Stockham (hpfft.cu:145-167 stage structure); result in data; tmp = L scratch */
void pvr_fft_c32(pvr_c32* data, pvr_c32* tmp, int L, const pvr_c32* tw, int inverse);
/* real FFT of N windowed samples -> N/2+1 bins (contract of the GPU analysis) */
/* contract v3 FFT (L in [128, 512]; see pvref.c) */
int pvr_fft_v3_applies(int L);
int pvr_fft_v3_table_size(int L);
void pvr_fft_v3_table(int L, pvr_c32* t);
void pvr_fft_c32_v3(pvr_c32* data, pvr_c32* tmp, int L, const pvr_c32* ptab, int inverse);
void pvr_split_c32(const pvr_c32* z, int L, const pvr_c32* tws, pvr_c32* X);
void pvr_rfft_win_c32(const float* x, const float* w, int N, const pvr_c32* tw, const pvr_c32* tws,
                      pvr_c32* X, pvr_c32* work);
void pvr_rfft_c32(const float* xw, int N, const pvr_c32* tw, const pvr_c32* tws,
                  pvr_c32* X, pvr_c32* work);
int pvr_unwrap_count(float phi, float phi_prev, float e);

/* ---------------- geometry helpers ---------------- */
int pvr_num_frames(long n, int hop);                     /* main.cpp:231 loop count     */
int pvr_out_hop(int N, int hop_div, int effect, float scale);

/* ---------------- PV_STANDARD ---------------- */
/* fp32 contract analysis: spec[t*(N/2+1)+k] = {mag, phase}; frames t read x[t*hop ...],
 * samples at index >= n read as 0. */
void pvr_std_analysis(const float* x, long n, int N, int hop, int frames, pvr_c32* spec);
/* full path: contract analysis + integer unwrap decisions + fp64 textbook synthesis.
 * out has frames*hop_s + N - hop_s samples (full overlap-add).  Returns hop_s. */
int pvr_std_process(const float* x, long n, int N, int hop_div, int effect, float scale,
                    int frames, double* out);

/* ---------------- REF_COMPAT (fp64 literal restatement) ---------------- */
/* one frame: x -> 2N {mag, atan(y/x)} (kernel.cu:299-348). nan_faithful=0: x=y=0 -> phase 0 */
void pvr_compat_analysis_frame(const float* frame, int N, const float* win,
                               pvr_c64* spec2N, int nan_faithful);
/* one frame resynthesis (kernel.cu:352-432) into y[N] (before OLA) */
void pvr_compat_resynth_frame(const pvr_c64* spec2N, int N, const float* win, double* y);
/* whole signal: analysis of `frames` frames, running OLA (main.cpp:253-297) over
 * `frames` resynthesis frames; out has frames*hop + N - hop samples. Returns hop. */
int pvr_compat_process(const float* x, long n, int N, int hop_div, int frames, double* out);
/* same with the caller's window (NULL = the 4-argument constructor's Hamming) and the
 * NaN-faithful phase of all-zero bins (kernel.cu:101-109; NaN then poisons the frame's
 * resynthesis and the N samples of overlap-add it touches, as in the reference). */
int pvr_compat_process_ex(const float* x, long n, int N, int hop_div, int frames,
                          const float* window, int nan_faithful, double* out);
/* the same with the out hop hs of a time scale (phaseVocoder.h:74, phaseVocoder.cpp:68):
 * out holds frames * hs + (N - hs) samples */
int pvr_compat_process_hs(const float* x, long n, int N, int hop_div, int hs, int frames,
                          const float* window, int nan_faithful, double* out);

/* ---------------- fp64 helpers (exposed for tests) ---------------- */
void pvr_fft_c64(pvr_c64* data, int L, int inverse);     /* unnormalised radix-2 DIT    */

/* ---------------- batched CPU baseline (OpenMP over channels) ---------------- */
/* x: C channels with stride ldx; out: C channels with stride ldo. Returns threads used. */
int pvr_std_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                          int effect, float scale, int frames, float* out, long ldo,
                          int threads);
/* the fp32 CPU port (oracle/pvport.c, bench.py's cpu_baseline): same arguments */
int pvr_port_std_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                               int effect, float scale, int frames, float* out, long ldo,
                               int threads);
/* the fp32 CPU port of REF_COMPAT (oracle/pvport.c, the compat line's cpu_baseline) */
int pvr_port_compat_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                                  int frames, float* out, long ldo, int threads);
/* REF_COMPAT (pvr_compat_process, the 4-argument constructor's Hamming) per channel */
int pvr_compat_process_batch(const float* x, long ldx, long n, int C, int N, int hop_div,
                             int frames, float* out, long ldo, int threads);

#ifdef __cplusplus
}
#endif
#endif
