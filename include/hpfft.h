// hpfft.h — header-only C++ drop-in for the reference's hand-written FFT API
// `FFT::HPFFT` (karnel/hpfft.h:6-11, karnel/hpfft.cu) on the libpv C-ABI (pv_fft_c2c).
//
//   computeGPUFFT(N, R, signal, intermediary)        hpfft.cu:187-193
//   computeGPUIFFT(N, R, signal, intermediary)       hpfft.cu:194-200
//   computeGPUFFT_RT / computeGPUIFFT_RT (+ stream)  hpfft.cu:173-186
//   computeFFTSh(h_signal, N, R, numThreads)         hpfft.cu:202-216 (host in -> malloc'd host out)
//   computeFFTCooley(h_signal, N, R, numThreads)     hpfft.cu:218-233 (host in -> malloc'd host out)
//   timer()                                          hpfft.cu:9-13
//
// Argument meaning kept: N points, radix R (the reference implements R = 2 only; other
// values print and exit), device buffers `signal` / `intermediary`, unnormalised in both
// directions.  Result location kept: the reference swaps only its local copies of the two
// pointers after each of the log2(N) stages (hpfft.cu:169-172), so the transform ends in
// `signal` when log2(N) is even and in `intermediary` when it is odd; so does this one.
// One batched launch replaces the reference's log2(N) single-block launches.
// computeFFTSh / computeFFTCooley return the correct forward DFT (the reference kernels
// FFTShMem / FFTCooley are only correct for particular N and thread counts).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "pv.h"

namespace FFT {
namespace HPFFT {

inline FFT::Common::PerformanceTimer& timer() {
    static FFT::Common::PerformanceTimer t;
    return t;
}

namespace detail {
inline void check(pv_status st, const char* what) {  // checkCUDAError_ (io.cpp:115-124)
    if (st != PV_OK) {
        std::fprintf(stderr, "Cuda error: %s: %s.\n", what, pv_last_error());
        std::exit(EXIT_FAILURE);
    }
}
inline int log2i(int n) {
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}
inline void run(int N, int R, float2* signal, float2* intermediary, int inverse, hipStream_t s,
                const char* what) {
    if (R != 2) {
        std::fprintf(stderr, "Cuda error: %s: radix %d not implemented (radix-2 only).\n", what, R);
        std::exit(EXIT_FAILURE);
    }
    float2* dst = (log2i(N) % 2 == 0) ? signal : intermediary;
    check(pv_fft_c2c((const pv_float2*)signal, (pv_float2*)dst, N, 1, inverse, s), what);
}
inline float2* host_fft(const float2* h_signal, int N, const char* what) {
    float2* d = nullptr;
    if (hipMalloc((void**)&d, sizeof(float2) * N) != hipSuccess) check(PV_ERR_NOMEM, what);
    (void)hipMemcpy(d, h_signal, sizeof(float2) * N, hipMemcpyHostToDevice);
    check(pv_fft_c2c((const pv_float2*)d, (pv_float2*)d, N, 1, 0, nullptr), what);
    float2* o = (float2*)std::malloc(sizeof(float2) * N);
    (void)hipMemcpy(o, d, sizeof(float2) * N, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return o;
}
}  // namespace detail

inline void computeGPUFFT(int N, int R, float2* h_signal, float2* intermediary) {
    detail::run(N, R, h_signal, intermediary, 0, nullptr, "computeGPUFFT");
}
inline void computeGPUIFFT(int N, int R, float2* h_signal, float2* intermediary) {
    detail::run(N, R, h_signal, intermediary, 1, nullptr, "computeGPUIFFT");
}
inline void computeGPUFFT_RT(int N, int R, float2* h_signal, float2* intermediary, hipStream_t* stream) {
    detail::run(N, R, h_signal, intermediary, 0, stream ? *stream : nullptr, "computeGPUFFT_RT");
}
inline void computeGPUIFFT_RT(int N, int R, float2* h_signal, float2* intermediary, hipStream_t* stream) {
    detail::run(N, R, h_signal, intermediary, 1, stream ? *stream : nullptr, "computeGPUIFFT_RT");
}
inline float2* computeFFTSh(float2* h_signal, int size, int radix, int numThreads) {
    (void)radix;
    (void)numThreads;
    return detail::host_fft(h_signal, size, "computeFFTSh");
}
inline float2* computeFFTCooley(float2* h_signal, int N, int R, int numThreads) {
    (void)R;
    (void)numThreads;
    return detail::host_fft(h_signal, N, "computeFFTCooley");
}

}  // namespace HPFFT
}  // namespace FFT
