// kernel.h — header-only C++ drop-in for the reference's `namespace CudaPhase`
// (karnel/kernel.h:13-21) on top of the libpv C-ABI (include/pv.h).
//
//   CudaPhase::pv_analysis_CUFFT(out2N, fft, in, interm, win, N)   kernel.cu:299-348
//   CudaPhase::resynthesis_CUFFT(out, back, spec, win, N, hop)     kernel.cu:352-432
//   CudaPhase::pv_analysis / resynthesis (hand-FFT variants)       kernel.cu:177-218, 262-288
//   CudaPhase::pv_analysis_RT(out2N, fft, in, interm, [win,] N, &s) kernel.cu:219-260, kernel.h:16
//   CudaPhase::test_overlap_add(...)                               kernel.cu:289-298
//   CudaPhase::timer()  PerformanceTimer (karnel/common.h:27-113) on hipEvents
//
// Every call runs the REF_COMPAT path of one frame on the legacy default stream and is
// bracketed by timer().startGpuTimer()/endGpuTimer() like the reference, so
// `CudaPhase::timer().getGpuElapsedTimeForPreviousOperation()` (main.cpp:240, :277) reads
// the call's device time.  The caller's window `win` (device or managed pointer, N floats)
// is honoured: it is handed to the handle with pv_set_window on every call, then multiplies
// the analysis frame (kernel.cu:301) and the resynthesised frame (kernel.cu:406).  `fft` /
// `intermediary` are unused (the window product stays on chip).  The handles behind the
// free functions are created on first use per (N, hop, nan_faithful) and cached for the
// process lifetime.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "pv.h"

namespace CudaPhase {

inline FFT::Common::PerformanceTimer& timer() {
    static FFT::Common::PerformanceTimer t;
    return t;
}

namespace detail {
inline void check(pv_status st, const char* msg) {  // checkCUDAError_ (io.cpp:115-124)
    if (st != PV_OK) {
        std::fprintf(stderr, "Cuda error: %s: %s.\n", msg, pv_last_error());
        std::exit(EXIT_FAILURE);
    }
}
// kernel.cu:101-109: atanf(0/0) = NaN for an all-zero bin (digital silence) poisons the
// frame; off by default (SURVEY.md §8c deviation 4), on = the reference's behaviour
inline int& nan_faithful_flag() {
    static int f = 0;
    return f;
}
inline pv_handle* compat_handle(int N, int hop) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int>, pv_handle*> cache;
    const int nf = nan_faithful_flag();
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({N, hop, nf});
    if (it != cache.end()) return it->second;
    pv_config cfg{};
    cfg.abi_version = PV_ABI_VERSION;
    cfg.n_samps = N;
    cfg.hop_div = (hop > 0 && N % hop == 0) ? N / hop : 2;
    cfg.effect = PV_TIME_SHIFT;
    cfg.scale = (hop > 0 && N % hop == 0) ? 1.0f : (float)hop / (float)(N / 2);
    cfg.mode = PV_MODE_REF_COMPAT;
    cfg.max_channels = 1;
    cfg.max_frames = 1;
    cfg.nan_faithful = nf;
    int dev = 0;
    (void)hipGetDevice(&dev);
    cfg.device = dev;
    pv_handle* h = nullptr;
    check(pv_create(&cfg, &h), "pv_create");
    cache[{N, hop, nf}] = h;
    return h;
}
// pv_analysis_RT's handle: REF_COMPAT with the inline periodic Hann of cudaWindow_HanRT
// (kernel.cu:85-91, = PV_WINDOW_HANN_REF) as its analysis window
inline pv_handle* rt_handle(int N) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int>, pv_handle*> cache;
    const int nf = nan_faithful_flag();
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({N, nf, dev});
    if (it != cache.end()) return it->second;
    pv_config cfg{};
    cfg.abi_version = PV_ABI_VERSION;
    cfg.n_samps = N;
    cfg.hop_div = 2;
    cfg.effect = PV_TIME_SHIFT;
    cfg.scale = 1.0f;
    cfg.mode = PV_MODE_REF_COMPAT;
    cfg.max_channels = 1;
    cfg.max_frames = 1;
    cfg.window = PV_WINDOW_HANN_REF;
    cfg.nan_faithful = nf;
    cfg.device = dev;
    pv_handle* h = nullptr;
    check(pv_create(&cfg, &h), "pv_create");
    cache[{N, nf, dev}] = h;
    return h;
}
inline int spec_stride(pv_handle* h) {
    pv_info info{};
    info.abi_version = PV_ABI_VERSION;
    pv_get_info(h, &info);
    return info.spec_stride;
}
}  // namespace detail

// Select the reference's NaN phase for all-zero bins (kernel.cu:101-109) for later calls.
inline void set_nan_faithful(bool on) { detail::nan_faithful_flag() = on ? 1 : 0; }

// kernel.cu:299-348: output = 2N {mag, atanf(Im/Re)} of the zero-phase, zero-padded,
// windowed frame input[0..N)
inline void pv_analysis_CUFFT(float2* output, float2* fft, float* input, float* intermediary,
                              float* win, int N) {
    (void)fft;
    (void)intermediary;
    timer().startGpuTimer();
    pv_handle* h = detail::compat_handle(N, N / 2);
    detail::check(pv_set_window(h, win, nullptr), "Window analysis");
    detail::check(pv_analysis(h, input, N, N, 1, 1, (pv_float2*)output, detail::spec_stride(h), nullptr),
                  "pv_analysis_CUFFT");
    timer().endGpuTimer();
}

// kernel.cu:352-432: output[0..N) = window * shift(C2R_N(timeScale(frontFrame)) / N)
// + backFrame[hopSize..N) shifted to the front (cudaOverlapAdd, kernel.cu:111-119).
// frontFrame is read only here (the reference's in-place cudaTimeScale clobbers it).
inline void resynthesis_CUFFT(float* output, float* backFrame, float2* frontFrame, float* win,
                              int N, int hopSize) {
    timer().startGpuTimer();
    pv_handle* h = detail::compat_handle(N, hopSize);
    detail::check(pv_set_window(h, win, nullptr), "window error");
    detail::check(pv_resynthesis(h, (const pv_float2*)frontFrame, detail::spec_stride(h), 1, 1,
                                 backFrame + hopSize, N, output, N, nullptr),
                  "resynthesis_CUFFT");
    timer().endGpuTimer();
}

// kernel.cu:177-218 / 262-288: the hand-FFT variants compute the same contract here
inline void pv_analysis(float2* output, float2* fft, float* input, float* intermediary, float* win,
                        int N) {
    pv_analysis_CUFFT(output, fft, input, intermediary, win, N);
}
inline void resynthesis(float* output, float* backFrame, float2* frontFrame, float2* intermediary,
                        float* win, int N, int hopSize) {
    (void)intermediary;
    resynthesis_CUFFT(output, backFrame, frontFrame, win, N, hopSize);
}

// kernel.cu:219-260 (the defined signature; `win` is unused there too): the frame
// input[0..N) windowed by the inline periodic Hann of cudaWindow_HanRT (kernel.cu:85-91),
// zero-phase shift + zero pad to 2N (cufftShiftPadZeros), 2N-point forward FFT
// (computeGPUFFT_RT), then {mag, atanf(Im/Re)} of all 2N bins in place (cudaMagFreq) ->
// output, all enqueued on *stream (the legacy default stream when stream is null) and not
// waited for, like the reference.  The FFT is the correct DFT: the reference's hand FFT
// leaves an odd stage count's result in `fft` (hpfft.cu:169-173), which is
// not reproduced.  `fft` / `intermediary` are unused (the product stays on chip).
inline void pv_analysis_RT(float2* output, float2* fft, float* input, float* intermediary, float* win,
                           int N, hipStream_t* stream) {
    (void)fft;
    (void)intermediary;
    (void)win;
    pv_handle* h = detail::rt_handle(N);
    detail::check(pv_analysis(h, input, N, N, 1, 1, (pv_float2*)output, detail::spec_stride(h),
                              stream ? (void*)*stream : nullptr),
                  "pv_analysis_RT");
}
// kernel.h:16 declares it without `win`
inline void pv_analysis_RT(float2* output, float2* fft, float* input, float* intermediary, int N,
                           hipStream_t* stream) {
    pv_analysis_RT(output, fft, input, intermediary, nullptr, N, stream);
}

// kernel.cu:289-298: window, shift, unshift, window, overlap-add (identity processing)
inline void test_overlap_add(float* input, float* output, float* intermediary, float* backFrame,
                             float* win, int N, int hopSize) {
    (void)intermediary;
    timer().startGpuTimer();
    detail::check(pv_test_overlap_add(input, win, backFrame, output, N, hopSize, nullptr),
                  "test_overlap_add");
    timer().endGpuTimer();
}

}  // namespace CudaPhase
