// phaseVocoder.h — header-only C++ drop-in for the reference's `class PhaseVocoder`
// (src/phaseVocoder.h:9-139, src/phaseVocoder.cpp:20-78) on top of the libpv C-ABI
// (include/pv.h).  Same class / enum / member / method names and argument meaning;
// buffers are device pointers (hipMalloc or hipMallocManaged), calls are synchronous on
// the default stream like the reference (cudaStreamSynchronize around every call,
// phaseVocoder.cpp:28-30), and failures print and exit like checkCUDAError_
// (src/io.cpp:115-124).
//
// What differs by construction: cuFFT plans, the three CUDA streams and
// the managed-memory attach calls do not exist (the handle owns its tables); the window
// table `imp` is a device copy of the same symmetric Hamming recipe (phaseVocoder.h:85-89).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pv.h"

#ifndef PV_DEFAULT_MAX_FRAMES
#define PV_DEFAULT_MAX_FRAMES 65536
#endif

enum Effect { TIME_SHIFT = 't', PITCH_SHIFT = 'p' };  // phaseVocoder.h:5-8

class PhaseVocoder {
   public:
    float* imp = nullptr;  // analysis/synthesis window (device), phaseVocoder.h:16
    int hopSize = 0;       // phaseVocoder.h:25
    int nSamps = 0;        // phaseVocoder.h:26
    int R = 1;
    int N = 0;
    float timeScale = 1.0f;  // phaseVocoder.h:29
    int outHopSize = 0;      // phaseVocoder.h:30
    int plan = 0;            // the cuFFT plan handle has no counterpart (kept for source compat)
    pv_handle* handle = nullptr;

    static void checkCUDAErrori(pv_status st, const char* msg, int line) {
        if (st != PV_OK) {  // phaseVocoder.h:35-44 / io.cpp:115-124: print + exit
            if (line >= -1) std::fprintf(stderr, "Line %d: ", line);
            std::fprintf(stderr, "Cuda error: %s: %s.\n", msg, pv_last_error());
            std::exit(EXIT_FAILURE);
        }
    }

    // phaseVocoder.h:46: PhaseVocoder(int samples) -> hop = samples/2, timeScale 1
    explicit PhaseVocoder(int samples, pv_mode mode = PV_MODE_REF_COMPAT)
        : PhaseVocoder(samples, TIME_SHIFT, 1.0f, 2, mode) {}

    // phaseVocoder.h:79-116: hop = samples / hop (the 4th argument is a divisor)
    PhaseVocoder(int samples, Effect e, float scaleFactor, int hop,
                 pv_mode mode = PV_MODE_REF_COMPAT, int max_channels = 1,
                 int max_frames = PV_DEFAULT_MAX_FRAMES, int device = 0) {
        pv_config cfg{};
        cfg.n_samps = samples;
        cfg.hop_div = hop;
        cfg.effect = (int)e;
        cfg.scale = scaleFactor;
        cfg.mode = (int)mode;
        cfg.max_channels = max_channels;
        cfg.max_frames = max_frames;
        cfg.device = device;
        checkCUDAErrori(pv_create(&cfg, &handle), "PhaseVocoder constructor", __LINE__);
        pv_info info{};
        pv_get_info(handle, &info);
        nSamps = N = info.n_samps;
        hopSize = info.hop;
        outHopSize = info.out_hop;
        timeScale = (e == TIME_SHIFT) ? scaleFactor : 1.0f;
        spec_stride_ = info.spec_stride;
        // imp: same recipe as phaseVocoder.h:85-89 (float omega, float cos)
        std::vector<float> w(samples);
        const float omega = (float)(2.0 * 3.14159265358979323846 / (samples - 1));
        for (int i = 0; i < samples; ++i) w[i] = 0.54f - 0.46f * cosf(omega * (float)i);
        if (mode == PV_MODE_STANDARD)
            for (int i = 0; i < samples; ++i)
                w[i] = (float)(0.5 - 0.5 * std::cos(2.0 * 3.14159265358979323846 * i / samples));
        if (hipMalloc((void**)&imp, sizeof(float) * samples) != hipSuccess ||
            hipMemcpy(imp, w.data(), sizeof(float) * samples, hipMemcpyHostToDevice) != hipSuccess)
            checkCUDAErrori(PV_ERR_HIP, "Malloc imp error", __LINE__);
    }

    PhaseVocoder(const PhaseVocoder&) = delete;
    PhaseVocoder& operator=(const PhaseVocoder&) = delete;
    ~PhaseVocoder() {  // phaseVocoder.h:128-130
        if (imp) (void)hipFree(imp);
        pv_destroy(handle);
    }

    int specStride() const { return spec_stride_; }

    // phaseVocoder.cpp:25-33 -> kernel.cu:299-348: one nSamps frame -> `output`
    // (2N float2 {mag, phase} in REF_COMPAT; N/2+1 in STANDARD).  `fft`, `intermediary`
    // are unused, as the reference's cuFFT path leaves `fft` untouched.
    void analysis_CUFFT(float* input, float2* output, float2* fft, float* intermediary) {
        (void)fft;
        (void)intermediary;
        checkCUDAErrori(pv_analysis(handle, input, nSamps, nSamps, 1, 1, (pv_float2*)output,
                                    spec_stride_, nullptr),
                        "pv_analysis ", __LINE__);
        sync();
    }
    // phaseVocoder.cpp:34-42 (hand-FFT path): same contract on this implementation
    void analysis(float* input, float2* output, float2* fft, float* intermediary) {
        analysis_CUFFT(input, output, fft, intermediary);
    }

    // phaseVocoder.cpp:60-76 -> kernel.cu:352-432: output[0..N) = frame(frontFrame) +
    // backFrame[outHop..N) (cudaOverlapAdd, kernel.cu:111-119)
    void resynthesis_CUFFT(float* backFrame, float2* frontFrame, float* output) {
        checkCUDAErrori(pv_resynthesis(handle, (const pv_float2*)frontFrame, spec_stride_, 1, 1,
                                       backFrame + outHopSize, nSamps, output, nSamps, nullptr),
                        "resynthesis", __LINE__);
        sync();
    }
    // phaseVocoder.cpp:44-58 (hand-FFT path): same contract on this implementation
    void resynthesis(float* backFrame, float2* frontFrame, float2* intermediary, float* output) {
        (void)intermediary;
        resynthesis_CUFFT(backFrame, frontFrame, output);
    }

    // phaseVocoder.cpp:20-23 -> kernel.cu:289-298: window, shift, unshift, window, OLA
    // (identity processing: output = w^2 * input + backFrame tail)
    void test_overlap_add(float* input, float* output, float* intermediary, float* backFrame, int n);

   private:
    int spec_stride_ = 0;
    static void sync() {
        if (hipStreamSynchronize(nullptr) != hipSuccess)
            checkCUDAErrori(PV_ERR_HIP, "stream sync error", __LINE__);
    }
};

inline void PhaseVocoder::test_overlap_add(float* input, float* output, float* intermediary,
                                           float* backFrame, int n) {
    (void)intermediary;
    checkCUDAErrori(pv_test_overlap_add(input, imp, backFrame, output, n, hopSize, nullptr),
                    "test_overlap_add", __LINE__);
    sync();
}
