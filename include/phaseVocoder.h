// phaseVocoder.h — header-only C++ drop-in for the reference's `class PhaseVocoder`
// (src/phaseVocoder.h:9-139, src/phaseVocoder.cpp:20-78) on top of the libpv C-ABI
// (include/pv.h) and the CudaPhase drop-in (include/kernel.h).  Same class / enum /
// member / method names and argument meaning; buffers are device or managed pointers
// (hipMalloc / hipMallocManaged); calls are synchronous on the default stream like the
// reference (cudaStreamSynchronize around every call, phaseVocoder.cpp:28-30); failures
// print and exit like checkCUDAError_ (src/io.cpp:115-124).
//
// Layering as in the reference: in REF_COMPAT mode the per-frame methods call
// CudaPhase::pv_analysis_CUFFT / resynthesis_CUFFT / test_overlap_add with this->imp as
// the window (phaseVocoder.cpp:20-76), so CudaPhase::timer() times them as main.cpp:240
// and :277 expect.  The two constructors build the reference's two windows:
//   PhaseVocoder(int samples)                    periodic Hann 0.5f*(1-cosf(2 pi i/N)),
//                                                hop N/2, timeScale 1 (phaseVocoder.h:46-78)
//   PhaseVocoder(int samples, Effect, float, int) symmetric Hamming, hop N/div
//                                                (phaseVocoder.h:79-116)
// The batched handle `handle` (pv_process etc.) is created with the same window.
//
// Real time (main.cpp:45-59 `callback`, RT block): the callback memcpys one RtAudio buffer
// into `curr_input` and calls analysis(); the reference declares analysis() and
// analysis(float*) (phaseVocoder.h:131-132) but only sketches them (phaseVocoder.cpp:6-19:
// pv_analysis_RT of the new samples on a round-robin stream).  Here they push the buffer's
// nSamps samples (main.cpp:85: bufferSize = nSamps) through libpv's real-time stream
// (pv_rt_push: input history, phases, unwrap counts and the overlap accumulator stay on the
// device between callbacks): the spectra of the buffer's nSamps/hopSize frames land in
// `curr_mag_phase`, the buffer's nSamps/hopSize * outHopSize emitted samples in
// `prev_output`.  The stream runs the STANDARD pipeline (the phase vocoder the reference's
// real-time design plans, README.md:46-50, with the object's effect and scale).
//
// What differs by construction: no cuFFT plans (`plan`, `ifft` are 0), the
// managed-memory attach calls do not exist, the real-time buffers are allocated by both
// constructors (sized for one callback), and STANDARD mode (an extension: the textbook
// vocoder the reference never implemented) runs on `handle` directly.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernel.h"
#include "pv.h"

#ifndef PV_DEFAULT_MAX_FRAMES
#define PV_DEFAULT_MAX_FRAMES 65536
#endif
#define NUM_STREAMS 3  // phaseVocoder.h:4

enum Effect { TIME_SHIFT = 't', PITCH_SHIFT = 'p' };  // phaseVocoder.h:5-8

class PhaseVocoder {
   public:
    float* imp = nullptr;              // analysis/synthesis window (managed), phaseVocoder.h:16
    float* imp1 = nullptr;             // phaseVocoder.h:17 (second window, unused by the path)
    float* curr_input = nullptr;       // real-time buffers, phaseVocoder.h:18-22 (managed,
    float* prev_input = nullptr;       //   allocated by the 1-argument constructor as in the
    float* prev_output = nullptr;      //   reference; main.cpp:49 memcpys into curr_input)
    float2* prev_mag_phase = nullptr;
    float2* curr_mag_phase = nullptr;
    int plan = 0, ifft = 0;  // the cuFFT plans have no counterpart (kept for source compat)
    int hopSize = 0;         // phaseVocoder.h:25
    int nSamps = 0;          // phaseVocoder.h:26
    int R = 1;
    int N = 0;
    float timeScale = 1.0f;  // phaseVocoder.h:29
    int outHopSize = 0;      // phaseVocoder.h:30
    int stream = 0;          // phaseVocoder.h:31
    hipStream_t streams[NUM_STREAMS] = {};
    pv_handle* handle = nullptr;  // batched C-ABI handle (same configuration and window)

    static void checkCUDAErrori(pv_status st, const char* msg, int line) {
        if (st != PV_OK) {  // phaseVocoder.h:35-44 / io.cpp:115-124: print + exit
            if (line >= -1) std::fprintf(stderr, "Line %d: ", line);
            std::fprintf(stderr, "Cuda error: %s: %s.\n", msg, pv_last_error());
            std::exit(EXIT_FAILURE);
        }
    }

    // phaseVocoder.h:46-78: hop = samples/2, timeScale 1, periodic Hann
    // imp[i] = 0.5f*(1.f - cosf(2.f*M_PI*i/samples)); the real-time buffers are allocated
    explicit PhaseVocoder(int samples, int max_channels = 1, int max_frames = PV_DEFAULT_MAX_FRAMES,
                          int device = 0)
        : PhaseVocoder(samples, PV_MODE_REF_COMPAT, max_channels, max_frames, device) {}

    // PhaseVocoder(int samples) with the mode chosen: REF_COMPAT is the 1-argument
    // constructor; STANDARD takes its geometry (hop N/2, time scale 1) with the STANDARD
    // periodic Hann window.  (Keeps `PhaseVocoder(N, PV_MODE_STANDARD)` from converting the
    // enum to the 1-argument constructor's max_channels.)
    PhaseVocoder(int samples, pv_mode mode, int max_channels = 1, int max_frames = PV_DEFAULT_MAX_FRAMES,
                 int device = 0) {
        init(samples, TIME_SHIFT, 1.0f, 2, mode, mode == PV_MODE_REF_COMPAT ? PV_WINDOW_HANN_REF : PV_WINDOW_DEFAULT,
             max_channels, max_frames, device);
        std::vector<float> w(2 * (size_t)samples);  // imp1: 2N entries (the reference writes
        for (int i = 0; i < 2 * samples; ++i)          // 2N into an N-float buffer)
            w[i] = 0.5f * (1.f - cosf((float)(2.0 * M_PI * (double)i / (double)samples)));
        imp1 = managed_copy(w.data(), 2 * (size_t)samples, "Malloc imp1 error");
    }

    // phaseVocoder.h:79-116: hop = samples / hop (the 4th argument is a divisor), symmetric
    // Hamming; TIME_SHIFT: outHopSize = scaleFactor*hopSize.  `mode` selects REF_COMPAT
    // (the reference's path, default) or STANDARD (the textbook vocoder, an extension).
    PhaseVocoder(int samples, Effect e, float scaleFactor, int hop,
                 pv_mode mode = PV_MODE_REF_COMPAT, int max_channels = 1,
                 int max_frames = PV_DEFAULT_MAX_FRAMES, int device = 0) {
        init(samples, e, scaleFactor, hop, mode, PV_WINDOW_DEFAULT, max_channels, max_frames, device);
        const float omega1 = (float)(2.0 * M_PI / (2 * samples - 1));  // phaseVocoder.h:90-94
        std::vector<float> w(samples);
        for (int i = 0; i < samples; ++i) w[i] = 0.54f - 0.46f * cosf(omega1 * (float)i);
        imp1 = managed_copy(w.data(), samples, "Malloc imp1 error");
    }

    PhaseVocoder(const PhaseVocoder&) = delete;
    PhaseVocoder& operator=(const PhaseVocoder&) = delete;
    ~PhaseVocoder() {  // phaseVocoder.h:128-130 frees imp; the rest is released here too
        void* bufs[] = {imp, imp1, curr_input, prev_input, prev_output, prev_mag_phase, curr_mag_phase};
        for (void* b : bufs)
            if (b) (void)hipFree(b);
        for (auto& s : streams)
            if (s) (void)hipStreamDestroy(s);
        pv_rt_destroy(rt_);
        pv_destroy(handle);
    }

    int specStride() const { return spec_stride_; }
    pv_mode mode() const { return mode_; }

    // phaseVocoder.h:118-126
    hipStream_t* getStream() {
        hipStream_t* out = &streams[stream++];
        stream %= NUM_STREAMS;
        return out;
    }
    hipStream_t* getPrevStream() { return &streams[(stream + NUM_STREAMS - 1) % NUM_STREAMS]; }

    // phaseVocoder.cpp:25-33 -> kernel.cu:299-348: one nSamps frame -> `output`
    // (2N float2 {mag, phase} in REF_COMPAT; N/2+1 in STANDARD)
    void analysis_CUFFT(float* input, float2* output, float2* fft, float* intermediary) {
        sync();
        if (mode_ == PV_MODE_REF_COMPAT) {
            CudaPhase::pv_analysis_CUFFT(output, fft, input, intermediary, imp, nSamps);
        } else {
            checkCUDAErrori(pv_analysis(handle, input, nSamps, nSamps, 1, 1, (pv_float2*)output,
                                        spec_stride_, nullptr),
                            "pv_analysis ", __LINE__);
        }
        sync();
    }
    // phaseVocoder.cpp:34-42 (hand-FFT path) -> CudaPhase::pv_analysis: same contract here
    void analysis(float* input, float2* output, float2* fft, float* intermediary) {
        analysis_CUFFT(input, output, fft, intermediary);
    }

    // phaseVocoder.cpp:60-76 -> kernel.cu:352-432: output[0..N) = frame(frontFrame) +
    // backFrame[outHop..N) (cudaOverlapAdd, kernel.cu:111-119)
    void resynthesis_CUFFT(float* backFrame, float2* frontFrame, float* output) {
        sync();
        if (mode_ == PV_MODE_REF_COMPAT) {
            CudaPhase::resynthesis_CUFFT(output, backFrame, frontFrame, imp, nSamps, outHopSize);
        } else {
            checkCUDAErrori(pv_resynthesis(handle, (const pv_float2*)frontFrame, spec_stride_, 1, 1,
                                           backFrame + outHopSize, nSamps, output, nSamps, nullptr),
                            "resynthesis", __LINE__);
        }
        sync();
    }
    // phaseVocoder.cpp:44-58 (hand-FFT path) -> CudaPhase::resynthesis: same contract here
    void resynthesis(float* backFrame, float2* frontFrame, float2* intermediary, float* output) {
        if (mode_ == PV_MODE_REF_COMPAT) {
            sync();
            CudaPhase::resynthesis(output, backFrame, frontFrame, intermediary, imp, nSamps, outHopSize);
            sync();
        } else {
            resynthesis_CUFFT(backFrame, frontFrame, output);
        }
    }
    // phaseVocoder.cpp:77-78: the processing-hook overload has an empty body in the
    // reference (its planned processing stage, README.md:22-23); it does nothing here either
    // (neither the hook nor a resynthesis runs)
    void resynthesis(float* backFrame, float2* magFreq, float* output, void (*processing)()) {
        (void)backFrame;
        (void)magFreq;
        (void)output;
        (void)processing;
    }

    // phaseVocoder.h:132, main.cpp:53-54: one RtAudio buffer of nSamps samples (host-written
    // managed or device memory) through the real-time stream; emitted samples ->
    // prev_output (rtOutputSamples() of them), analysed rows -> curr_mag_phase
    // (rtFrames() rows of specStride() {mag, phase} float2 each).  Synchronous.
    void analysis(float* input) {
        ensure_rt();
        sync();
        const int fr = rtFrames();
        checkCUDAErrori(pv_rt_push(rt_, input, nSamps, fr, prev_output, (long long)fr * outHopSize,
                                   (pv_float2*)curr_mag_phase, (long long)fr * rt_spec_stride_, nullptr),
                        "pv_analysis_RT", __LINE__);
        sync();
    }
    // phaseVocoder.h:131: the callback's form, on curr_input (main.cpp:53 memcpys into it)
    void analysis() { analysis(curr_input); }
    int rtFrames() const { return hopSize > 0 ? nSamps / hopSize : 0; }  // frames per buffer
    int rtOutputSamples() const { return rtFrames() * outHopSize; }    // emitted per buffer
    int rtSpecStride() const { return rt_spec_stride_; }               // float2 per curr_mag_phase row
    // start a new real-time stream (zero history, phases, overlap accumulator)
    void rtReset() {
        ensure_rt();
        checkCUDAErrori(pv_rt_reset(rt_, nullptr), "pv_rt_reset", __LINE__);
        sync();
    }

    // phaseVocoder.cpp:20-23 -> kernel.cu:289-298: window, shift, unshift, window, OLA
    // (identity processing: output = w^2 * input + backFrame tail)
    void test_overlap_add(float* input, float* output, float* intermediary, float* backFrame, int n) {
        sync();
        CudaPhase::test_overlap_add(input, output, intermediary, backFrame, imp, n, hopSize);
        sync();
    }

   private:
    int spec_stride_ = 0;
    pv_mode mode_ = PV_MODE_REF_COMPAT;
    Effect effect_ = TIME_SHIFT;
    float scale_ = 1.0f;
    int device_ = 0;
    pv_rt* rt_ = nullptr;  // real-time stream behind analysis() (created on first use)
    int rt_spec_stride_ = 0;

    void ensure_rt() {
        if (rt_) return;
        pv_config cfg{};
        cfg.abi_version = PV_ABI_VERSION;
        cfg.n_samps = nSamps;
        cfg.hop_div = nSamps / hopSize;
        cfg.effect = (int)effect_;
        cfg.scale = scale_;
        cfg.mode = PV_MODE_STANDARD;
        cfg.max_channels = 1;
        cfg.max_frames = rtFrames();
        cfg.device = device_;
        checkCUDAErrori(pv_rt_create(&cfg, 1, &rt_), "pv_rt_create", __LINE__);
    }
    void alloc_rt_buffers() {
        // sized for one callback of nSamps samples (the reference's sizes are per frame)
        const size_t N = (size_t)nSamps, fr = (size_t)rtFrames();
        rt_spec_stride_ = (int)(((N / 2 + 1) + 7) & ~(size_t)7);
        const size_t out_n = std::max(N, fr * (size_t)outHopSize);
        prev_mag_phase = (float2*)managed_zero(sizeof(float2) * fr * rt_spec_stride_, "Malloc prev_mag_phase error");
        prev_input = (float*)managed_zero(sizeof(float) * N, "Malloc prev_input");
        prev_output = (float*)managed_zero(sizeof(float) * out_n, "Malloc prev_output");
        curr_mag_phase = (float2*)managed_zero(sizeof(float2) * fr * rt_spec_stride_, "Malloc curr_mag_phase");
        curr_input = (float*)managed_zero(sizeof(float) * N, "Malloc curr_input");
    }

    static void sync() {
        if (hipStreamSynchronize(nullptr) != hipSuccess)
            checkCUDAErrori(PV_ERR_HIP, "stream sync error", __LINE__);
    }
    static float* managed_copy(const float* src, size_t n, const char* what) {
        float* p = nullptr;
        if (hipMallocManaged((void**)&p, sizeof(float) * n) != hipSuccess) checkCUDAErrori(PV_ERR_HIP, what, __LINE__);
        for (size_t i = 0; i < n; ++i) p[i] = src[i];
        return p;
    }
    static void* managed_zero(size_t bytes, const char* what) {
        void* p = nullptr;
        if (hipMallocManaged(&p, bytes) != hipSuccess) checkCUDAErrori(PV_ERR_HIP, what, __LINE__);
        std::memset(p, 0, bytes);
        return p;
    }

    void init(int samples, Effect e, float scaleFactor, int hop, pv_mode mode, int window,
              int max_channels, int max_frames, int device) {
        pv_config cfg{};
        cfg.abi_version = PV_ABI_VERSION;
        cfg.n_samps = samples;
        cfg.hop_div = hop;
        cfg.effect = (int)e;
        cfg.scale = scaleFactor;
        cfg.mode = (int)mode;
        cfg.max_channels = max_channels;
        cfg.max_frames = max_frames;
        cfg.device = device;
        cfg.window = window;
        cfg.nan_faithful = CudaPhase::detail::nan_faithful_flag();
        checkCUDAErrori(pv_create(&cfg, &handle), "PhaseVocoder constructor", __LINE__);
        pv_info info{};
        info.abi_version = PV_ABI_VERSION;
        pv_get_info(handle, &info);
        nSamps = N = info.n_samps;
        hopSize = info.hop;
        outHopSize = info.out_hop;
        timeScale = (e == TIME_SHIFT) ? scaleFactor : 1.0f;
        spec_stride_ = info.spec_stride;
        mode_ = mode;
        effect_ = e;
        scale_ = scaleFactor;
        device_ = device;
        // imp: the constructor's recipe (float argument, float cos as in the reference)
        std::vector<float> w(samples);
        if (mode == PV_MODE_STANDARD) {
            for (int i = 0; i < samples; ++i)
                w[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / samples));
        } else if (window == PV_WINDOW_HANN_REF) {  // phaseVocoder.h:64-66
            for (int i = 0; i < samples; ++i)
                w[i] = 0.5f * (1.f - cosf((float)(2.0 * M_PI * (double)i / (double)samples)));
        } else {  // phaseVocoder.h:85-89
            const float omega = (float)(2.0 * M_PI / (samples - 1));
            for (int i = 0; i < samples; ++i) w[i] = 0.54f - 0.46f * cosf(omega * (float)i);
        }
        imp = managed_copy(w.data(), samples, "Malloc imp error");
        for (auto& s : streams)  // phaseVocoder.h:112-114
            if (hipStreamCreate(&s) != hipSuccess) checkCUDAErrori(PV_ERR_HIP, "stream create", __LINE__);
        alloc_rt_buffers();
    }
};
