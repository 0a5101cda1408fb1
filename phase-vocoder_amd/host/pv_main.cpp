// pv_main.cpp — the build's counterpart of the reference driver src/main.cpp (offline
// vocoding of a WAV file).  main.cpp itself cannot compile unchanged (it calls the CUDA
// runtime, cuFFT and RtAudio directly and hard-codes /home/davis/... paths),
// so this driver keeps its argv positions and its offline loop on top of the drop-in
// headers (include/phaseVocoder.h), plus a batched mode that runs every channel through
// one pv_process call.
//
//   pv_main <in.wav> [effect t|p] [out.wav] [options]
//     --N 256 --hopdiv 2 --scale 1       PhaseVocoder(256, effect, 1, 2)  (main.cpp:84)
//     --mode ref|std                     REF_COMPAT (default) or PV_STANDARD
//     --batched                          all channels in one pv_process call
//     --single-arg                       PhaseVocoder(N): periodic Hann, hop N/2 (phaseVocoder.h:46-78)
//     --nan-faithful                     atanf(0/0) = NaN phases as the reference (kernel.cu:101-109)
//     --timer                            print CudaPhase::timer() per call (main.cpp:238-241, 275-278)
//     --dump-f32 <file>                  raw float32 of the emitted channel-0 samples
//     --rt                               main.cpp's RT block instead of the offline loop: the
//                                        RtAudio `callback` (main.cpp:45-59) is called on
//                                        successive nSamps-sample buffers of channel 0
//                                        (main.cpp:85 bufferSize = nSamps); each memcpys into
//                                        curr_input and runs analysis(); the buffer's emitted
//                                        samples (prev_output) are the output stream
//
// The per-frame REF_COMPAT calls go PhaseVocoder -> CudaPhase (include/kernel.h) with the
// object's window, as phaseVocoder.cpp -> kernel.cu do.
// Per-frame mode reproduces main.cpp:204-309: analysis_CUFFT of every channel's frames
// i = 0, hop, ... < n - hop into pre-zeroed 2N-bin spectra; resynthesis of frames
// i < n/outHop with the running backFrame (main.cpp:253-297); only channel 0 is
// resynthesised and duplicated into R (the `numChannels = 1` assignment, main.cpp:288);
// output is 16-bit stereo of timeScale*n samples (main.cpp:140-143).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/phaseVocoder.h"
#include "wav.hpp"

#define HIPCHECK(x)                                                                   \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "Line %d: Cuda error: %s: %s.\n", __LINE__, #x,      \
                         hipGetErrorString(e_));                                      \
            std::exit(EXIT_FAILURE);                                                  \
        }                                                                             \
    } while (0)

// main.cpp:45-59 (RT): the RtAudio callback, on this build's drop-in.  The output buffer
// receives the buffer's emitted samples (the reference leaves its resynthesis commented
// out, main.cpp:55).
static int callback(void* outputBuffer, void* inputBuffer, unsigned int nBufferFrames, double streamTime,
                    unsigned int status, void* UserData) {
    (void)streamTime;
    PhaseVocoder* pv = (PhaseVocoder*)UserData;
    if (status) std::printf("Stream underflow detected!\n");
    std::memcpy(pv->curr_input, inputBuffer, sizeof(float) * nBufferFrames);  // main.cpp:53
    pv->analysis();                                                            // main.cpp:54
    // the buffer's emitted samples, never more than the device buffer holds (main() rejects
    // an RT run whose buffers emit more than they take: a stretch above 1)
    const unsigned int n = std::min<unsigned int>((unsigned int)pv->rtOutputSamples(), nBufferFrames);
    std::memcpy(outputBuffer, pv->prev_output, sizeof(float) * n);
    return 0;
}

int main(int argc, char** argv) {
    std::string in = "testtones/1000sine.wav", out = "out.wav", dump;
    Effect effect = TIME_SHIFT;
    int N = 256, hopdiv = 2;
    float scale = 1.0f;
    bool batched = false, single_arg = false, show_timer = false, rt = false;
    double ana_ms = 0.0, syn_ms = 0.0;
    pv_mode mode = PV_MODE_REF_COMPAT;
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--N" && i + 1 < argc) N = std::atoi(argv[++i]);
        else if (a == "--hopdiv" && i + 1 < argc) hopdiv = std::atoi(argv[++i]);
        else if (a == "--scale" && i + 1 < argc) scale = (float)std::atof(argv[++i]);
        else if (a == "--mode" && i + 1 < argc) mode = std::string(argv[++i]) == "std" ? PV_MODE_STANDARD : PV_MODE_REF_COMPAT;
        else if (a == "--batched") batched = true;
        else if (a == "--single-arg") single_arg = true;
        else if (a == "--nan-faithful") CudaPhase::set_nan_faithful(true);
        else if (a == "--timer") show_timer = true;
        else if (a == "--dump-f32" && i + 1 < argc) dump = argv[++i];
        else if (a == "--rt") rt = true;
        else pos.push_back(a);
    }
    if (pos.size() >= 1) in = pos[0];                                    // main.cpp:69-81
    if (pos.size() >= 2) effect = static_cast<Effect>(pos[1][0]);
    if (pos.size() >= 3) out = pos[2];

    std::printf("Offline Vocoding\n");
    pvwav::Audio audio;
    std::string err;
    if (!pvwav::load(in, audio, err)) {
        std::printf("err: wav failed to load (%s)\n", err.c_str());
        return 1;
    }
    const int numChannels = (int)audio.samples.size();
    const int numSamples = numChannels ? (int)audio.samples[0].size() : 0;
    std::printf("channels %d, samples per channel %d, rate %d, bits %d\n", numChannels, numSamples,
                audio.sample_rate, audio.bit_depth);

    if (single_arg) {  // PhaseVocoder(int samples): hop N/2, timeScale 1, REF_COMPAT
        hopdiv = 2;
        scale = 1.0f;
        mode = PV_MODE_REF_COMPAT;
    }
    const int hop = N / hopdiv;
    const int frames = pv_frame_count(numSamples, hop);
    const int padN = numSamples + 2 * N;  // frames near the end read zeros (deviation 1)
    const int cap = frames + numSamples / std::max(1, (int)(scale * hop)) + 2;
    std::unique_ptr<PhaseVocoder> owner(
        single_arg ? new PhaseVocoder(N, numChannels > 0 ? numChannels : 1, cap)  // phaseVocoder.h:46
                   : new PhaseVocoder(N, effect, scale, hopdiv, mode, numChannels > 0 ? numChannels : 1, cap));
    PhaseVocoder& phase = *owner;
    const int outLen = (int)(phase.timeScale * numSamples);
    std::vector<std::vector<float>> outFile(2, std::vector<float>(outLen > 0 ? outLen : 0, 0.f));

    float* d_input = nullptr;  // [channel][padN], zero padded
    HIPCHECK(hipMalloc((void**)&d_input, sizeof(float) * (size_t)padN * std::max(numChannels, 1)));
    HIPCHECK(hipMemset(d_input, 0, sizeof(float) * (size_t)padN * std::max(numChannels, 1)));
    for (int c = 0; c < numChannels; ++c)
        HIPCHECK(hipMemcpy(d_input + (size_t)c * padN, audio.samples[c].data(),
                           sizeof(float) * numSamples, hipMemcpyHostToDevice));
    std::vector<float> emitted;

    if (rt) {
        // main.cpp:84-101 + RT block: buffers of bufferSize = nSamps frames of channel 0
        const unsigned int bufferSize = phase.nSamps;
        if (phase.rtOutputSamples() > (int)bufferSize) {
            std::fprintf(stderr, "err: --rt emits %d samples per %u-sample buffer (scale > 1); an RtAudio "
                         "output buffer holds %u\n", phase.rtOutputSamples(), bufferSize, bufferSize);
            return 1;
        }
        std::vector<float> inBuf(bufferSize), outBuf((size_t)std::max(phase.rtOutputSamples(), 1));
        std::printf("Real-time callbacks\n");
        int outIndex = 0;
        for (int i = 0; i + (int)bufferSize <= numSamples; i += bufferSize) {
            std::memcpy(inBuf.data(), audio.samples[0].data() + i, sizeof(float) * bufferSize);
            callback(outBuf.data(), inBuf.data(), bufferSize, (double)i / audio.sample_rate, 0, &phase);
            for (int j = 0; j < phase.rtOutputSamples(); ++j, ++outIndex) {
                if (outIndex < outLen) outFile[0][outIndex] = outFile[1][outIndex] = outBuf[j];
                emitted.push_back(outBuf[j]);
            }
        }
    } else if (batched) {
        const int S = phase.specStride();
        const long long olen = pv_output_length(phase.handle, frames);
        pv_float2* d_spec = nullptr;
        float* d_out = nullptr;
        HIPCHECK(hipMalloc((void**)&d_spec, sizeof(pv_float2) * (size_t)std::max(frames, 1) * S * numChannels));
        HIPCHECK(hipMalloc((void**)&d_out, sizeof(float) * (size_t)std::max(olen, 1LL) * numChannels));
        PhaseVocoder::checkCUDAErrori(pv_process(phase.handle, d_input, padN, numSamples, numChannels, frames,
                                                 d_spec, (long long)frames * S, d_out, olen, nullptr),
                                      "pv_process", __LINE__);
        HIPCHECK(hipDeviceSynchronize());
        std::vector<float> h((size_t)std::max(olen, 1LL));
        // main.cpp:264-297 writes channel 0's first floor(n/outHop)*outHop samples to L and R
        // (the `numChannels = 1` assignment ends its channel loop); every channel was
        // processed, as main.cpp analyses every channel
        const long long n_emit = std::min<long long>((long long)(numSamples / phase.outHopSize) * phase.outHopSize,
                                                     std::min<long long>(olen, outLen));
        HIPCHECK(hipMemcpy(h.data(), d_out, sizeof(float) * olen, hipMemcpyDeviceToHost));
        for (long long i = 0; i < n_emit; ++i) outFile[0][i] = outFile[1][i] = h[i];
        emitted.assign(h.begin(), h.begin() + n_emit);
        HIPCHECK(hipFree(d_spec));
        HIPCHECK(hipFree(d_out));
    } else {
        // main.cpp:204-219: one pre-zeroed 2N-bin spectrum per hop position
        const int S = phase.specStride();
        const int nspec = numSamples / hop + 1;
        float2* d_output = nullptr;
        HIPCHECK(hipMalloc((void**)&d_output, sizeof(float2) * (size_t)S * nspec * numChannels));
        HIPCHECK(hipMemset(d_output, 0, sizeof(float2) * (size_t)S * nspec * numChannels));
        std::printf("analysis...\n");
        for (int channel = 0; channel < numChannels; channel++)                  // main.cpp:228
            for (int i = 0; i < numSamples - hop; i += hop)                       // main.cpp:231
            {
                phase.analysis_CUFFT(d_input + (size_t)channel * padN + i,
                                     d_output + ((size_t)channel * nspec + i / hop) * S, nullptr, nullptr);
                ana_ms += CudaPhase::timer().getGpuElapsedTimeForPreviousOperation();  // main.cpp:240
            }
        float *backFrame = nullptr, *final_output = nullptr;
        HIPCHECK(hipMalloc((void**)&backFrame, sizeof(float) * N));
        HIPCHECK(hipMalloc((void**)&final_output, sizeof(float) * N));
        HIPCHECK(hipMemset(backFrame, 0, sizeof(float) * N));
        std::printf("resynthesis...\n");
        if (effect == TIME_SHIFT) {
            std::vector<float> h(N);
            const int channel = 0;  // main.cpp:288: `numChannels = 1` ends the channel loop
            int outIndex = 0;
            for (int i = 0; i < numSamples / phase.outHopSize; i++) {            // main.cpp:266
                const int si = i < nspec ? i : nspec - 1;
                phase.resynthesis_CUFFT(backFrame, d_output + ((size_t)channel * nspec + si) * S, final_output);
                syn_ms += CudaPhase::timer().getGpuElapsedTimeForPreviousOperation();  // main.cpp:277
                HIPCHECK(hipMemcpy(backFrame, final_output, sizeof(float) * N, hipMemcpyDeviceToDevice));
                HIPCHECK(hipMemcpy(h.data(), backFrame, sizeof(float) * N, hipMemcpyDeviceToHost));
                for (int j = 0; j < phase.outHopSize; j++) {
                    const int idx = outIndex + j;
                    if (idx >= 0 && idx < outLen) {
                        outFile[channel][idx] = h[j];
                        outFile[1][idx] = h[j];
                    }
                    emitted.push_back(h[j]);
                }
                outIndex += phase.outHopSize;
            }
        }
        HIPCHECK(hipFree(backFrame));
        HIPCHECK(hipFree(final_output));
        HIPCHECK(hipFree(d_output));
    }
    HIPCHECK(hipFree(d_input));
    if (show_timer && !batched)
        std::printf("CudaPhase::timer(): analysis %.3f ms total, resynthesis %.3f ms total\n", ana_ms, syn_ms);
    std::printf("writing to file\n");
    if (!pvwav::save16(out, outFile, 44100)) {
        std::printf("err: could not write %s\n", out.c_str());
        return 1;
    }
    if (!dump.empty()) {
        FILE* f = std::fopen(dump.c_str(), "wb");
        if (!f) return 1;
        std::fwrite(emitted.data(), sizeof(float), emitted.size(), f);
        std::fclose(f);
    }
    return 0;
}
