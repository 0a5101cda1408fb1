// fft_bench.cpp — the reference's FFT micro-benchmark (milestone1_565.pdf slide 7, the
// src/50Hz/*.dat inputs) on the hpfft.h drop-in, plus the batched
// throughput of the same op.
//
//   fft_bench bench                    one JSON line per N: ms per single FFT (timer()
//                                      around computeGPUFFT, as the reference timed it) and
//                                      batched FFTs/s (pv_fft_c2c, 65536 transforms)
//   fft_bench check in.c64 N out.c64 [inverse]
//                                      computeGPUFFT/IFFT of N complex64 values from a file,
//                                      output taken from where the reference leaves it
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hpfft.h"

static int check_file(const char* in, int N, const char* out, bool inverse) {
    std::vector<float2> h(N);
    FILE* f = std::fopen(in, "rb");
    if (!f || std::fread(h.data(), sizeof(float2), N, f) != (size_t)N) {
        std::fprintf(stderr, "cannot read %d values from %s\n", N, in);
        return 2;
    }
    std::fclose(f);
    float2 *sig = nullptr, *inter = nullptr;
    (void)hipMalloc((void**)&sig, sizeof(float2) * N);
    (void)hipMalloc((void**)&inter, sizeof(float2) * N);
    (void)hipMemcpy(sig, h.data(), sizeof(float2) * N, hipMemcpyHostToDevice);
    if (inverse) FFT::HPFFT::computeGPUIFFT(N, 2, sig, inter);
    else FFT::HPFFT::computeGPUFFT(N, 2, sig, inter);
    (void)hipDeviceSynchronize();
    int l = 0;
    while ((1 << l) < N) ++l;
    (void)hipMemcpy(h.data(), (l % 2 == 0) ? sig : inter, sizeof(float2) * N, hipMemcpyDeviceToHost);
    f = std::fopen(out, "wb");
    std::fwrite(h.data(), sizeof(float2), N, f);
    std::fclose(f);
    (void)hipFree(sig);
    (void)hipFree(inter);
    return 0;
}

static int bench() {
    const int sizes[] = {2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048};
    const int batch = 65536;
    float2 *sig = nullptr, *inter = nullptr, *big = nullptr;
    (void)hipMalloc((void**)&sig, sizeof(float2) * 2048);
    (void)hipMalloc((void**)&inter, sizeof(float2) * 2048);
    (void)hipMalloc((void**)&big, sizeof(float2) * 2048 * (size_t)batch);
    std::vector<float2> h(2048);
    for (int i = 0; i < 2048; ++i) h[i] = make_float2(std::sin(2.0 * M_PI * 50.0 * i / 44100.0), 0.f);
    (void)hipMemcpy(sig, h.data(), sizeof(float2) * 2048, hipMemcpyHostToDevice);
    (void)hipMemset(big, 0, sizeof(float2) * 2048 * (size_t)batch);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int N : sizes) {
        for (int i = 0; i < 20; ++i) FFT::HPFFT::computeGPUFFT(N, 2, sig, inter);
        const int reps = 200;
        float acc = 0.f;
        for (int i = 0; i < reps; ++i) {  // the reference: timer around one computeGPUFFT
            FFT::HPFFT::timer().startGpuTimer();
            FFT::HPFFT::computeGPUFFT(N, 2, sig, inter);
            FFT::HPFFT::timer().endGpuTimer();
            acc += FFT::HPFFT::timer().getGpuElapsedTimeForPreviousOperation();
        }
        // the whole 1 GiB buffer at every N (2^27 points): no size fits the 256 MB MALL
        const int nb = (int)((size_t)batch * 2048 / N);
        for (int i = 0; i < 3; ++i) (void)pv_fft_c2c((pv_float2*)big, (pv_float2*)big, N, nb, 0, nullptr);
        (void)hipEventRecord(e0);
        const int breps = 20;
        for (int i = 0; i < breps; ++i) (void)pv_fft_c2c((pv_float2*)big, (pv_float2*)big, N, nb, 0, nullptr);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double per = ms / breps;
        const double bytes = 2.0 * 8.0 * N * (double)nb;  // read + write of the batch
        std::printf("{\"N\": %d, \"single_fft_ms\": %.6f, \"batch\": %d, \"batched_ms\": %.4f, "
                    "\"ffts_per_s\": %.4e, \"batched_GBps\": %.1f}\n",
                    N, acc / reps, nb, per, nb / (per * 1e-3), bytes / (per * 1e-3) / 1e9);
    }
    (void)hipFree(sig);
    (void)hipFree(inter);
    (void)hipFree(big);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && std::strcmp(argv[1], "bench") == 0) return bench();
    if (argc >= 5 && std::strcmp(argv[1], "check") == 0)
        return check_file(argv[2], std::atoi(argv[3]), argv[4], argc >= 6 && std::atoi(argv[5]) != 0);
    std::fprintf(stderr, "usage: fft_bench bench | fft_bench check in.c64 N out.c64 [inverse]\n");
    return 2;
}
