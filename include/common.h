// common.h — FFT::Common::PerformanceTimer of the reference (karnel/common.h:27-113): a
// CPU timer (std::chrono) and a GPU timer (events on the default stream), shared by the
// drop-in headers kernel.h (CudaPhase::timer) and hpfft.h (FFT::HPFFT::timer).
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>

namespace FFT {
namespace Common {
// karnel/common.h:27-113: cpu timer (chrono) + gpu timer (events)
class PerformanceTimer {
   public:
    PerformanceTimer() {
        (void)hipEventCreate(&start_);
        (void)hipEventCreate(&stop_);
    }
    ~PerformanceTimer() {
        (void)hipEventDestroy(start_);
        (void)hipEventDestroy(stop_);
    }
    void startCpuTimer() { cpu0_ = std::chrono::high_resolution_clock::now(); }
    void endCpuTimer() {
        auto t = std::chrono::high_resolution_clock::now();
        prev_cpu_ms_ = std::chrono::duration<float, std::milli>(t - cpu0_).count();
    }
    void startGpuTimer() { (void)hipEventRecord(start_); }
    void endGpuTimer() {
        (void)hipEventRecord(stop_);
        (void)hipEventSynchronize(stop_);
        (void)hipEventElapsedTime(&prev_gpu_ms_, start_, stop_);
    }
    float getCpuElapsedTimeForPreviousOperation() { return prev_cpu_ms_; }
    float getGpuElapsedTimeForPreviousOperation() { return prev_gpu_ms_; }

   private:
    hipEvent_t start_{}, stop_{};
    std::chrono::high_resolution_clock::time_point cpu0_{};
    float prev_cpu_ms_ = 0.f, prev_gpu_ms_ = 0.f;
};
}  // namespace Common
}  // namespace FFT
