// kernel_h_check — drives the drop-in `CudaPhase::pv_analysis_RT` (include/kernel.h, the
// reference's karnel/kernel.h:16 / kernel.cu:219-260) the way an RtAudio client would: one
// frame on the caller's HIP stream.  Used by tests/test_gpu_dropin.py.
//
//   kernel_h_check <N> <frame.f32> <out.f32>
//
// Reads N float32 samples, writes the 2N {mag, phase} float2 of pv_analysis_RT to out.f32 and
// prints one JSON line:
//   pending_while_stream_busy  the call was enqueued behind a ~0.3 s busy kernel on the given
//                              non-blocking stream: right after it returns, the output (read on
//                              another stream) still holds its sentinel fill
//   overloads_equal            the declared 6-argument overload (kernel.h:16) gives the same bits
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernel.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "HIP %s at line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// bounded busy wait (s_memrealtime runs at 100 MHz): holds the stream for `ticks`
__global__ void k_busy(unsigned long long ticks, int* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    int n = 0;
    while (t - t0 < ticks) {
        t = __builtin_amdgcn_s_memrealtime();
        ++n;
    }
    if (threadIdx.x == 0 && n == -1) *sink = n;
}

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: kernel_h_check <N> <frame.f32> <out.f32>\n");
        return 2;
    }
    const int N = std::atoi(argv[1]);
    std::vector<float> frame(N);
    FILE* f = std::fopen(argv[2], "rb");
    if (!f || std::fread(frame.data(), sizeof(float), N, f) != (size_t)N) {
        std::fprintf(stderr, "cannot read %d samples from %s\n", N, argv[2]);
        return 2;
    }
    std::fclose(f);
    float *d_in, *d_interm, *d_win;
    float2 *d_out, *d_fft;
    int* d_sink;
    CK(hipMalloc(&d_in, sizeof(float) * N));
    CK(hipMalloc(&d_interm, sizeof(float) * N));
    CK(hipMalloc(&d_win, sizeof(float) * N));
    CK(hipMalloc(&d_out, sizeof(float2) * 2 * N));
    CK(hipMalloc(&d_fft, sizeof(float2) * 2 * N));
    CK(hipMalloc(&d_sink, sizeof(int)));
    CK(hipMemcpy(d_in, frame.data(), sizeof(float) * N, hipMemcpyHostToDevice));
    hipStream_t s, side;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));

    // first call builds the cached handle (allocations, table uploads)
    CudaPhase::pv_analysis_RT(d_out, d_fft, d_in, d_interm, d_win, N, &s);
    CK(hipStreamSynchronize(s));

    std::vector<float2> sentinel(2 * N), early(2 * N), got(2 * N), got6(2 * N);
    for (auto& v : sentinel) v = make_float2(-12345.0f, -54321.0f);
    CK(hipMemcpy(d_out, sentinel.data(), sizeof(float2) * 2 * N, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s, 30000000ull, d_sink);  // ~0.3 s
    CudaPhase::pv_analysis_RT(d_out, d_fft, d_in, d_interm, d_win, N, &s);
    CK(hipMemcpyAsync(early.data(), d_out, sizeof(float2) * 2 * N, hipMemcpyDeviceToHost, side));
    CK(hipStreamSynchronize(side));
    bool pending = std::memcmp(early.data(), sentinel.data(), sizeof(float2) * 2 * N) == 0;
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), d_out, sizeof(float2) * 2 * N, hipMemcpyDeviceToHost));

    CK(hipMemcpy(d_out, sentinel.data(), sizeof(float2) * 2 * N, hipMemcpyHostToDevice));
    CudaPhase::pv_analysis_RT(d_out, d_fft, d_in, d_interm, N, &s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got6.data(), d_out, sizeof(float2) * 2 * N, hipMemcpyDeviceToHost));
    const bool same = std::memcmp(got.data(), got6.data(), sizeof(float2) * 2 * N) == 0;

    FILE* o = std::fopen(argv[3], "wb");
    if (!o || std::fwrite(got.data(), sizeof(float2), 2 * N, o) != (size_t)(2 * N)) return 2;
    std::fclose(o);
    std::printf("{\"pending_while_stream_busy\": %s, \"overloads_equal\": %s}\n", pending ? "true" : "false",
                same ? "true" : "false");
    return 0;
}
