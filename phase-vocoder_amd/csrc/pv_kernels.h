// pv_kernels.h — kernel parameter blocks and launchers (host <-> device interface of libpv).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

// Diagnostic builds.  The timing-only ablation switches (PV_ABL_*) give WRONG outputs and
// PV_FUSED_STAMPS writes per-wave clock stamps; a build that defines one must say so with
// PV_DIAGNOSTIC_BUILD, and the library then reports it (pv_diagnostic_build() = 1): bench.py
// refuses to check or report such a build as the product, and the GPU tests refuse it.
#if (defined(PV_ABL_NOSTORE) || defined(PV_ABL_NOATAN) || defined(PV_ABL_NOFFT) || defined(PV_ABL_NOWIN) ||   \
     defined(PV_ABL_L2IN) || defined(PV_ABL_L2ROWS) || defined(PV_ABL_NOSINCOS) || defined(PV_ABL_NOGATHER) || \
     defined(PV_FUSED_STAMPS)) &&                                                                            \
    !defined(PV_DIAGNOSTIC_BUILD)
#error "diagnostic / timing-only switch without PV_DIAGNOSTIC_BUILD (its outputs are wrong or instrumented)"
#endif

namespace pv {

// STANDARD run record per (channel, run): kRecFields rows of bins_pad int32 words —
// S = sum of the unwrap decisions of the run's frames after its first, then phi of the run's
// first and of its last frame (float bits).  k_carry makes the first frame's decision from
// phi(t0) and the previous run's last phase.
constexpr int kRecFields = 3;

struct AnaParams {
    const float* x;
    long long ldx, n;
    int hop, frames, F, nruns;
    int aligned;            // x base, ldx and hop allow 8-byte vector loads
    const float* win;       // analysis window (N)
    const float2* tw;       // stage-major twiddles of the L-point FFT (L entries)
    const float2* tws;      // real-split twiddles e^{-2 pi i k / (2L)}, k <= L
    const float* ek;        // expected advance (STANDARD), bins
    int ek_lane;            // 64 % hop_div == 0: e_k = ek[k mod 64] (per-lane constant)
    float2* spec;
    long long ld_spec;
    int spec_stride;
    int* runsum;            // [C][nruns][kRecFields][bins_pad] run records or nullptr
    int bins_pad;
    int nan_faithful;       // REF_COMPAT: x=y=0 -> NaN phase (kernel.cu:108)
    int packed;             // STANDARD rows in the PV_SPEC_PACKED layout (bin L in slot 0)
    int src_hi;             // STANDARD, L >= 1024: bins above it are not analysed (their row
                            // slots are not written; the synthesis does not read them:
                            // k_synthesis NR) — pv_process without a spectrum output; L
                            // otherwise
};

struct ScanParams {
    const float2* spec;
    long long ld_spec;
    int spec_stride, frames, F, nruns, L, bins_pad;
    int packed;                        // PV_SPEC_PACKED rows
    const float* ek;
    int* runsum;
    int* carry;
    // a segment of a longer stream (pv_segment_resynthesis), or nullptr: the unwrap count
    // before the segment's first frame and the phase of the frame before it, [C][bins_pad]
    const int* carry_in;
    const float* phi_in;
};

// per-segment summaries of a stream split into consecutive frame segments
// (pv_segment_summary / pv_segment_resynthesis): [seg][C][kSegFields][bins_pad] int32 —
// the segment's unwrap decisions after its first frame, phi of its first and of its last frame
constexpr int kSegFields = 3;
struct SegParams {
    const int* runsum;                 // the segment's run records (k_runsum)
    int nruns, L, bins_pad, channels;
    const float* ek;
    int* summary;                      // k_segsum: this segment's [C][kSegFields][bins_pad]
    const int* summaries;              // k_segcarry: the earlier segments' summaries
    int seg;                           // k_segcarry: how many segments come before this one
    int* carry_in;                     // k_segcarry outputs, [C][bins_pad]
    float* phi_in;
};

struct SynParams {
    const float2* spec;
    long long ld_spec;
    int spec_stride, frames, F, nruns, bins_pad;
    const int* carry;
    const float* ek;
    const unsigned* jk_mod;            // (p * j_k) mod q
    const int* src_first;              // pitch map
    const int* src_cnt;
    int pitch;
    float rho;
    unsigned long long p_mod, q;
    int q_pow2;
    float inv_q;
    const float2* tw;                  // stage-major twiddles, L-point
    const float2* tws;                 // e^{-2 pi i k/N}, k <= L
    const float* gain;                 // synthesis window * norm / N   (N)
    int rot;                           // 0 (STANDARD) or N/2 (REF_COMPAT swap halves)
    int hs;                            // out hop
    float* out;
    long long ldo, out_len;
    int out_aligned;                   // out base and ldo allow 8-byte vector stores
    float* tails;                      // [C][nwg][tail_len], nwg = ceil(nruns/4)
    int tail_len;
    int k_lane;                        // e_k, (p j_k) mod q depend on k mod 64 only (syn_run LANEK)
    int packed;                        // PV_SPEC_PACKED rows (bins 0 and L in slot 0)
    int src_hi;                        // highest analysis bin an output bin reads (single-
                                       // source pitch: the row slots above it are not read)
    unsigned t_off;                    // (index of the first frame in the whole stream) mod q:
                                       // 0 unless a segment of a longer stream
};

// single-launch STANDARD path for q = 1 (pv_fused.hip)
struct FusedParams {
    const float* x;
    long long ldx, n;
    int hop, frames, F, nruns;
    int aligned;                       // x base, ldx and hop allow 8-byte vector loads
    const float* win;                  // analysis window (N)
    const float2* tw;                  // stage-major twiddles, L-point (analysis = synthesis)
    const float2* tws;                 // e^{-2 pi i k/N}, k <= L
    const int* src_first;              // pitch map
    const int* src_cnt;
    float rho;
    const float* gain;                 // synthesis window * norm / N   (N)
    const float2* tw_half;             // stage-major L/2-point table (pitch 2: MODE 4) or nullptr
    int hs;                            // out hop
    float2* spec;
    long long ld_spec;
    int spec_stride;
    float* out;
    long long ldo, out_len;
    int out_aligned;
    float* tails;                      // [C][nwg][tail_len], nwg = ceil(nruns/4)
    int tail_len;
    int* seam_flags;                   // [C][nwg] arrival counters, 0 between launches
    int packed;                        // PV_SPEC_PACKED rows
    int src_hi;                        // highest analysis bin an output bin reads (pitch > 1:
                                       // about L / pitch): with spec == nullptr the bins above
                                       // it are not analysed (nothing reads their phase)
    int nwg;                           // workgroups per channel (grid.x)
    int n4;                            // > 0: balanced runs — n4 of them have F + 1 frames
                                       // (k_fused: which ones, so that no SIMD holds more than
                                       // two of them); 0: every run F frames
#ifdef PV_FUSED_STAMPS
    unsigned long long* stamps;        // diagnostic build only: kFusedStampSlots per wave
#endif
};
#ifdef PV_FUSED_STAMPS
constexpr int kFusedStampSlots = 16;  // rt start, mt start, setup, frame 0..F-1, loop, end rt/mt, hw id
#endif

struct SeamParams {
    float* out;
    long long ldo, out_len;
    const float* tails;
    const float* ola_in;
    long long ld_ola;
    int nruns, nwg, F, hs, tail_len;
};

// real-time mode (pv_rt.hip): one launch per callback, a wave per channel
struct RtParams {
    const float* in;                   // [C][nframes * hop] new samples (row stride ldi)
    long long ldi;
    float* out;                        // [C][nframes * hs] emitted samples (row stride ldo)
    long long ldo;
    float2* spec;                      // optional [C][nframes][spec_stride] {mag, phase}
    long long ld_spec;
    int spec_stride;
    int channels, nframes, hop, hs, bins_pad;
    float* hist;                       // [C][N] stream state (see pv_rt.hip)
    float* ola;                        // [C][N]
    float* phprev;                     // [C][bins_pad]
    int* M;                            // [C][bins_pad]
    unsigned* tcount;                  // [C]
    const float* win;
    const float* gain;
    const float2* tw;
    const float2* tws;
    const float* ek;
    const unsigned* jk_mod;
    const int* src_first;
    const int* src_cnt;
    float rho;
    unsigned long long p_mod, q;
    int q_pow2;
    float inv_q;
};

// harmoniser mix: dst[c][i] = sum_k gain[k] * src[k][c][i]
struct MixParams {
    const float* src;
    long long ldo, ld_voice;
    int voices;
    float gain[64];
    float* dst;
    long long ld_mix, len;
    int channels;
};

hipError_t launch_std_analysis(int L, int channels, const AnaParams& p, hipStream_t s);
int std_analysis_wgs_per_cu(int L, int hop, bool ek_lane, bool packed, int* waves_per_wg);
hipError_t launch_compat_analysis(int L, int channels, const AnaParams& p, hipStream_t s);
hipError_t launch_runsum(int channels, const ScanParams& p, hipStream_t s);
hipError_t launch_carry(int channels, const ScanParams& p, hipStream_t s);
hipError_t launch_segsum(const SegParams& p, hipStream_t s);
hipError_t launch_segcarry(const SegParams& p, hipStream_t s);
hipError_t launch_synthesis(int L, int mode, int channels, const SynParams& p, hipStream_t s);
// the synthesis kernel for this geometry can take SynParams.k_lane (register overlap-add,
// power-of-two q, STANDARD)
bool synthesis_lane_kernel(int L, int mode, int hs, bool q_pow2, unsigned long long q);
hipError_t launch_seam(int channels, const SeamParams& p, hipStream_t s);
bool fused_supported(int L, int hs);
hipError_t launch_fused(int L, int mode, int channels, const FusedParams& p, hipStream_t s);
size_t synthesis_lds_bytes(int L, int hs);
hipError_t launch_fft(int n, int inverse, const float2* in, float2* out, const float2* tw, int batch,
                      hipStream_t s);
hipError_t launch_mix(const MixParams& p, hipStream_t s);
hipError_t launch_rt(int L, int mode, const RtParams& p, hipStream_t s);
size_t rt_lds_bytes(int L);
hipError_t launch_window_gain(const float* win, float* dwin, float* gain, int n, hipStream_t s);
hipError_t launch_overlap_test(const float* in, const float* win, const float* back, float* out,
                               int n, int hop, hipStream_t s);

}  // namespace pv
