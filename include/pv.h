/*
 * pv.h — C-ABI of the MI355X phase-vocoder hot path (libpv.so).
 *
 * Plain pointers and sizes only; every float / pv_float2 pointer handed to a compute
 * entry point is a DEVICE pointer (hipMalloc / torch CUDA tensor) on the handle's device,
 * and `stream` is a hipStream_t (NULL = the legacy default stream).  All calls are
 * asynchronous with respect to the host (graph-capturable: no allocation, no sync) — the
 * one exception is pv_process(spec = NULL) on the split path, whose first call allocates
 * the handle's own rows unless pv_reserve_spectrum did (under capture it refuses instead).
 *
 * Which reference interface each entry point replaces (reference @ /root/reference):
 *   pv_create        PhaseVocoder(int samples, Effect e, float scale, int hop)
 *                      src/phaseVocoder.h:79-116  (window imp[], hop = samples/hop,
 *                      outHopSize = scale*hop, cuFFT plans, streams)
 *   pv_destroy       ~PhaseVocoder()  src/phaseVocoder.h:128-130; cufftDestroy main.cpp:396
 *   pv_analysis      PhaseVocoder::analysis_CUFFT  src/phaseVocoder.cpp:25-33
 *                      -> CudaPhase::pv_analysis_CUFFT  karnel/kernel.cu:299-348
 *                      batched over channels x frames (main.cpp:228-250 loop)
 *   pv_resynthesis   PhaseVocoder::resynthesis_CUFFT  src/phaseVocoder.cpp:60-76
 *                      -> CudaPhase::resynthesis_CUFFT  karnel/kernel.cu:352-432
 *                      batched, including the running overlap-add main.cpp:261-297
 *   pv_process       analysis -> processing -> resynthesis fused pipeline (the offline
 *                      loop of main.cpp:228-297 in one call); no reference counterpart
 *   pv_frame_*       the hop/frame arithmetic of main.cpp:231 and main.cpp:266
 *   pv_rt_*          the real-time design: RtAudio `callback` (main.cpp:45-59) copying each
 *                      buffer into PhaseVocoder::curr_input and calling the per-callback
 *                      PhaseVocoder::analysis() over prev_input / prev_mag_phase /
 *                      prev_output (phaseVocoder.h:16-31; pv_analysis_RT kernel.cu:219-250;
 *                      README.md:46-50); one hipGraph replay per callback
 *   pv_segment_*     one long stream split into consecutive frame segments, e.g. one per
 *                      GPU (the optional time shard); no reference
 *                      counterpart (the reference processes one stream frame by frame)
 *   pv_harmon*       the harmoniser the README plans ("multiple pitch shifts on a single
 *                      input", README.md:50): one analysis, K pitch-shift resyntheses
 *   pv_fft_c2c       FFT::HPFFT::computeGPUFFT / computeGPUIFFT (karnel/hpfft.h:6-11,
 *                      hpfft.cu:145-203): radix-2 Stockham FFT, batched in one launch
 *
 * Errors: status codes instead of the reference's print-and-exit (io.cpp:115-124).  The
 * header-only C++ drop-in (include/phaseVocoder.h) restores print-and-exit on top.
 *
 * Environment overrides (read by pv_create / pv_rt_capture; the tests use them to reach
 * every kernel geometry; none changes a result beyond run-boundary roundings):
 *   PV_RUN_FRAMES=F      frames per wave run of the split path (even, 8..256)
 *   PV_SYN_LANEK=0       per-bin unwrap constants from LDS instead of per-lane registers
 *   PV_FUSED=0           the split path even where the q = 1 single launch applies
 *   PV_FUSED_FRAMES=F    frames per run of the q = 1 single launch
 *   PV_FUSED_HALF=0      pitch 2 single launch: the MODE 3 gather and full-size inverse FFT
 *                        instead of the half-size resynthesis of X^2/|X| (MODE 4)
 *   PV_FUSED_BALANCE=0   single launch of one channel: uniform runs (no balanced F+1 runs)
 *   PV_COMPAT_ANA_FRAMES=F  REF_COMPAT analysis run length (1..256, default 4)
 *   PV_RT_LAUNCH=direct  pv_rt_callback launches the kernel instead of replaying the graph
 *
 * Concurrency: a handle's compute calls share its workspace (run records, carries, seam
 * tails, segment state), so the calls on one handle must be ordered — one stream, or
 * streams synchronised between calls; different handles are independent.  pv_last_error
 * is per thread; pv_reserve_spectrum is thread-safe.
 */
#ifndef PV_H
#define PV_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PV_ABI_VERSION 5  /* 2: pv_config.window / nan_faithful, pv_set_window;
                             3: pv_info.single_launch / single_launch_frames / lane_constants;
                             4: leading abi_version in pv_config / pv_info (checked: a caller
                                built against another header gets PV_ERR_ARG, not a
                                misread struct), pv_config.spec_layout, the chained path
                                and pv_check_device removed;
                             5: pv_config.tables_external, pv_process(spec = NULL) on the
                                single launch (later additions are functions only, no
                                struct change: pv_sources_sha, pv_reserve_spectrum,
                                pv_segment_*) */

typedef struct pv_handle pv_handle;

/* layout-compatible with HIP/CUDA float2 {x, y} (8 bytes, 8-byte aligned) */
typedef struct pv_float2 {
    float x, y;
} pv_float2;

typedef enum pv_status {
    PV_OK = 0,
    PV_ERR_ARG = 1,         /* invalid argument / size out of the handle's capacity */
    PV_ERR_UNSUPPORTED = 2, /* configuration not supported (e.g. N not a power of 2) */
    PV_ERR_HIP = 3,         /* HIP runtime error (pv_last_error() has the text)       */
    PV_ERR_NOMEM = 4        /* device allocation failed                               */
} pv_status;

typedef enum pv_effect {
    PV_TIME_SHIFT = 't',  /* phaseVocoder.h:6  */
    PV_PITCH_SHIFT = 'p'  /* phaseVocoder.h:7  */
} pv_effect;

typedef enum pv_mode {
    PV_MODE_REF_COMPAT = 0, /* the reference's active path, bugs included */
    PV_MODE_STANDARD = 1    /* textbook phase vocoder (Hann, unwrap, true frequency)     */
} pv_mode;

/* STANDARD spectrum row layout (pv_config.spec_layout) */
typedef enum pv_spec_layout {
    PV_SPEC_NATURAL = 0, /* {mag, phase} of bins k = 0 .. N/2 (spec_bins = N/2+1), rows padded
                            to spec_stride = N/2 + 8                                          */
    PV_SPEC_PACKED = 1   /* rows of exactly N/2 float2 (spec_stride = spec_bins = N/2): bins
                            1 .. N/2-1 as {mag, phase}; bin 0 and bin N/2, both real, share
                            slot 0 as {s0, sN/2} with s = +mag for phase 0, -mag for phase pi
                            (the sign bit carries the phase; pv_unpack_bins below).  Every
                            row store is whole 64-byte segments (no 8-byte partial write for
                            bin N/2).  STANDARD handles only; the real-time mode rejects it */
} pv_spec_layout;

typedef enum pv_window {
    PV_WINDOW_DEFAULT = 0,     /* the mode's window: REF_COMPAT the symmetric Hamming of the
                                  4-argument constructor, STANDARD the periodic Hann        */
    PV_WINDOW_HAMMING_REF = 1, /* 0.54f - 0.46f*cosf(w*i), w = (float)(2pi/(N-1))
                                  (src/phaseVocoder.h:85-89; REF_COMPAT)                    */
    PV_WINDOW_HANN_REF = 2     /* 0.5f*(1.f - cosf((float)(2pi*i/N))) of the 1-argument
                                  constructor (src/phaseVocoder.h:64-66; REF_COMPAT)        */
} pv_window;

typedef struct pv_config {
    int abi_version;  /* = PV_ABI_VERSION (pv_create rejects any other value)          */
    int n_samps;      /* N, window length: power of 2 in [256, 2048] (both modes)       */
    int hop_div;      /* hop = N / hop_div (phaseVocoder.h:79 4th argument is a divisor)  */
    int effect;       /* pv_effect                                                      */
    float scale;      /* TIME_SHIFT: out_hop = (int)(scale*hop); PITCH_SHIFT: pitch ratio */
    int mode;         /* pv_mode                                                        */
    int max_channels; /* workspace capacity                                             */
    int max_frames;   /* workspace capacity, frames per channel                          */
    int device;       /* HIP device ordinal                                             */
    int window;       /* pv_window (0 = the mode's default); STANDARD accepts only 0      */
    int nan_faithful; /* REF_COMPAT: a bin with Re = Im = 0 gets phase atanf(0/0) = NaN as
                         in the reference (kernel.cu:101-109), which poisons that frame's
                         resynthesis; 0 (default) gives phase 0 (SURVEY.md §8c deviation 4) */
    int spec_layout;  /* pv_spec_layout (STANDARD only; REF_COMPAT accepts 0)              */
    int tables_external; /* 1: the handle's constant tables (windows, gains, twiddles, unwrap
                            and pitch maps) are not built here — the device tables start
                            zeroed and every compute call returns PV_ERR_ARG until
                            pv_import_tables loads a blob (a non-root rank of a multi-GPU
                            job receives rank 0's over RCCL, pvamd.dist.broadcast_tables);
                            0 (default): built by pv_create.  Batch handles only (pv_rt /
                            harmoniser reject it) */
} pv_config;

typedef struct pv_info {
    int abi_version;    /* the caller sets PV_ABI_VERSION (pv_get_info checks it)           */
    int n_samps, hop, out_hop;
    int spec_bins;      /* slots written per frame: N/2+1 (STANDARD natural), N/2 (STANDARD
                           packed) or 2N (REF_COMPAT)                                     */
    int spec_stride;    /* pv_float2 elements between consecutive frames of a channel   */
    int frames_per_run; /* frames per wave run; chosen from           */
                        /* max_channels x max_frames, or the environment variable       */
                        /* PV_RUN_FRAMES (even, 8..256) read by pv_create               */
    int mode, effect;
    float scale;
    int single_launch;        /* what pv_process launches: 0 the split path (analysis, scan,
                                 synthesis, seams), 1 one q = 1 launch (pv_fused.hip)      */
    int single_launch_frames; /* frames per run of that launch (0 for the split path)     */
    int lane_constants;       /* 1: the split synthesis keeps the per-bin unwrap constants
                                 in registers (e_k and (p j_k) mod q repeat every 64 bins:
                                 64 a multiple of N / hop and q of 64 hop / N, e.g. config
                                 3 and 4); PV_SYN_LANEK=0 read by pv_create turns it off  */
    int spec_layout;          /* pv_spec_layout of the handle's spectrum rows               */
} pv_info;

/* A PV_SPEC_PACKED row's slot 0 -> {mag, phase} of bin 0 and bin N/2.  Exact: the packed
 * phases are +0 or the float nearest pi (0x1.921fb6p+1f) and the magnitude is the sign-free
 * slot value. */
static inline void pv_unpack_bins(pv_float2 slot0, pv_float2* bin0, pv_float2* bin_half) {
    const float pi = 0x1.921fb6p+1f;
    union { float f; unsigned u; } a, b;
    a.f = slot0.x;
    b.f = slot0.y;
    const unsigned sa = a.u >> 31, sb = b.u >> 31;
    a.u &= 0x7fffffffu;
    b.u &= 0x7fffffffu;
    bin0->x = a.f;
    bin0->y = sa ? pi : 0.0f;
    bin_half->x = b.f;
    bin_half->y = sb ? pi : 0.0f;
}

int pv_abi_version(void);
/* version of the fp32 PV_STANDARD analysis contract (the exact operation sequence of the
 * phases and unwrap decisions) this build computes; the CPU oracle states the
 * version it restates (oracle/pvref.h PVR_CONTRACT_VERSION) and the two must agree */
int pv_contract_version(void);
/* 1 for a diagnostic build (timing-only ablations or instrumentation compiled in with
 * PV_DIAGNOSTIC_BUILD: outputs are not the product's), 0 for the product */
int pv_diagnostic_build(void);
/* sha256[:16] of the sources this library was built from (phase-vocoder_amd/csrc: every
 * *.hip *.hpp *.h *.cpp and the Makefile in byte order, then include/pv.h), compiled in by the
 * Makefile: the Python binding refuses a library whose hash is not its tree's */
const char* pv_sources_sha(void);
const char* pv_status_string(pv_status s);
const char* pv_last_error(void); /* thread-local text of the last failure */

pv_status pv_create(const pv_config* cfg, pv_handle** out);
void pv_destroy(pv_handle* h);
pv_status pv_get_info(const pv_handle* h, pv_info* info);

/* main.cpp:231 — analysis frames of an n-sample channel: ceil((n - hop)/hop), >= 0 */
int pv_frame_count(long long n_samples, int hop);
/* samples of the full overlap-add of `frames` frames: frames*out_hop + N - out_hop */
long long pv_output_length(const pv_handle* h, int frames);

/* Analysis of `frames` frames per channel.  Frame t of channel c reads
 * x[c*ldx + t*hop + i], i < N; samples at index >= n_samples read as 0.
 * spec[c*ld_spec + t*spec_stride + k] = {magnitude, phase}, k < spec_bins. */
pv_status pv_analysis(pv_handle* h, const float* x, long long ldx, long long n_samples,
                      int channels, int frames, pv_float2* spec, long long ld_spec, void* stream);

/* Processing + resynthesis of `frames` analysed frames per channel (spec is read only).
 * out[c*ldo + i], i < pv_output_length(h, frames): the full overlap-add.  ola_in
 * (nullable) holds N - out_hop samples per channel (stride ld_ola) already accumulated
 * at the start of this block (the reference's backFrame tail). */
pv_status pv_resynthesis(pv_handle* h, const pv_float2* spec, long long ld_spec, int channels,
                         int frames, const float* ola_in, long long ld_ola, float* out,
                         long long ldo, void* stream);

/* One long stream as consecutive non-empty frame segments s = 0, 1, ... (frames [f_s,
 * f_s + n_s) of every channel, e.g. one segment per GPU): segment s is analysed alone
 * (pv_analysis of x + f_s * hop), summarised (pv_segment_summary: per bin, its unwrap
 * decisions after its first frame and its first and last phase — pv_segment_summary_words(h)
 * int32 per channel, device memory [channels][words]), and after the summaries of segments
 * 0 .. s - 1 are known (gathered, in order, as [s][channels][words]), resynthesised by
 * pv_segment_resynthesis with frame0 = f_s: the unwrap counts and output phases are then those
 * of the whole stream bit for bit (integer sums; the boundary decisions are made on the GPU
 * with the contract's operations).  out holds the segment's own overlap-add,
 * pv_output_length(h, n_s) samples per channel starting at stream position f_s * out_hop;
 * its first N - out_hop samples overlap the previous segment's last ones (the caller adds
 * them).  STANDARD handles (REF_COMPAT has no unwrap state: pv_segment_resynthesis is then
 * pv_resynthesis).  pv_segment_summary of an empty segment is PV_ERR_ARG. */
int pv_segment_summary_words(const pv_handle* h);
pv_status pv_segment_summary(pv_handle* h, const pv_float2* spec, long long ld_spec, int channels,
                             int frames, int* summary, void* stream);
pv_status pv_segment_resynthesis(pv_handle* h, const pv_float2* spec, long long ld_spec, int channels,
                                 int frames, long long frame0, const int* summaries, int seg, float* out,
                                 long long ldo, void* stream);

/* analysis + processing + resynthesis (spec is the caller-owned spectrum buffer).  spec may
 * be NULL when the caller does not want the spectrum: on the single launch (pv_info.
 * single_launch = 1) it is then computed and consumed on chip and not written (SURVEY §8(d)
 * fused mode); on the split path it goes through the handle's own buffer (max_channels x
 * max_frames rows, zeroed, allocated by pv_reserve_spectrum or by the first such call:
 * PV_ERR_NOMEM if that fails; a first call made while `stream` is being captured returns
 * PV_ERR_ARG, since an allocation cannot be captured).  Either way, for pitch > 1 the bins
 * no output bin reads (above about L / scale) may be left unanalysed and are not read; the
 * output is the same bits as with a spectrum buffer. */
/* allocate (once, zeroed) the handle's own spectrum rows that pv_process(spec = NULL) uses
 * on the split path, so that such calls can then be captured into a graph; thread-safe; a
 * no-op for a single-launch handle.  Not capturable itself (it allocates). */
pv_status pv_reserve_spectrum(pv_handle* h);

pv_status pv_process(pv_handle* h, const float* x, long long ldx, long long n_samples,
                     int channels, int frames, pv_float2* spec, long long ld_spec, float* out,
                     long long ldo, void* stream);

/* ---------------------------------------------------------------- real-time mode
 * A pv_rt streams `channels` mono channels through the STANDARD pipeline one callback at a
 * time.  State (input history, previous phases, unwrap counts, overlap accumulator) lives
 * on the device between calls.  A push of `nframes` frames consumes nframes*hop new
 * samples per channel and emits nframes*out_hop final samples per channel; the emitted
 * stream equals pv_process() of the same stream prefixed with N - hop zeros.
 * Supported: PV_MODE_STANDARD, n_samps in [256, 2048]. */
typedef struct pv_rt pv_rt;

pv_status pv_rt_create(const pv_config* cfg, int channels, pv_rt** out);
void pv_rt_destroy(pv_rt* rt);
/* zero the stream state (start of a new stream) */
pv_status pv_rt_reset(pv_rt* rt, void* stream);
/* device pointers: in[c*ldi + i], i < nframes*hop; out[c*ldo + i], i < nframes*out_hop;
 * spec (nullable) receives the analysed {mag, phase} rows: spec[c*ld_spec + f*spec_stride + k] */
pv_status pv_rt_push(pv_rt* rt, const float* in, long long ldi, int nframes, float* out,
                     long long ldo, pv_float2* spec, long long ld_spec, void* stream);
/* Capture one callback of `nframes` frames into a hipGraph: pinned host input -> device,
 * pv_rt_push, device -> pinned host output.  The pinned buffers are planar
 * [channels][nframes*hop] and [channels][nframes*out_hop] (pv_rt_host_buffers). */
pv_status pv_rt_capture(pv_rt* rt, int nframes);
pv_status pv_rt_host_buffers(pv_rt* rt, float** host_in, float** host_out);
/* One synchronous callback on the captured graph: copies `in` (host, planar, may be the
 * pinned buffer itself) into the pinned input, replays the graph, waits, copies the
 * result to `out` (host, may be the pinned output itself). */
pv_status pv_rt_callback(pv_rt* rt, const float* in, float* out);

/* ---------------------------------------------------------------- harmoniser
 * K voices, voice k = PITCH_SHIFT by ratios[k] of the same input, all from ONE analysis
 * and one unwrap scan (cfg: STANDARD; effect and scale are ignored).  voices_out[k*ld_voice
 * + c*ldo + i], i < pv_output_length (every voice has out_hop = hop); each voice equals
 * pv_process() with its ratio.  mix (nullable): mix[c*ld_mix + i] = sum_k gains[k] * voice
 * k (gains: host array of K floats).  spec (required) receives the shared analysis, as
 * pv_process's.  At most 64 voices.  channels or frames 0: nothing is done (PV_OK). */
typedef struct pv_harmonizer pv_harmonizer;
pv_status pv_harmonizer_create(const pv_config* cfg, const float* ratios, int voices, pv_harmonizer** out);
void pv_harmonizer_destroy(pv_harmonizer* hz);
pv_status pv_harmonize(pv_harmonizer* hz, const float* x, long long ldx, long long n_samples,
                       int channels, int frames, pv_float2* spec, long long ld_spec, float* voices_out,
                       long long ldo, long long ld_voice, const float* gains, float* mix,
                       long long ld_mix, void* stream);

/* ---------------------------------------------------------------- standalone FFT
 * Batched unnormalised complex FFT (both directions, like the reference's GPU_FFT):
 * out[b*n + k] = sum_j in[b*n + j] * exp(-+2 pi i jk/n), b < batch, n a power of two in
 * [2, 2048]; in == out (in place) is allowed.  inverse != 0 uses exp(+...).  Device
 * pointers on the current HIP device; the first call per (device, n) builds that size's
 * twiddle table (allocation: not capturable), later calls are. */
pv_status pv_fft_c2c(const pv_float2* in, pv_float2* out, int n, int batch, int inverse, void* stream);

/* REF_COMPAT: replace the handle's window by the caller's (device pointer, n_samps
 * floats; copied on `stream`, the pointer is not kept).  The reference passes the window
 * to every call (CudaPhase::pv_analysis_CUFFT / resynthesis_CUFFT `win`, kernel.cu:301
 * and :406): it multiplies the analysis frame and the resynthesised frame.  Here the
 * analysis window becomes `win` and the synthesis gain win[k]/N (cudaDivVec kernel.cu:380
 * then cudaWindow :406).  STANDARD handles: PV_ERR_UNSUPPORTED (their synthesis
 * normalisation is derived from the Hann window at pv_create). */
pv_status pv_set_window(pv_handle* h, const float* win, void* stream);

/* Constant tables of a handle (windows, gains, twiddles, unwrap tables, pitch map) as one
 * device blob, so that one rank can build them and the others receive them over RCCL
 * (DESIGN.md §6).  export with dst == NULL only reports *bytes.  import validates the
 * blob's header against the handle's configuration and replaces the tables. */
pv_status pv_export_tables(const pv_handle* h, void* dst, size_t cap, size_t* bytes, void* stream);
pv_status pv_import_tables(pv_handle* h, const void* src, size_t bytes, void* stream);

/* kernel.cu:289-298 (OVERLAPTEST, main.cpp:156-202): identity processing of one frame,
 * out[k] = win[k]^2 * in[k] + (k + hop < N ? back[k + hop] : 0).  Device pointers. */
pv_status pv_test_overlap_add(const float* in, const float* win, const float* back, float* out,
                              int n, int hop, void* stream);

/* Per-kernel timing with hipEvents recorded on the launch stream (for bench.py).  enable:
 * 0 off, 1 every launch, k > 1 the launches of every k-th pv_analysis / pv_resynthesis /
 * pv_process / pv_rt_push call (an event record costs the queue a few us).  Within one call
 * the launches share events: launch i+1's timing starts at launch i's stop event, so any
 * GPU idle time while the host enqueues launch i+1 counts toward launch i+1 (a bias of a few
 * us at most, visible only on the short carry / seam launches). */
pv_status pv_profile_enable(pv_handle* h, int enable);
/* names[i] (static strings), total ms and launch count of each kernel since the last
 * reset; returns number of kernels written (<= cap). Synchronises the recorded events. */
int pv_profile_read(pv_handle* h, const char** names, double* total_ms, int* launches, int cap);
void pv_profile_reset(pv_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* PV_H */
