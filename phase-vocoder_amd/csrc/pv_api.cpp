// pv_api.cpp — host side of libpv: the C-ABI declared in include/pv.h.
//
// Owns the per-handle constant tables (windows, twiddles, unwrap tables, pitch map),
// the workspace (run sums, carries, overlap tails) and the launch sequence of the
// pipeline.  No allocation or synchronisation happens inside the compute
// entry points, so a caller may capture them into a hipGraph.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pv.h"
#include "pv_kernels.h"

namespace {

thread_local std::string g_last_error;

pv_status fail(pv_status s, const std::string& msg) {
    g_last_error = msg;
    return s;
}

#define PV_HIP(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(e_ == hipErrorOutOfMemory ? PV_ERR_NOMEM : PV_ERR_HIP,          \
                        std::string(#expr) + ": " + hipGetErrorString(e_));             \
    } while (0)

constexpr double kPi = 3.14159265358979323846;
constexpr int kNumKernels = 8;
const char* kKernelNames[kNumKernels] = {"analysis", "runsum", "carry", "synthesis",
                                         "seam", "compat_analysis", "rt", "fused"};
enum { KA = 0, KRS = 1, KC = 2, KS = 3, KSEAM = 4, KCA = 5, KRT = 6, KF = 7 };

bool is_pow2(long long v) { return v > 0 && (v & (v - 1)) == 0; }

// ---- table recipes (identical double -> float formulas to the oracle, pvref.c) ----
void hann_periodic(int N, std::vector<float>& w) {
    w.resize(N);
    for (int n = 0; n < N; ++n)
        w[n] = (float)(0.5 - 0.5 * std::cos(2.0 * kPi * (double)n / (double)N));
}

void hann_ref(int N, std::vector<float>& w) {
    // phaseVocoder.h:64-66 (1-argument constructor): 0.5f * (1.f - cosf(2.f*M_PI*i / samples));
    // 2.f*M_PI*i/samples is evaluated in double and rounded to float for cosf
    w.resize(N);
    for (int i = 0; i < N; ++i) w[i] = 0.5f * (1.f - cosf((float)(2.0 * kPi * (double)i / (double)N)));
}

void hamming_ref(int N, std::vector<float>& w) {
    // phaseVocoder.h:85-89
    w.resize(N);
    float omega = (float)(2.0 * kPi / (double)(N - 1));
    for (int i = 0; i < N; ++i) {
        float arg = omega * (float)i;
        w[i] = 0.54f - 0.46f * cosf(arg);
    }
}

float2 tw_entry(long long m, long long L) {
    double a = 2.0 * kPi * (double)m / (double)L;
    return make_float2((float)std::cos(a), (float)(-std::sin(a)));
}

// stage-major table for an L-point Stockham FFT: stage Ns at [Ns-1, 2Ns-1)
void stage_twiddles(int L, std::vector<float2>& t) {
    t.assign(L, make_float2(0.f, 0.f));
    for (int Ns = 1; Ns < L; Ns <<= 1)
        for (int idx = 0; idx < Ns; ++idx) t[Ns - 1 + idx] = tw_entry((long long)idx * (L / (2 * Ns)), L);
}

// The FFT table of an L-point transform: the contract-v3 pass table for L in [128, 512]
// (pass P >= 1: S rows of R - 1 entries e^{-2 pi i m q/(R S)}, the oracle's
// pvr_fft_v3_table), the stage-major radix-2 table otherwise; L entries either way.  v3: the
// pass table at any L (the batched synthesis's L = 1024 inverse FFT, which no contract binds).
void fft_table(int L, std::vector<float2>& t, bool v3 = false) {
    if (!v3 && (L < 128 || L > 512)) {
        stage_twiddles(L, t);
        return;
    }
    t.assign(L, make_float2(0.f, 0.f));
    const int E = L / 64;
    int off = 0;
    for (int S = E; S < L;) {
        const int R = std::min(E, L / S);
        for (int m = 0; m < S; ++m)
            for (int q = 1; q < R; ++q)
                t[off + m * (R - 1) + (q - 1)] = tw_entry(((long long)m * q * (L / (R * S))) % L, L);
        off += S * (R - 1);
        S *= R;
    }
}

// d_tw_syn: the synthesis-side L-point table (stage-major or v3, fft_table), then at L = 1024
// the v3 pass table of the batched synthesis's inverse FFT (k_synthesis reads tw + L; the
// real-time and fused kernels run the analysis transform from the first table too), at
// L = 256, 512 the L/2-point table of the fused pitch-2 resynthesis (k_fused MODE 4, tw + L;
// the single launch exists for L <= 512 only)
int tw_syn_len(int L) { return L == 1024 ? 2 * L : (L == 256 || L == 512) ? L + L / 2 : L; }

void split_twiddles(int N, std::vector<float2>& t) {
    t.resize(N / 2 + 1);
    for (int k = 0; k <= N / 2; ++k) t[k] = tw_entry(k, N);
}

struct Profile {
    bool enabled = false;
    int stride = 1;        // time every stride-th pv_analysis / pv_resynthesis / pv_process call
    long long calls = 0;
    bool active = true;    // this call's launches are timed
    // consecutive launches of one call share an event: launch i's stop is launch i+1's start
    // (nothing else is enqueued between them), one event record per launch instead of two
    bool chain_ok = false;
    hipEvent_t chain_ev = nullptr;
    hipStream_t chain_s = nullptr;
    std::vector<hipEvent_t> ev_start, ev_stop;
    std::vector<char> ev_shared;   // ev_start[i] is ev_stop[i-1] (returned to the pool once)
    std::vector<hipEvent_t> pool;  // read-out events, reused (hipEventCreate per launch costs µs)
    std::vector<int> ev_kernel;
    double total_ms[kNumKernels] = {0};
    int launches[kNumKernels] = {0};
};

}  // namespace

struct pv_handle {
    pv_config cfg{};
    int N = 0, hop = 0, hs = 0, L_ana = 0, L_syn = 0, bins = 0, bins_pad = 0;
    int spec_bins = 0, spec_stride = 0, F = 16, tail_len = 0, max_runs = 0;
    int F_fused = 0;  // frames per run of the single-launch q = 1 path (0: not available)
    // environment overrides, read once by pv_create (pv.h lists them)
    int compat_ana_frames = 4;  // PV_COMPAT_ANA_FRAMES: REF_COMPAT analysis run length
    int fused_half = 1;         // PV_FUSED_HALF=0: pitch 2 single launch without MODE 4
    int fused_balance = 1;      // PV_FUSED_BALANCE=0: uniform runs on the single launch
    int src_hi = 0;   // highest analysis bin any output bin reads (pitch map; L otherwise)
    int tables_ready = 1;  // 0: pv_config.tables_external until pv_import_tables
    int mode = 0, effect = 0, pitch = 0, aligned_hop = 1, nan_faithful = 0;
    int packed = 0;  // PV_SPEC_PACKED rows (STANDARD)
    float scale = 1.0f, rho = 1.0f, inv_q = 1.0f;
    unsigned long long p_mod = 0, q = 1;
    int q_pow2 = 1;
    int k_lane = 0;  // e_k and (p j_k) mod q depend on k mod 64 only (synthesis LANEK kernels)
    // device tables
    float *d_win = nullptr, *d_gain = nullptr, *d_ek = nullptr;
    float2 *d_tw_ana = nullptr, *d_tws_ana = nullptr, *d_tw_syn = nullptr, *d_tws_syn = nullptr;
    unsigned* d_jk_mod = nullptr;
    int *d_src_first = nullptr, *d_src_cnt = nullptr;
    // workspace
    int *d_runsum = nullptr, *d_carry = nullptr;
    int* d_seg_carry = nullptr;  // [C][bins_pad] unwrap count before a stream segment
    float* d_seg_phi = nullptr;  // [C][bins_pad] phase of the frame before it
    float* d_tails = nullptr;
    // pv_process without a spectrum buffer on the split path: the handle's own rows
    // (max_channels x max_frames, zeroed; allocated by pv_reserve_spectrum or the first such
    // call outside a stream capture — spec_mu orders concurrent first calls)
    pv_float2* d_spec_own = nullptr;
    std::mutex spec_mu;
    int* d_seam_flags = nullptr;  // fused path: per (channel, workgroup) arrival counters
#ifdef PV_FUSED_STAMPS
    unsigned long long* d_stamps = nullptr;  // diagnostic build: per-wave phase stamps of k_fused
    size_t n_stamps = 0;
#endif
    Profile prof;
};

namespace {

template <typename T>
pv_status upload(T** dst, const std::vector<T>& src);
// a constant table of the handle: uploaded, or (pv_config.tables_external) allocated zeroed
// for pv_import_tables to fill — the host copy never reaches the device
template <typename T>
pv_status upload_table(T** dst, const std::vector<T>& src, bool external) {
    if (!external) return upload(dst, src);
    const size_t bytes = sizeof(T) * (src.empty() ? 1 : src.size());
    PV_HIP(hipMalloc((void**)dst, bytes));
    PV_HIP(hipMemset(*dst, 0, bytes));
    return PV_OK;
}
template <typename T>
pv_status upload(T** dst, const std::vector<T>& src) {
    PV_HIP(hipMalloc((void**)dst, sizeof(T) * (src.empty() ? 1 : src.size())));
    if (!src.empty()) PV_HIP(hipMemcpy(*dst, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice));
    return PV_OK;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// one public call (pv_analysis / pv_resynthesis / pv_process / pv_rt_push): with a stride k > 1 only every
// k-th call's launches get events (each event record costs the queue a few us, which a
// 40-us single-stream step would otherwise carry in its timed region)
void prof_tick(pv_handle* h) {
    if (h->prof.enabled) h->prof.active = (h->prof.calls++ % h->prof.stride) == 0;
}

// the launches of one pv_analysis / pv_resynthesis / pv_process call, which enqueue nothing
// but kernels, may chain their events
struct ProfCall {
    pv_handle* h;
    explicit ProfCall(pv_handle* hh) : h(hh) {
        prof_tick(h);
        h->prof.chain_ok = true;
        h->prof.chain_ev = nullptr;
    }
    ~ProfCall() { h->prof.chain_ok = false; h->prof.chain_ev = nullptr; }
};

pv_status prof_begin(pv_handle* h, int kernel, hipStream_t s) {
    if (!h->prof.enabled || !h->prof.active) return PV_OK;
    hipEvent_t a, b;
    auto take = [&](hipEvent_t* e) -> pv_status {
        if (!h->prof.pool.empty()) {
            *e = h->prof.pool.back();
            h->prof.pool.pop_back();
            return PV_OK;
        }
        PV_HIP(hipEventCreate(e));
        return PV_OK;
    };
    const bool shared = h->prof.chain_ok && h->prof.chain_ev && h->prof.chain_s == s;
    pv_status st = PV_OK;
    if (shared) a = h->prof.chain_ev;
    else st = take(&a);
    if (st == PV_OK) st = take(&b);
    if (st != PV_OK) return st;
    if (!shared) PV_HIP(hipEventRecord(a, s));
    h->prof.ev_start.push_back(a);
    h->prof.ev_stop.push_back(b);
    h->prof.ev_shared.push_back(shared ? 1 : 0);
    h->prof.ev_kernel.push_back(kernel);
    return PV_OK;
}

pv_status prof_end(pv_handle* h, hipStream_t s) {
    if (!h->prof.enabled || !h->prof.active) return PV_OK;
    PV_HIP(hipEventRecord(h->prof.ev_stop.back(), s));
    if (h->prof.chain_ok) {
        h->prof.chain_ev = h->prof.ev_stop.back();
        h->prof.chain_s = s;
    }
    return PV_OK;
}

#define PV_LAUNCH(h, kid, s, call)                                                    \
    do {                                                                              \
        pv_status st_ = prof_begin(h, kid, s);                                        \
        if (st_ != PV_OK) return st_;                                                 \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(PV_ERR_HIP, std::string(kKernelNames[kid]) + " launch: " +    \
                                        hipGetErrorString(e_));                       \
        st_ = prof_end(h, s);                                                         \
        if (st_ != PV_OK) return st_;                                                 \
    } while (0)

int nruns_of(const pv_handle* h, int frames) { return (frames + h->F - 1) / h->F; }

pv_status check_common(const pv_handle* h, int channels, int frames) {
    if (!h) return fail(PV_ERR_ARG, "null handle");
    if (!h->tables_ready)
        return fail(PV_ERR_ARG, "tables_external handle: no tables yet (pv_import_tables first)");
    if (channels < 0 || frames < 0) return fail(PV_ERR_ARG, "negative channels/frames");
    if (channels > h->cfg.max_channels || frames > h->cfg.max_frames)
        return fail(PV_ERR_ARG, "channels/frames exceed the handle's capacity (max_channels, max_frames)");
    return PV_OK;
}

// src_hi < 0: every bin analysed (the spectrum is an output); otherwise the bins above it
// may be left out (pv_process without a spectrum buffer: no output bin reads them)
pv_status do_analysis(pv_handle* h, const float* x, long long ldx, long long n, int C, int frames,
                      pv_float2* spec, long long ld_spec, bool want_runsum, hipStream_t s,
                      int src_hi = -1) {
    if (C == 0 || frames == 0) return PV_OK;
    if (!x || !spec) return fail(PV_ERR_ARG, "null x/spec");
    if (ld_spec < (long long)frames * h->spec_stride)
        return fail(PV_ERR_ARG, "ld_spec < frames * spec_stride");
    if (C > 1 && ldx < n) return fail(PV_ERR_ARG, "ldx < n_samples");
    pv::AnaParams p{};
    p.x = x;
    p.ldx = ldx;
    p.n = n;
    p.hop = h->hop;
    p.frames = frames;
    p.F = h->F;
    p.nruns = nruns_of(h, frames);
    p.aligned = (((uintptr_t)x & 7) == 0) && (ldx % 2 == 0) && (h->hop % 2 == 0);
    p.win = h->d_win;
    p.tw = h->d_tw_ana;
    p.tws = h->d_tws_ana;
    p.ek = h->d_ek;
    p.ek_lane = (64 % h->cfg.hop_div == 0 && h->bins >= 64) ? 1 : 0;
    p.spec = reinterpret_cast<float2*>(spec);
    p.ld_spec = ld_spec;
    p.spec_stride = h->spec_stride;
    p.runsum = want_runsum ? h->d_runsum : nullptr;
    p.bins_pad = h->bins_pad;
    p.nan_faithful = h->nan_faithful;
    p.packed = h->packed;
    p.src_hi = (src_hi < 0) ? h->L_ana : std::min(src_hi, h->L_ana);
    if (h->mode == PV_MODE_REF_COMPAT) {
        // the REF_COMPAT analysis has no run records: its runs only set which rows a wave
        // writes in turn, and short runs (fewer rows written concurrently per channel, more
        // channels' rows in address order) stream faster (profiles/r05_ab_compat_F.txt);
        // the synthesis keeps h->F (its seams)
        const int fa = h->compat_ana_frames;
        p.F = fa;
        p.nruns = (frames + fa - 1) / fa;
    }
    if (h->mode == PV_MODE_STANDARD)
        PV_LAUNCH(h, KA, s, pv::launch_std_analysis(h->L_ana, C, p, s));
    else
        PV_LAUNCH(h, KCA, s, pv::launch_compat_analysis(h->L_ana, C, p, s));
    return PV_OK;
}

// the state before a segment of a longer stream (pv_segment_resynthesis)
struct SegState {
    const int* carry_in;
    const float* phi_in;
    unsigned t_off;
};

// carry_from: unwrap carries already scanned by another handle of the same analysis
// geometry (the harmoniser's voices share one scan); nullptr = scan here.
pv_status do_resynthesis(pv_handle* h, const pv_float2* spec, long long ld_spec, int C, int frames,
                         const float* ola_in, long long ld_ola, float* out, long long ldo,
                         bool have_runsum, hipStream_t s, const int* carry_from = nullptr,
                         bool force_scan = false, const SegState* seg = nullptr) {
    if (C == 0 || frames == 0) {
        return PV_OK;
    }
    if (!spec || !out) return fail(PV_ERR_ARG, "null spec/out");
    const long long olen = pv_output_length(h, frames);
    if (C > 1 && ldo < olen) return fail(PV_ERR_ARG, "ldo < pv_output_length");
    if (ld_spec < (long long)frames * h->spec_stride)
        return fail(PV_ERR_ARG, "ld_spec < frames * spec_stride");
    const int nruns = nruns_of(h, frames);
    const float2* sp = reinterpret_cast<const float2*>(spec);
    // q = 1 (e.g. pitch 2.0): the output phase rho (phi + 2 pi M) is independent of the
    // unwrap count M mod 1, so no scan is needed
    const bool need_scan = h->mode == PV_MODE_STANDARD && (h->q > 1 || force_scan);
    if (need_scan && carry_from == nullptr) {
        pv::ScanParams sc{};
        sc.spec = sp;
        sc.ld_spec = ld_spec;
        sc.spec_stride = h->spec_stride;
        sc.frames = frames;
        sc.F = h->F;
        sc.nruns = nruns;
        sc.L = h->L_syn;
        sc.bins_pad = h->bins_pad;
        sc.packed = h->packed;
        sc.ek = h->d_ek;
        sc.runsum = h->d_runsum;
        sc.carry = h->d_carry;
        sc.carry_in = seg ? seg->carry_in : nullptr;
        sc.phi_in = seg ? seg->phi_in : nullptr;
        if (!have_runsum) PV_LAUNCH(h, KRS, s, pv::launch_runsum(C, sc, s));
        PV_LAUNCH(h, KC, s, pv::launch_carry(C, sc, s));
    }
    pv::SynParams p{};
    p.spec = sp;
    p.ld_spec = ld_spec;
    p.spec_stride = h->spec_stride;
    p.frames = frames;
    p.F = h->F;
    p.nruns = nruns;
    p.bins_pad = h->bins_pad;
    p.carry = carry_from ? carry_from : (need_scan ? h->d_carry : nullptr);
    p.ek = h->d_ek;
    p.jk_mod = h->d_jk_mod;
    p.src_first = h->d_src_first;
    p.src_cnt = h->d_src_cnt;
    p.pitch = h->pitch;
    p.rho = h->rho;
    p.p_mod = h->p_mod;
    p.q = h->q;
    p.q_pow2 = h->q_pow2;
    p.inv_q = h->inv_q;
    p.tw = h->d_tw_syn + (h->L_syn == 1024 ? h->L_syn : 0);  // L = 1024: the v3 pass table
    p.tws = h->d_tws_syn;
    p.gain = h->d_gain;
    p.rot = (h->mode == PV_MODE_REF_COMPAT) ? h->N / 2 : 0;
    p.hs = h->hs;
    p.out = out;
    p.ldo = ldo;
    p.out_len = olen;
    p.out_aligned = ((reinterpret_cast<uintptr_t>(out) & 7) == 0) && ((ldo & 1) == 0);
    p.tails = h->d_tails;
    p.tail_len = h->tail_len;
    p.k_lane = h->k_lane;
    p.packed = h->packed;
    p.src_hi = h->src_hi;
    p.t_off = seg ? seg->t_off : 0u;
    const int smode = (h->mode == PV_MODE_REF_COMPAT) ? 1 : (h->pitch ? 2 : 0);
    PV_LAUNCH(h, KS, s, pv::launch_synthesis(h->L_syn, smode, C, p, s));
    const int nwg = (nruns + 3) / 4;
    if (nwg > 1 || ola_in != nullptr) {
        pv::SeamParams sm{};
        sm.out = out;
        sm.ldo = ldo;
        sm.out_len = olen;
        sm.tails = h->d_tails;
        sm.ola_in = ola_in;
        sm.ld_ola = ld_ola;
        sm.nruns = nruns;
        sm.nwg = nwg;
        sm.F = h->F;
        sm.hs = h->hs;
        sm.tail_len = h->tail_len;
        PV_LAUNCH(h, KSEAM, s, pv::launch_seam(C, sm, s));
    }
    return PV_OK;
}

// q = 1 (STANDARD): analysis, processing, resynthesis and every seam in one launch
// (pv_fused.hip); outputs equal to do_analysis + do_resynthesis (bit for bit at equal F)
pv_status do_fused(pv_handle* h, const float* x, long long ldx, long long n, int C, int frames,
                   pv_float2* spec, long long ld_spec, float* out, long long ldo, hipStream_t s) {
    if (C == 0 || frames == 0) return PV_OK;
    if (!x || !out) return fail(PV_ERR_ARG, "null x/out");
    // spec == NULL: no spectrum output (the single launch keeps the rows on chip)
    if (spec && ld_spec < (long long)frames * h->spec_stride)
        return fail(PV_ERR_ARG, "ld_spec < frames * spec_stride");
    if (C > 1 && ldx < n) return fail(PV_ERR_ARG, "ldx < n_samples");
    const long long olen = pv_output_length(h, frames);
    if (C > 1 && ldo < olen) return fail(PV_ERR_ARG, "ldo < pv_output_length");
    const int F = h->F_fused;
    const int nruns = (frames + F - 1) / F;
    pv::FusedParams p{};
    p.x = x;
    p.ldx = ldx;
    p.n = n;
    p.hop = h->hop;
    p.frames = frames;
    p.F = F;
    p.nruns = nruns;
    p.aligned = (((uintptr_t)x & 7) == 0) && (ldx % 2 == 0) && (h->hop % 2 == 0);
    p.win = h->d_win;
    p.tw = h->d_tw_syn;    // the stage-major L-point table serves both directions
    p.tws = h->d_tws_syn;  // e^{-2 pi i k/N}, k <= N/2: the analysis split's table too
    p.src_first = h->d_src_first;
    p.src_cnt = h->d_src_cnt;
    p.rho = h->rho;
    p.gain = h->d_gain;
    // pitch 2: the periodic half-size resynthesis (k_fused MODE 4); PV_FUSED_HALF=0 keeps the
    // MODE 3 gather and the full-size inverse FFT (tests compare the two)
    p.tw_half = (tw_syn_len(h->L_syn) == h->L_syn + h->L_syn / 2) ? h->d_tw_syn + h->L_syn : nullptr;
    if (!h->fused_half) p.tw_half = nullptr;
    p.hs = h->hs;
    p.spec = reinterpret_cast<float2*>(spec);
    p.ld_spec = ld_spec;
    p.spec_stride = h->spec_stride;
    p.out = out;
    p.ldo = ldo;
    p.out_len = olen;
    p.out_aligned = ((reinterpret_cast<uintptr_t>(out) & 7) == 0) && ((ldo & 1) == 0);
    p.tails = h->d_tails;
    p.tail_len = h->tail_len;
    p.seam_flags = h->d_seam_flags;
    p.packed = h->packed;
    p.src_hi = h->src_hi;
    p.nwg = (nruns + 3) / 4;
    p.n4 = 0;
    // a stream whose workgroups do not fill whole rounds of the 256 CUs (config 2: 862 =
    // 3 x 256 + 94, so 94 CUs ran a 4th workgroup, 12 frames on their SIMDs against 9):
    // exactly `rounds` workgroups per CU, some runs one frame longer (k_fused "balanced";
    // PV_FUSED_BALANCE=0 turns it off).  The run boundaries move, so the seams' rounding
    // does (<= 1e-6); the output depends only on the configuration.
    {
        constexpr int kRoundCUs = 256;  // MI355X
        const int rounds = p.nwg / kRoundCUs;
        const bool on = h->fused_balance != 0;
        // (decided from the frame count alone, for any number of channels: a channel's runs
        // and so its output bits are the same alone or in a batch — ADVICE r5)
        if (on && rounds >= 1 && p.nwg % kRoundCUs != 0) {
            const int G = rounds * kRoundCUs;
            const long long n4 = (long long)frames - 4LL * F * G;
            if (n4 > 0 && n4 <= 4LL * G) {
                p.nwg = G;
                p.n4 = (int)n4;
            }
        }
    }
#ifdef PV_FUSED_STAMPS
    p.stamps = h->d_stamps;
#endif
    PV_LAUNCH(h, KF, s, pv::launch_fused(h->L_syn, h->pitch ? 2 : 0, C, p, s));
    return PV_OK;
}

}  // namespace

extern "C" {

int pv_abi_version(void) { return PV_ABI_VERSION; }

// 2 (round 4): fused real-split accumulation, one-rounding unwrap decision (pv_device.hpp);
// 3: twiddle-first radix-E FFT passes with the window folded in, L <= 512 (fft_pass v3)
int pv_contract_version(void) { return 4; }
#ifndef PV_SOURCES_SHA
#define PV_SOURCES_SHA "unset"
#endif
const char* pv_sources_sha(void) { return PV_SOURCES_SHA; }
int pv_diagnostic_build(void) {
#ifdef PV_DIAGNOSTIC_BUILD
    return 1;
#else
    return 0;
#endif
}

const char* pv_status_string(pv_status s) {
    switch (s) {
        case PV_OK: return "PV_OK";
        case PV_ERR_ARG: return "PV_ERR_ARG";
        case PV_ERR_UNSUPPORTED: return "PV_ERR_UNSUPPORTED";
        case PV_ERR_HIP: return "PV_ERR_HIP";
        case PV_ERR_NOMEM: return "PV_ERR_NOMEM";
    }
    return "PV_ERR_UNKNOWN";
}

const char* pv_last_error(void) { return g_last_error.c_str(); }

int pv_frame_count(long long n_samples, int hop) {
    // main.cpp:231: for (i = 0; i < numSamples - hopSize; i += hopSize)
    if (hop <= 0) return 0;
    long long span = n_samples - hop;
    if (span <= 0) return 0;
    return (int)((span + hop - 1) / hop);
}

long long pv_output_length(const pv_handle* h, int frames) {
    if (!h || frames <= 0) return 0;
    return (long long)frames * h->hs + (h->N - h->hs);
}

pv_status pv_get_info(const pv_handle* h, pv_info* info) {
    if (!h || !info) return fail(PV_ERR_ARG, "null argument");
    if (info->abi_version != PV_ABI_VERSION)
        return fail(PV_ERR_ARG, "pv_info.abi_version != PV_ABI_VERSION (caller built against another pv.h)");
    info->n_samps = h->N;
    info->hop = h->hop;
    info->out_hop = h->hs;
    info->spec_bins = h->spec_bins;
    info->spec_stride = h->spec_stride;
    info->frames_per_run = h->F;
    info->mode = h->mode;
    info->effect = h->effect;
    info->scale = h->scale;
    info->single_launch = h->F_fused > 0 ? 1 : 0;
    info->single_launch_frames = h->F_fused;
    info->lane_constants = h->k_lane;
    info->spec_layout = h->packed ? PV_SPEC_PACKED : PV_SPEC_NATURAL;
    return PV_OK;
}

#ifdef PV_FUSED_STAMPS
// diagnostic build only (make variant NAME=stamps DEFS=-DPV_FUSED_STAMPS): the per-wave
// phase stamps of the last k_fused launch, kFusedStampSlots per wave (scripts/fused_stamps.py)
pv_status pv_debug_stamps(const pv_handle* h, unsigned long long* dst, size_t count) {
    if (!h || !dst || !h->d_stamps) return PV_ERR_ARG;
    DeviceGuard g(h->cfg.device);
    if (hipDeviceSynchronize() != hipSuccess) return PV_ERR_HIP;
    if (hipMemcpy(dst, h->d_stamps, sizeof(unsigned long long) * std::min(count, h->n_stamps),
                  hipMemcpyDeviceToHost) != hipSuccess)
        return PV_ERR_HIP;
    return PV_OK;
}
#endif

void pv_destroy(pv_handle* h) {
    if (!h) return;
    DeviceGuard g(h->cfg.device);
    void* ptrs[] = {h->d_win, h->d_gain, h->d_ek, h->d_tw_ana, h->d_tws_ana, h->d_tw_syn,
                    h->d_tws_syn, h->d_jk_mod, h->d_src_first, h->d_src_cnt, h->d_runsum,
                    h->d_carry, h->d_tails, h->d_seam_flags, h->d_spec_own, h->d_seg_carry,
                    h->d_seg_phi};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
#ifdef PV_FUSED_STAMPS
    if (h->d_stamps) (void)hipFree(h->d_stamps);
#endif
    for (size_t i = 0; i < h->prof.ev_start.size(); ++i)
        if (!h->prof.ev_shared[i]) (void)hipEventDestroy(h->prof.ev_start[i]);
    for (auto e : h->prof.ev_stop) (void)hipEventDestroy(e);
    for (auto e : h->prof.pool) (void)hipEventDestroy(e);
    delete h;
}

pv_status pv_create(const pv_config* cfg, pv_handle** out) {
    if (!cfg || !out) return fail(PV_ERR_ARG, "null argument");
    *out = nullptr;
    if (cfg->abi_version != PV_ABI_VERSION)
        return fail(PV_ERR_ARG, "pv_config.abi_version != PV_ABI_VERSION (caller built against another pv.h)");
    const int N = cfg->n_samps;
    if (!is_pow2(N)) return fail(PV_ERR_UNSUPPORTED, "n_samps must be a power of two");
    if (cfg->mode != PV_MODE_STANDARD && cfg->mode != PV_MODE_REF_COMPAT)
        return fail(PV_ERR_ARG, "unknown mode");
    if (cfg->effect != PV_TIME_SHIFT && cfg->effect != PV_PITCH_SHIFT)
        return fail(PV_ERR_ARG, "unknown effect");
    if (cfg->hop_div <= 0 || N / cfg->hop_div <= 0) return fail(PV_ERR_ARG, "bad hop_div");
    if (cfg->max_channels < 0 || cfg->max_frames < 0) return fail(PV_ERR_ARG, "negative capacity");
    if (!(cfg->scale > 0.0f) || !std::isfinite(cfg->scale)) return fail(PV_ERR_ARG, "scale must be > 0");
    if (cfg->mode == PV_MODE_STANDARD && (N < 256 || N > 2048))
        return fail(PV_ERR_UNSUPPORTED, "STANDARD mode: n_samps in [256, 2048]");
    if (cfg->mode == PV_MODE_REF_COMPAT && (N < 256 || N > 2048))
        return fail(PV_ERR_UNSUPPORTED, "REF_COMPAT mode: n_samps in [256, 2048]");
    if (cfg->window < PV_WINDOW_DEFAULT || cfg->window > PV_WINDOW_HANN_REF)
        return fail(PV_ERR_ARG, "unknown window");
    if (cfg->mode == PV_MODE_STANDARD && cfg->window != PV_WINDOW_DEFAULT)
        return fail(PV_ERR_UNSUPPORTED, "STANDARD mode: the periodic Hann window only (window = 0)");
    if (cfg->spec_layout != PV_SPEC_NATURAL && cfg->spec_layout != PV_SPEC_PACKED)
        return fail(PV_ERR_ARG, "unknown spec_layout");
    if (cfg->spec_layout == PV_SPEC_PACKED && cfg->mode != PV_MODE_STANDARD)
        return fail(PV_ERR_UNSUPPORTED, "PV_SPEC_PACKED: STANDARD handles only");

    pv_handle* h = new pv_handle();
    h->cfg = *cfg;
    h->N = N;
    h->mode = cfg->mode;
    h->effect = cfg->effect;
    h->scale = cfg->scale;
    h->nan_faithful = (cfg->mode == PV_MODE_REF_COMPAT && cfg->nan_faithful) ? 1 : 0;
    h->hop = N / cfg->hop_div;  // phaseVocoder.h:79
    if (cfg->effect == PV_TIME_SHIFT) {
        float f = cfg->scale * (float)h->hop;  // phaseVocoder.h:104 (float -> int)
        h->hs = (int)f;
    } else {
        h->hs = h->hop;  // PITCH_SHIFT: defined by the build (reference leaves it unset)
    }
    if (h->hs <= 0 || h->hs > N) {
        delete h;
        return fail(PV_ERR_UNSUPPORTED, "out hop must be in [1, N]");
    }
    if (h->mode == PV_MODE_REF_COMPAT && cfg->effect == PV_PITCH_SHIFT && cfg->scale != 1.0f) {
        delete h;
        return fail(PV_ERR_UNSUPPORTED, "REF_COMPAT implements no pitch shift (phaseVocoder.h:107-110)");
    }
    if (h->mode == PV_MODE_REF_COMPAT && cfg->effect == PV_TIME_SHIFT && h->hs != h->hop) {
        // kernel.cu:354 hard-codes timeScale = 1: the reference only changes the OLA hop.
    }
    h->pitch = (cfg->mode == PV_MODE_STANDARD && cfg->effect == PV_PITCH_SHIFT) ? 1 : 0;
    h->L_syn = N / 2;
    h->L_ana = (h->mode == PV_MODE_STANDARD) ? N / 2 : N;
    h->bins = N / 2 + 1;
    h->bins_pad = (h->bins + 7) & ~7;
    h->packed = (cfg->spec_layout == PV_SPEC_PACKED) ? 1 : 0;
    // packed rows are exactly N/2 float2: bin N/2 rides in slot 0
    h->spec_bins = (h->mode == PV_MODE_STANDARD) ? (h->packed ? N / 2 : h->bins) : 2 * N;
    h->spec_stride = (h->spec_bins + 7) & ~7;
    if (h->L_ana > 2048 || h->L_syn > 2048 || h->L_syn < 128) {
        delete h;
        return fail(PV_ERR_UNSUPPORTED, "FFT length outside [128, 2048]");
    }
    h->tail_len = N - h->hs;
    // frames per wave-run: longer runs amortise the halo frame each run transforms (1/F of
    // the analysis work) as long as the batch still yields >= 2048 workgroups of 4 runs;
    // a run's output span must cover the overlap tail
    const long long work = (long long)std::max(cfg->max_channels, 1) * std::max(cfg->max_frames, 1);
    // (measured on config 3: F = 32 / 48 / 64 / 96 -> 3.64 / 3.74 / 3.72 / 3.62e8 frames/s)
    int F = (work >= 2048LL * 4 * 48) ? 48 : (work >= 2048LL * 4 * 32) ? 32 : (work >= 1024LL * 4 * 16) ? 16 : 8;
    // a frame at L >= 1024 is twice the work: runs of 32 (measured on the config-4 slice,
    // 1024 channels x 861 frames: F = 24 / 32 / 40 / 48 / 64 -> 1.51-1.52 / 1.53-1.54 /
    // 1.47-1.48 / 1.49-1.50 / 1.46-1.49e8 frames/s)
    if (h->L_syn >= 1024 && F > 32) F = 32;
    // Large STANDARD batches at L <= 512: the analysis grid runs in rounds of (workgroups one
    // CU holds) x CUs, and a last partial round leaves most of the chip idle while its runs
    // finish.  Among F = 48, 56, .. 96 take the one with the fewest frame-times, rounds x F
    // (near-ties: the longer runs, below).  Config 3 at round 5's 5 workgroups per CU: 48 gives
    // 9216 workgroups = 8 rounds (the last a fifth full) x 48 = 384, 88 gives 5120 = 4 x 88 =
    // 352 (measured on two boxes: +1.7 / +1.8 % frames/s, profiles/r04_ab_c3_F.txt; what the
    // longer runs buy is the carry, seam and synthesis time — the analysis kernel itself is
    // within +-2 % from F = 24 to 88, profiles/r05_ab_c3_F_sweep.txt).  The rounds are counted
    // on the MI355X's 256 CUs whatever device the handle is on, and the workgroups per CU
    // come from the compiled kernel's resources: F, which sets where the overlap-add sums are
    // split into run seams (their rounding, <= 1e-6), depends only on the configuration, so
    // the same batch gives the same output bits on any gfx950 device or partition mode.
    if (F == 48 && h->L_ana <= 512 && h->mode == PV_MODE_STANDARD) {
        DeviceGuard g0(cfg->device);
        constexpr int kRoundCUs = 256;  // MI355X
        const bool ekl = (64 % cfg->hop_div == 0 && h->bins >= 64);
        int W = 4;
        const int wpc = pv::std_analysis_wgs_per_cu(h->L_ana, h->hop, ekl, h->packed != 0, &W);
        if (wpc > 0) {
            const long long slots = (long long)kRoundCUs * wpc;
            const long long C = std::max(cfg->max_channels, 1), T = std::max(cfg->max_frames, 1);
            // (round 6: the longest run within 2 % of the fewest frame-times — each run costs a
            // record, a carry and a seam; with the 4-wave/SIMD analysis config 3 has 48 -> 432
            // and 88 -> 440 frame-times, and F = 88 measured +1.9 % frames/s over 48)
            long long best = -1;
            long long cost_of[7];
            for (int j = 0, f = 48; f <= 96; f += 8, ++j) {
                const long long wgs = C * (((T + f - 1) / f + W - 1) / W);
                cost_of[j] = ((wgs + slots - 1) / slots) * f;
                if (best < 0 || cost_of[j] < best) best = cost_of[j];
            }
            for (int j = 0, f = 48; f <= 96; f += 8, ++j)
                if (cost_of[j] * 100 <= best * 102) F = f;
        }
    }
    // the single-launch and REF_COMPAT overrides (pv.h), read once here
    if (const char* ev = std::getenv("PV_COMPAT_ANA_FRAMES")) {
        const int f = std::atoi(ev);
        if (f >= 1 && f <= 256) h->compat_ana_frames = f;
    }
    if (const char* eh = std::getenv("PV_FUSED_HALF")) h->fused_half = (eh[0] == '0') ? 0 : 1;
    if (const char* eb = std::getenv("PV_FUSED_BALANCE")) h->fused_balance = (eb[0] == '0') ? 0 : 1;
    // tuning override (even, 8..256): PV_RUN_FRAMES
    if (const char* ev = std::getenv("PV_RUN_FRAMES")) {
        const int f = std::atoi(ev);
        if (f >= 8 && f <= 256 && f % 2 == 0) F = f;
    }
    while ((long long)F * h->hs < h->tail_len) F += 4;
    h->F = F;
    h->max_runs = (cfg->max_frames + F - 1) / F;

    DeviceGuard g(cfg->device);
    pv_status st = PV_OK;
    auto bail = [&](pv_status s) {
        pv_destroy(h);
        return s;
    };

    // ---- constant tables (pv_config.tables_external: allocated zeroed, filled only by
    // pv_import_tables — a non-root rank of a multi-GPU job receives rank 0's)
    const bool ext_tables = cfg->tables_external != 0;
    h->tables_ready = ext_tables ? 0 : 1;
    auto upload_tab = [&](auto** dst, const auto& v) { return upload_table(dst, v, ext_tables); };

    // ---- windows and gains
    std::vector<float> win, gain(N);
    if (h->mode == PV_MODE_STANDARD) {
        hann_periodic(N, win);
        double sw2 = 0.0;
        std::vector<double> wd(N);
        for (int i = 0; i < N; ++i) {
            wd[i] = 0.5 - 0.5 * std::cos(2.0 * kPi * (double)i / (double)N);
            sw2 += wd[i] * wd[i];
        }
        for (int i = 0; i < N; ++i) gain[i] = (float)(wd[i] * ((double)h->hs / sw2) / (double)N);
    } else {
        if (cfg->window == PV_WINDOW_HANN_REF) hann_ref(N, win);  // PhaseVocoder(int samples)
        else hamming_ref(N, win);
        for (int i = 0; i < N; ++i) gain[i] = win[i] / (float)N;  // kernel.cu:380 /N, :406 window
    }
    if ((st = upload_tab(&h->d_win, win)) != PV_OK) return bail(st);
    if ((st = upload_tab(&h->d_gain, gain)) != PV_OK) return bail(st);

    // ---- twiddles
    std::vector<float2> t;
    fft_table(h->L_ana, t);
    if ((st = upload_tab(&h->d_tw_ana, t)) != PV_OK) return bail(st);
    split_twiddles(2 * h->L_ana, t);
    if ((st = upload_tab(&h->d_tws_ana, t)) != PV_OK) return bail(st);
    fft_table(h->L_syn, t);
    if (h->L_syn == 1024) {
        std::vector<float2> t3;
        fft_table(h->L_syn, t3, true);
        t.insert(t.end(), t3.begin(), t3.end());
    } else if (tw_syn_len(h->L_syn) > h->L_syn) {
        std::vector<float2> th;
        fft_table(h->L_syn / 2, th);
        t.insert(t.end(), th.begin(), th.end());
    }
    if ((st = upload_tab(&h->d_tw_syn, t)) != PV_OK) return bail(st);
    split_twiddles(N, t);
    if ((st = upload_tab(&h->d_tws_syn, t)) != PV_OK) return bail(st);

    // ---- unwrap tables and the rational output-phase factor rho = p/q
    const int B = h->bins;
    std::vector<float> ek(B);
    std::vector<long long> jk(B);
    for (int k = 0; k < B; ++k) {
        long long kh = (long long)k * h->hop;
        long long r = kh % N;
        long long rr = (r > N / 2) ? r - N : r;
        ek[k] = (float)(2.0 * kPi * (double)rr / (double)N);
        jk[k] = (kh - rr) / N;
    }
    unsigned long long pn = 1, qd = 1;
    if (h->pitch) {
        int e2 = 0;
        double m = std::frexp((double)cfg->scale, &e2);  // scale = m * 2^e2, m in [0.5,1)
        long long mant = (long long)std::ldexp(m, 24);   // exact: float has 24 bits
        int ex = e2 - 24;
        while ((mant & 1) == 0 && ex < 0) { mant >>= 1; ++ex; }
        if (ex >= 0) { pn = (unsigned long long)mant << ex; qd = 1; }
        else { pn = (unsigned long long)mant; qd = 1ull << (-ex); }
        h->rho = cfg->scale;
    } else {
        long long a = h->hs, b = h->hop;
        long long x = a, y = b;
        while (y) { long long tt = x % y; x = y; y = tt; }
        pn = a / x;
        qd = b / x;
        h->rho = (float)((double)h->hs / (double)h->hop);
    }
    h->q = qd;
    h->p_mod = pn % qd;
    h->q_pow2 = is_pow2((long long)qd) ? 1 : 0;
    h->inv_q = (float)(1.0 / (double)qd);
    if (!h->q_pow2 && qd > 32768) return bail(fail(PV_ERR_UNSUPPORTED, "output-phase ratio denominator too large"));
    std::vector<unsigned> jkm(B);
    for (int k = 0; k < B; ++k) {
        unsigned long long v = ((pn % qd) * ((unsigned long long)jk[k] % qd)) % qd;
        jkm[k] = (unsigned)v;
    }
    if ((st = upload_tab(&h->d_ek, ek)) != PV_OK) return bail(st);
    if ((st = upload_tab(&h->d_jk_mod, jkm)) != PV_OK) return bail(st);
    {
        // per-lane unwrap constants (the synthesis keeps them in two registers): every bin
        // k < L repeats bin k mod 64, and bin L's e equals bin 0's
        const int smode = (h->mode == PV_MODE_REF_COMPAT) ? 1 : (h->pitch ? 2 : 0);
        bool kl = B > 64 && ek[B - 1] == ek[0] &&
                  pv::synthesis_lane_kernel(h->L_syn, smode, h->hs, h->q_pow2 != 0, h->q);
        for (int k = 64; kl && k < B - 1; ++k) kl = (ek[k] == ek[k & 63]) && (jkm[k] == jkm[k & 63]);
        if (const char* ev = std::getenv("PV_SYN_LANEK"))
            if (ev[0] == '0') kl = false;
        h->k_lane = kl ? 1 : 0;
    }

    // ---- pitch map: k' = floor(beta*k + 0.5) (magnitudes summed, phase from smallest k)
    std::vector<int> first(B, -1), cnt(B, 0);
    if (h->pitch) {
        const double beta = (double)cfg->scale;
        for (int k = 0; k < B; ++k) {
            long long kp = (long long)std::floor(beta * (double)k + 0.5);
            if (kp < 0 || kp >= B) continue;
            if (first[kp] < 0) first[kp] = k;
            cnt[kp]++;
        }
    }
    if ((st = upload_tab(&h->d_src_first, first)) != PV_OK) return bail(st);
    if ((st = upload_tab(&h->d_src_cnt, cnt)) != PV_OK) return bail(st);
    h->src_hi = B - 1;
    if (h->pitch) {
        h->src_hi = -1;
        for (int k = 0; k < B; ++k)
            if (cnt[k] > 0) h->src_hi = std::max(h->src_hi, first[k] + cnt[k] - 1);
    }

    // ---- single-launch path (q = 1): no halo frame, so runs can be as short as the overlap
    // tail allows (F hs >= N - hs) to give a single stream enough waves; PV_FUSED=0 disables
    // it (tests compare both paths), PV_FUSED_FRAMES overrides its run length
    if (h->mode == PV_MODE_STANDARD && h->q == 1 && pv::fused_supported(h->L_syn, h->hs)) {
        const int fmin = std::max(2, (h->tail_len + h->hs - 1) / h->hs);
        int Ff = (int)std::min<long long>(h->F, std::max<long long>(fmin, work / 4096));
        if (const char* ev = std::getenv("PV_FUSED_FRAMES")) {
            const int f = std::atoi(ev);
            if (f >= fmin && f <= 256) Ff = f;
        }
        const char* en = std::getenv("PV_FUSED");
        if (!(en && en[0] == '0')) h->F_fused = Ff;
    }
    const int runs_fused = h->F_fused > 0 ? (cfg->max_frames + h->F_fused - 1) / h->F_fused : 0;

    // ---- workspace
    const size_t chans = (size_t)std::max(cfg->max_channels, 1);
    const size_t runs_total = chans * std::max(h->max_runs, 1);
    const size_t wg_total = chans * std::max((std::max(h->max_runs, runs_fused) + 3) / 4, 1);
    if (h->mode == PV_MODE_STANDARD) {
        PV_HIP(hipMalloc((void**)&h->d_runsum, sizeof(int) * runs_total * pv::kRecFields * h->bins_pad));
        PV_HIP(hipMalloc((void**)&h->d_carry, sizeof(int) * runs_total * h->bins_pad));
        PV_HIP(hipMalloc((void**)&h->d_seg_carry, sizeof(int) * chans * h->bins_pad));
        PV_HIP(hipMalloc((void**)&h->d_seg_phi, sizeof(float) * chans * h->bins_pad));
    }
    PV_HIP(hipMalloc((void**)&h->d_tails, sizeof(float) * wg_total * std::max(h->tail_len, 1)));
    if (h->F_fused > 0) {
        PV_HIP(hipMalloc((void**)&h->d_seam_flags, sizeof(int) * wg_total));
        PV_HIP(hipMemset(h->d_seam_flags, 0, sizeof(int) * wg_total));
#ifdef PV_FUSED_STAMPS
        h->n_stamps = wg_total * 4 * pv::kFusedStampSlots;
        PV_HIP(hipMalloc((void**)&h->d_stamps, sizeof(unsigned long long) * h->n_stamps));
        PV_HIP(hipMemset(h->d_stamps, 0, sizeof(unsigned long long) * h->n_stamps));
#endif
    }

    // LDS budget check for the synthesis kernel (largest)
    size_t lds = pv::synthesis_lds_bytes(h->L_syn, h->hs);
    if (lds > 160 * 1024) return bail(fail(PV_ERR_UNSUPPORTED, "LDS budget exceeded"));
    *out = h;
    return PV_OK;
}

pv_status pv_analysis(pv_handle* h, const float* x, long long ldx, long long n_samples,
                      int channels, int frames, pv_float2* spec, long long ld_spec, void* stream) {
    pv_status st = check_common(h, channels, frames);
    if (st != PV_OK) return st;
    DeviceGuard g(h->cfg.device);
    ProfCall pc_(h);
    return do_analysis(h, x, ldx, n_samples, channels, frames, spec, ld_spec, false,
                       (hipStream_t)stream);
}

pv_status pv_resynthesis(pv_handle* h, const pv_float2* spec, long long ld_spec, int channels,
                         int frames, const float* ola_in, long long ld_ola, float* out,
                         long long ldo, void* stream) {
    pv_status st = check_common(h, channels, frames);
    if (st != PV_OK) return st;
    DeviceGuard g(h->cfg.device);
    ProfCall pc_(h);
    return do_resynthesis(h, spec, ld_spec, channels, frames, ola_in, ld_ola, out, ldo, false,
                          (hipStream_t)stream);
}

int pv_segment_summary_words(const pv_handle* h) {
    return h ? pv::kSegFields * h->bins_pad : 0;
}

// run records of a spectrum (k_runsum, as pv_resynthesis makes them) -> the segment summary
pv_status pv_segment_summary(pv_handle* h, const pv_float2* spec, long long ld_spec, int channels,
                             int frames, int* summary, void* stream) {
    pv_status st = check_common(h, channels, frames);
    if (st != PV_OK) return st;
    if (h->mode != PV_MODE_STANDARD) return fail(PV_ERR_UNSUPPORTED, "pv_segment_summary: STANDARD handles only");
    if (channels == 0) return PV_OK;
    if (!summary) return fail(PV_ERR_ARG, "null summary");
    // (an empty segment has no first or last phase: the caller leaves it out of the order)
    if (frames == 0) return fail(PV_ERR_ARG, "pv_segment_summary: empty segment");
    if (!spec) return fail(PV_ERR_ARG, "null spec");
    if (ld_spec < (long long)frames * h->spec_stride) return fail(PV_ERR_ARG, "ld_spec < frames * spec_stride");
    DeviceGuard g(h->cfg.device);
    ProfCall pc_(h);
    hipStream_t s = (hipStream_t)stream;
    pv::ScanParams sc{};
    sc.spec = reinterpret_cast<const float2*>(spec);
    sc.ld_spec = ld_spec;
    sc.spec_stride = h->spec_stride;
    sc.frames = frames;
    sc.F = h->F;
    sc.nruns = nruns_of(h, frames);
    sc.L = h->L_syn;
    sc.bins_pad = h->bins_pad;
    sc.packed = h->packed;
    sc.ek = h->d_ek;
    sc.runsum = h->d_runsum;
    PV_LAUNCH(h, KRS, s, pv::launch_runsum(channels, sc, s));
    pv::SegParams sp{};
    sp.runsum = h->d_runsum;
    sp.nruns = sc.nruns;
    sp.L = h->L_syn;
    sp.bins_pad = h->bins_pad;
    sp.channels = channels;
    sp.ek = h->d_ek;
    sp.summary = summary;
    PV_LAUNCH(h, KRS, s, pv::launch_segsum(sp, s));
    return PV_OK;
}

pv_status pv_segment_resynthesis(pv_handle* h, const pv_float2* spec, long long ld_spec, int channels,
                                 int frames, long long frame0, const int* summaries, int seg, float* out,
                                 long long ldo, void* stream) {
    pv_status st = check_common(h, channels, frames);
    if (st != PV_OK) return st;
    if (frame0 < 0 || seg < 0) return fail(PV_ERR_ARG, "negative frame0 / seg");
    if (seg > 0 && !summaries) return fail(PV_ERR_ARG, "null summaries");
    if (channels == 0 || frames == 0) return PV_OK;
    DeviceGuard g(h->cfg.device);
    ProfCall pc_(h);
    hipStream_t s = (hipStream_t)stream;
    if (h->mode != PV_MODE_STANDARD)  // no unwrap state: the segment is a plain resynthesis
        return do_resynthesis(h, spec, ld_spec, channels, frames, nullptr, 0, out, ldo, false, s);
    pv::SegParams sp{};
    sp.L = h->L_syn;
    sp.bins_pad = h->bins_pad;
    sp.channels = channels;
    sp.ek = h->d_ek;
    sp.summaries = summaries;
    sp.seg = seg;
    sp.carry_in = h->d_seg_carry;
    sp.phi_in = h->d_seg_phi;
    PV_LAUNCH(h, KC, s, pv::launch_segcarry(sp, s));
    const SegState ss{h->d_seg_carry, h->d_seg_phi, (unsigned)((unsigned long long)frame0 % h->q)};
    return do_resynthesis(h, spec, ld_spec, channels, frames, nullptr, 0, out, ldo, false, s, nullptr,
                          /*force_scan*/ false, &ss);
}

// the handle's own spectrum rows (split path, pv_process with spec = NULL): allocated and
// zeroed once, under the handle's lock, so two threads' first calls allocate one buffer
static pv_status reserve_spec_own(pv_handle* h) {
    std::lock_guard<std::mutex> lk(h->spec_mu);
    if (h->d_spec_own) return PV_OK;
    const size_t bytes = sizeof(pv_float2) * (size_t)h->cfg.max_channels * (size_t)h->cfg.max_frames *
                         (size_t)h->spec_stride;
    pv_float2* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return fail(PV_ERR_NOMEM, "spectrum rows of a spec = NULL call");
    // (synchronised: the caller's stream may be a non-blocking one, which the null stream's
    // memset would not order before the first analysis)
    if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(p);
        return fail(PV_ERR_HIP, "zeroing the spectrum rows of a spec = NULL call");
    }
    h->d_spec_own = p;
    return PV_OK;
}

pv_status pv_reserve_spectrum(pv_handle* h) {
    if (!h) return fail(PV_ERR_ARG, "null handle");
    DeviceGuard g(h->cfg.device);
    if (h->F_fused > 0) return PV_OK;  // the single launch keeps a spec = NULL spectrum on chip
    return reserve_spec_own(h);
}

pv_status pv_process(pv_handle* h, const float* x, long long ldx, long long n_samples,
                     int channels, int frames, pv_float2* spec, long long ld_spec, float* out,
                     long long ldo, void* stream) {
    pv_status st = check_common(h, channels, frames);
    if (st != PV_OK) return st;
    DeviceGuard g(h->cfg.device);
    ProfCall pc_(h);
    hipStream_t s = (hipStream_t)stream;
    if (h->F_fused > 0) return do_fused(h, x, ldx, n_samples, channels, frames, spec, ld_spec, out, ldo, s);
    // spec == NULL: the rows go through the handle's own buffer, and bins no output bin reads
    // (pitch > 1) are not analysed
    int src_hi = -1;
    if (!spec && channels > 0 && frames > 0) {
        bool have;
        {
            std::lock_guard<std::mutex> lk(h->spec_mu);
            have = h->d_spec_own != nullptr;
        }
        if (!have) {
            // an allocation cannot be captured: under capture the rows must exist already
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
                return fail(PV_ERR_ARG, "pv_process(spec = NULL) under stream capture: call pv_reserve_spectrum first");
            if ((st = reserve_spec_own(h)) != PV_OK) return st;
        }
        spec = h->d_spec_own;
        ld_spec = (long long)h->cfg.max_frames * h->spec_stride;
        if (h->mode == PV_MODE_STANDARD) src_hi = h->src_hi;
    }
    const bool std_mode = (h->mode == PV_MODE_STANDARD) && h->q > 1;  // run records feed the scan
    st = do_analysis(h, x, ldx, n_samples, channels, frames, spec, ld_spec, std_mode, s, src_hi);
    if (st != PV_OK) return st;
    // (single-source pitch: the synthesis reads only the row slots of bins <= src_hi, the
    // ones the analysis wrote, k_synthesis NR)
    return do_resynthesis(h, spec, ld_spec, channels, frames, nullptr, 0, out, ldo, std_mode, s);
}

}  // extern "C"

namespace {
struct TableBlobHeader {
    uint32_t magic, version;
    int32_t n_samps, hop, hs, mode, effect, pitch;
    float scale;
    int32_t L_ana, L_syn, bins;
    uint32_t pad[4];
};
static_assert(sizeof(TableBlobHeader) == 64, "blob header is 64 bytes");
constexpr uint32_t kBlobMagic = 0x50565442u;  // "PVTB"

struct TableSeg {
    void* ptr;
    size_t bytes;
};
std::vector<TableSeg> table_segments(const pv_handle* h) {
    const size_t N = h->N, B = h->bins;
    return {{h->d_win, sizeof(float) * N},
            {h->d_gain, sizeof(float) * N},
            {h->d_tw_ana, sizeof(float2) * h->L_ana},
            {h->d_tws_ana, sizeof(float2) * (h->L_ana + 1)},
            {h->d_tw_syn, sizeof(float2) * tw_syn_len(h->L_syn)},
            {h->d_tws_syn, sizeof(float2) * (N / 2 + 1)},
            {h->d_ek, sizeof(float) * B},
            {h->d_jk_mod, sizeof(unsigned) * B},
            {h->d_src_first, sizeof(int) * B},
            {h->d_src_cnt, sizeof(int) * B}};
}
TableBlobHeader blob_header(const pv_handle* h) {
    TableBlobHeader hd{};
    hd.magic = kBlobMagic;
    hd.version = 2;  // 2: the L/2 synthesis table only at L = 256, 512 (tw_syn_len)
    hd.n_samps = h->N;
    hd.hop = h->hop;
    hd.hs = h->hs;
    hd.mode = h->mode;
    hd.effect = h->effect;
    hd.pitch = h->pitch;
    hd.scale = h->scale;
    hd.L_ana = h->L_ana;
    hd.L_syn = h->L_syn;
    hd.bins = h->bins;
    return hd;
}
size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }
}  // namespace

extern "C" {

pv_status pv_export_tables(const pv_handle* h, void* dst, size_t cap, size_t* bytes, void* stream) {
    if (!h || !bytes) return fail(PV_ERR_ARG, "null argument");
    if (dst && !h->tables_ready) return fail(PV_ERR_ARG, "tables_external handle: no tables to export yet");
    size_t total = sizeof(TableBlobHeader);
    for (const auto& sg : table_segments(h)) total += align16(sg.bytes);
    *bytes = total;
    if (!dst) return PV_OK;
    if (cap < total) return fail(PV_ERR_ARG, "export buffer too small");
    DeviceGuard g(h->cfg.device);
    hipStream_t s = (hipStream_t)stream;
    static thread_local TableBlobHeader hd;  // host source must outlive the async copy
    hd = blob_header(h);
    PV_HIP(hipMemcpyAsync(dst, &hd, sizeof(hd), hipMemcpyHostToDevice, s));
    size_t off = sizeof(TableBlobHeader);
    for (const auto& sg : table_segments(h)) {
        PV_HIP(hipMemcpyAsync((char*)dst + off, sg.ptr, sg.bytes, hipMemcpyDeviceToDevice, s));
        off += align16(sg.bytes);
    }
    PV_HIP(hipStreamSynchronize(s));
    return PV_OK;
}

pv_status pv_import_tables(pv_handle* h, const void* src, size_t bytes, void* stream) {
    if (!h || !src) return fail(PV_ERR_ARG, "null argument");
    size_t total = 0;
    pv_export_tables(h, nullptr, 0, &total, nullptr);
    if (bytes != total) return fail(PV_ERR_ARG, "table blob size does not match this handle");
    DeviceGuard g(h->cfg.device);
    hipStream_t s = (hipStream_t)stream;
    TableBlobHeader hd{};
    PV_HIP(hipMemcpyAsync(&hd, src, sizeof(hd), hipMemcpyDeviceToHost, s));
    PV_HIP(hipStreamSynchronize(s));
    TableBlobHeader mine = blob_header(h);
    if (std::memcmp(&hd, &mine, sizeof(hd)) != 0)
        return fail(PV_ERR_ARG, "table blob was built for a different configuration");
    size_t off = sizeof(TableBlobHeader);
    for (const auto& sg : table_segments(h)) {
        PV_HIP(hipMemcpyAsync(sg.ptr, (const char*)src + off, sg.bytes, hipMemcpyDeviceToDevice, s));
        off += align16(sg.bytes);
    }
    PV_HIP(hipStreamSynchronize(s));
    h->tables_ready = 1;
    return PV_OK;
}

pv_status pv_set_window(pv_handle* h, const float* win, void* stream) {
    if (!h || !win) return fail(PV_ERR_ARG, "null argument");
    if (h->mode != PV_MODE_REF_COMPAT)
        return fail(PV_ERR_UNSUPPORTED, "pv_set_window: REF_COMPAT handles only");
    DeviceGuard g(h->cfg.device);
    hipError_t e = pv::launch_window_gain(win, h->d_win, h->d_gain, h->N, (hipStream_t)stream);
    if (e != hipSuccess) return fail(PV_ERR_HIP, std::string("pv_set_window: ") + hipGetErrorString(e));
    return PV_OK;
}

pv_status pv_test_overlap_add(const float* in, const float* win, const float* back, float* out,
                              int n, int hop, void* stream) {
    if (!in || !win || !back || !out || n <= 0 || hop < 0) return fail(PV_ERR_ARG, "bad argument");
    hipError_t e = pv::launch_overlap_test(in, win, back, out, n, hop, (hipStream_t)stream);
    if (e != hipSuccess) return fail(PV_ERR_HIP, std::string("test_overlap_add: ") + hipGetErrorString(e));
    return PV_OK;
}

pv_status pv_profile_enable(pv_handle* h, int enable) {
    if (!h) return fail(PV_ERR_ARG, "null handle");
    if (enable < 0) return fail(PV_ERR_ARG, "negative profile stride");
    h->prof.enabled = enable != 0;
    h->prof.stride = enable > 1 ? enable : 1;
    h->prof.calls = 0;
    h->prof.active = true;
    if (h->prof.enabled) {  // events for the first launches, created here, not per launch
        DeviceGuard g(h->cfg.device);
        while (h->prof.pool.size() < 512) {
            hipEvent_t e;
            PV_HIP(hipEventCreate(&e));
            h->prof.pool.push_back(e);
        }
    }
    return PV_OK;
}

int pv_profile_read(pv_handle* h, const char** names, double* total_ms, int* launches, int cap) {
    if (!h) return 0;
    DeviceGuard g(h->cfg.device);
    for (size_t i = 0; i < h->prof.ev_start.size(); ++i) {
        float ms = 0.f;
        if (hipEventSynchronize(h->prof.ev_stop[i]) == hipSuccess &&
            hipEventElapsedTime(&ms, h->prof.ev_start[i], h->prof.ev_stop[i]) == hipSuccess) {
            h->prof.total_ms[h->prof.ev_kernel[i]] += ms;
            h->prof.launches[h->prof.ev_kernel[i]] += 1;
        }
        if (!h->prof.ev_shared[i]) h->prof.pool.push_back(h->prof.ev_start[i]);
        h->prof.pool.push_back(h->prof.ev_stop[i]);
    }
    h->prof.ev_start.clear();
    h->prof.ev_stop.clear();
    h->prof.ev_shared.clear();
    h->prof.ev_kernel.clear();
    h->prof.chain_ev = nullptr;
    int n = 0;
    for (int k = 0; k < kNumKernels && n < cap; ++k) {
        if (h->prof.launches[k] == 0) continue;
        if (names) names[n] = kKernelNames[k];
        if (total_ms) total_ms[n] = h->prof.total_ms[k];
        if (launches) launches[n] = h->prof.launches[k];
        ++n;
    }
    return n;
}

void pv_profile_reset(pv_handle* h) {
    if (!h) return;
    (void)pv_profile_read(h, nullptr, nullptr, nullptr, 0);
    for (int k = 0; k < kNumKernels; ++k) {
        h->prof.total_ms[k] = 0;
        h->prof.launches[k] = 0;
    }
}

}  // extern "C"

// ---------------------------------------------------------------- real-time mode
// pv_rt: a pv_handle (tables) + per-channel stream state + an optional captured graph
// of one callback (pinned host in -> device -> pv_rt_push -> pinned host out).
struct pv_rt {
    pv_handle* h = nullptr;
    int channels = 0;
    float *d_hist = nullptr, *d_ola = nullptr, *d_phprev = nullptr;
    int* d_M = nullptr;
    unsigned* d_tcount = nullptr;
    // captured callback
    int g_nframes = 0;
    float *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
    hipStream_t g_stream = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    float *m_in = nullptr, *m_out = nullptr;  // device views of h_in / h_out (zero-copy)
    int direct = 0;  // PV_RT_LAUNCH=direct: launch pv_rt_push per callback instead of replaying
                     // the captured graph (BASELINE config 5's form, the default): measured p50
                     // 21 vs 28 us per callback on ROCm 7.2
};

namespace {
void rt_release_graph(pv_rt* rt) {
    if (rt->exec) (void)hipGraphExecDestroy(rt->exec);
    if (rt->graph) (void)hipGraphDestroy(rt->graph);
    if (rt->h_in) (void)hipHostFree(rt->h_in);
    if (rt->h_out) (void)hipHostFree(rt->h_out);
    if (rt->d_in) (void)hipFree(rt->d_in);
    if (rt->d_out) (void)hipFree(rt->d_out);
    rt->exec = nullptr;
    rt->graph = nullptr;
    rt->h_in = rt->h_out = rt->d_in = rt->d_out = nullptr;
    rt->g_nframes = 0;
}
}  // namespace

extern "C" {

void pv_rt_destroy(pv_rt* rt) {
    if (!rt) return;
    if (rt->h) {
        DeviceGuard g(rt->h->cfg.device);
        rt_release_graph(rt);
        if (rt->g_stream) (void)hipStreamDestroy(rt->g_stream);
        void* ptrs[] = {rt->d_hist, rt->d_ola, rt->d_phprev, rt->d_M, rt->d_tcount};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        pv_destroy(rt->h);
    }
    delete rt;
}

pv_status pv_rt_reset(pv_rt* rt, void* stream) {
    if (!rt) return fail(PV_ERR_ARG, "null rt");
    DeviceGuard g(rt->h->cfg.device);
    hipStream_t s = (hipStream_t)stream;
    const size_t C = (size_t)rt->channels, N = rt->h->N, BP = rt->h->bins_pad;
    PV_HIP(hipMemsetAsync(rt->d_hist, 0, sizeof(float) * C * N, s));
    PV_HIP(hipMemsetAsync(rt->d_ola, 0, sizeof(float) * C * N, s));
    PV_HIP(hipMemsetAsync(rt->d_phprev, 0, sizeof(float) * C * BP, s));
    PV_HIP(hipMemsetAsync(rt->d_M, 0, sizeof(int) * C * BP, s));
    PV_HIP(hipMemsetAsync(rt->d_tcount, 0, sizeof(unsigned) * C, s));
    return PV_OK;
}

pv_status pv_rt_create(const pv_config* cfg, int channels, pv_rt** out) {
    if (!cfg || !out) return fail(PV_ERR_ARG, "null argument");
    // the version first: no other field of a caller's struct is read before it matches
    if (cfg->abi_version != PV_ABI_VERSION)
        return fail(PV_ERR_ARG, "pv_config.abi_version != PV_ABI_VERSION (caller built against another pv.h)");
    if (cfg->tables_external) return fail(PV_ERR_UNSUPPORTED, "tables_external: batch handles only");
    *out = nullptr;
    if (cfg->mode != PV_MODE_STANDARD)
        return fail(PV_ERR_UNSUPPORTED, "real-time mode runs the STANDARD pipeline only");
    if (cfg->spec_layout != PV_SPEC_NATURAL)
        return fail(PV_ERR_UNSUPPORTED, "real-time mode: natural spectrum rows only");
    if (channels <= 0) return fail(PV_ERR_ARG, "channels must be > 0");
    pv_config c = *cfg;
    c.max_channels = channels;
    c.max_frames = std::max(c.max_frames, 1);
    pv_rt* rt = new pv_rt();
    pv_status st = pv_create(&c, &rt->h);
    if (st != PV_OK) {
        delete rt;
        return st;
    }
    rt->channels = channels;
    if (pv::rt_lds_bytes(rt->h->L_syn) == 0) {
        pv_rt_destroy(rt);
        return fail(PV_ERR_UNSUPPORTED, "real-time mode: n_samps in [256, 2048]");
    }
    DeviceGuard g(cfg->device);
    const size_t C = (size_t)channels, N = rt->h->N, BP = rt->h->bins_pad;
    auto alloc = [&](void** p, size_t bytes) -> pv_status {
        hipError_t e = hipMalloc(p, bytes);
        if (e != hipSuccess) return fail(PV_ERR_NOMEM, std::string("pv_rt_create: ") + hipGetErrorString(e));
        return PV_OK;
    };
    if ((st = alloc((void**)&rt->d_hist, sizeof(float) * C * N)) != PV_OK ||
        (st = alloc((void**)&rt->d_ola, sizeof(float) * C * N)) != PV_OK ||
        (st = alloc((void**)&rt->d_phprev, sizeof(float) * C * BP)) != PV_OK ||
        (st = alloc((void**)&rt->d_M, sizeof(int) * C * BP)) != PV_OK ||
        (st = alloc((void**)&rt->d_tcount, sizeof(unsigned) * C)) != PV_OK) {
        pv_rt_destroy(rt);
        return st;
    }
    if ((st = pv_rt_reset(rt, nullptr)) != PV_OK || hipDeviceSynchronize() != hipSuccess) {
        pv_rt_destroy(rt);
        return st != PV_OK ? st : fail(PV_ERR_HIP, "pv_rt_create: reset failed");
    }
    *out = rt;
    return PV_OK;
}

pv_status pv_rt_push(pv_rt* rt, const float* in, long long ldi, int nframes, float* out,
                     long long ldo, pv_float2* spec, long long ld_spec, void* stream) {
    if (!rt) return fail(PV_ERR_ARG, "null rt");
    if (nframes < 0) return fail(PV_ERR_ARG, "negative nframes");
    if (nframes == 0) return PV_OK;
    pv_handle* h = rt->h;
    if (!in || !out) return fail(PV_ERR_ARG, "null in/out");
    if (rt->channels > 1 && (ldi < (long long)nframes * h->hop || ldo < (long long)nframes * h->hs))
        return fail(PV_ERR_ARG, "ldi/ldo smaller than one callback");
    if (spec && rt->channels > 1 && ld_spec < (long long)nframes * h->spec_stride)
        return fail(PV_ERR_ARG, "ld_spec < nframes * spec_stride");
    DeviceGuard g(h->cfg.device);
    pv::RtParams p{};
    p.in = in;
    p.ldi = ldi;
    p.out = out;
    p.ldo = ldo;
    p.spec = reinterpret_cast<float2*>(spec);
    p.ld_spec = ld_spec;
    p.spec_stride = h->spec_stride;
    p.channels = rt->channels;
    p.nframes = nframes;
    p.hop = h->hop;
    p.hs = h->hs;
    p.bins_pad = h->bins_pad;
    p.hist = rt->d_hist;
    p.ola = rt->d_ola;
    p.phprev = rt->d_phprev;
    p.M = rt->d_M;
    p.tcount = rt->d_tcount;
    p.win = h->d_win;
    p.gain = h->d_gain;
    p.tw = h->d_tw_syn;
    p.tws = h->d_tws_syn;
    p.ek = h->d_ek;
    p.jk_mod = h->d_jk_mod;
    p.src_first = h->d_src_first;
    p.src_cnt = h->d_src_cnt;
    p.rho = h->rho;
    p.p_mod = h->p_mod;
    p.q = h->q;
    p.q_pow2 = h->q_pow2;
    p.inv_q = h->inv_q;
    hipStream_t s = (hipStream_t)stream;
    prof_tick(h);  // one public call: the profile stride counts pv_rt_push calls too
    PV_LAUNCH(h, KRT, s, pv::launch_rt(h->L_syn, h->pitch ? 2 : 0, p, s));
    return PV_OK;
}

pv_status pv_rt_capture(pv_rt* rt, int nframes) {
    if (!rt) return fail(PV_ERR_ARG, "null rt");
    if (nframes <= 0) return fail(PV_ERR_ARG, "nframes must be > 0");
    pv_handle* h = rt->h;
    DeviceGuard g(h->cfg.device);
    rt_release_graph(rt);
    if (!rt->g_stream) PV_HIP(hipStreamCreateWithFlags(&rt->g_stream, hipStreamNonBlocking));
    const size_t C = (size_t)rt->channels;
    const size_t ni = (size_t)nframes * h->hop, no = (size_t)nframes * h->hs;
    // pinned, device-mapped host buffers: the captured kernel reads the callback's input
    // and writes its output in place over the bus (zero-copy: the graph is one kernel
    // node, no copy nodes); if the runtime cannot map them, the graph copies H2D / D2H
    // around the kernel instead
    PV_HIP(hipHostMalloc((void**)&rt->h_in, sizeof(float) * C * ni, hipHostMallocMapped));
    PV_HIP(hipHostMalloc((void**)&rt->h_out, sizeof(float) * C * no, hipHostMallocMapped));
    std::memset(rt->h_in, 0, sizeof(float) * C * ni);
    std::memset(rt->h_out, 0, sizeof(float) * C * no);
    float *m_in = nullptr, *m_out = nullptr;
    bool zero_copy = hipHostGetDevicePointer((void**)&m_in, rt->h_in, 0) == hipSuccess &&
                     hipHostGetDevicePointer((void**)&m_out, rt->h_out, 0) == hipSuccess && m_in && m_out;
    if (!zero_copy) {
        (void)hipGetLastError();
        PV_HIP(hipMalloc((void**)&rt->d_in, sizeof(float) * C * ni));
        PV_HIP(hipMalloc((void**)&rt->d_out, sizeof(float) * C * no));
    }
    const bool was_prof = h->prof.enabled;
    h->prof.enabled = false;  // no event records inside the graph
    hipStream_t s = rt->g_stream;
    PV_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    pv_status st = PV_OK;
    if (zero_copy) {
        st = pv_rt_push(rt, m_in, (long long)ni, nframes, m_out, (long long)no, nullptr, 0, s);
    } else {
        if (hipMemcpyAsync(rt->d_in, rt->h_in, sizeof(float) * C * ni, hipMemcpyHostToDevice, s) != hipSuccess)
            st = fail(PV_ERR_HIP, "pv_rt_capture: H2D capture failed");
        if (st == PV_OK)
            st = pv_rt_push(rt, rt->d_in, (long long)ni, nframes, rt->d_out, (long long)no, nullptr, 0, s);
        if (st == PV_OK &&
            hipMemcpyAsync(rt->h_out, rt->d_out, sizeof(float) * C * no, hipMemcpyDeviceToHost, s) != hipSuccess)
            st = fail(PV_ERR_HIP, "pv_rt_capture: D2H capture failed");
    }
    hipGraph_t graph = nullptr;
    hipError_t e = hipStreamEndCapture(s, &graph);
    h->prof.enabled = was_prof;
    if (st != PV_OK) {
        if (graph) (void)hipGraphDestroy(graph);
        return st;
    }
    if (e != hipSuccess) return fail(PV_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    rt->graph = graph;
    PV_HIP(hipGraphInstantiate(&rt->exec, graph, nullptr, nullptr, 0));
    rt->g_nframes = nframes;
    rt->m_in = zero_copy ? m_in : nullptr;
    rt->m_out = zero_copy ? m_out : nullptr;
    const char* lv = std::getenv("PV_RT_LAUNCH");
    rt->direct = (zero_copy && lv && std::string(lv) == "direct") ? 1 : 0;
    return PV_OK;
}

pv_status pv_rt_host_buffers(pv_rt* rt, float** host_in, float** host_out) {
    if (!rt || !rt->exec) return fail(PV_ERR_ARG, "no captured callback (pv_rt_capture)");
    if (host_in) *host_in = rt->h_in;
    if (host_out) *host_out = rt->h_out;
    return PV_OK;
}

pv_status pv_rt_callback(pv_rt* rt, const float* in, float* out) {
    if (!rt || !rt->exec) return fail(PV_ERR_ARG, "no captured callback (pv_rt_capture)");
    pv_handle* h = rt->h;
    DeviceGuard g(h->cfg.device);
    const size_t C = (size_t)rt->channels;
    const size_t ni = (size_t)rt->g_nframes * h->hop, no = (size_t)rt->g_nframes * h->hs;
    if (in && in != rt->h_in) std::memcpy(rt->h_in, in, sizeof(float) * C * ni);  // main.cpp:49
    if (rt->direct) {
        pv_status st = pv_rt_push(rt, rt->m_in, (long long)ni, rt->g_nframes, rt->m_out, (long long)no, nullptr, 0,
                                  rt->g_stream);
        if (st != PV_OK) return st;
    } else {
        PV_HIP(hipGraphLaunch(rt->exec, rt->g_stream));
    }
    PV_HIP(hipStreamSynchronize(rt->g_stream));
    if (out && out != rt->h_out) std::memcpy(out, rt->h_out, sizeof(float) * C * no);
    return PV_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- standalone FFT
namespace {
std::mutex g_fft_mu;
std::map<std::pair<int, int>, float2*> g_fft_tw;  // (device, n) -> stage-major twiddles
}  // namespace

extern "C" pv_status pv_fft_c2c(const pv_float2* in, pv_float2* out, int n, int batch, int inverse,
                                void* stream) {
    if (!in || !out) return fail(PV_ERR_ARG, "null in/out");
    if (batch < 0) return fail(PV_ERR_ARG, "negative batch");
    if (!is_pow2(n) || n < 2 || n > 2048) return fail(PV_ERR_UNSUPPORTED, "fft size: power of two in [2, 2048]");
    if (batch == 0) return PV_OK;
    int dev = 0;
    PV_HIP(hipGetDevice(&dev));
    float2* tw = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_fft_mu);
        auto it = g_fft_tw.find({dev, n});
        if (it == g_fft_tw.end()) {
            std::vector<float2> t;
            fft_table(n, t);
            pv_status st = upload(&tw, t);
            if (st != PV_OK) return st;
            g_fft_tw[{dev, n}] = tw;
        } else {
            tw = it->second;
        }
    }
    hipError_t e = pv::launch_fft(n, inverse ? 1 : 0, reinterpret_cast<const float2*>(in),
                                  reinterpret_cast<float2*>(out), tw, batch, (hipStream_t)stream);
    if (e != hipSuccess) return fail(PV_ERR_HIP, std::string("fft launch: ") + hipGetErrorString(e));
    return PV_OK;
}

// ---------------------------------------------------------------- harmoniser
// README.md:50 "harmonization of input signals (i.e. multiple pitch shifts on a single
// input)": one analysis + one unwrap scan, then one synthesis per voice (its own pitch
// map and output-phase ratio), optionally mixed.
struct pv_harmonizer {
    std::vector<pv_handle*> voices;
};

extern "C" {

void pv_harmonizer_destroy(pv_harmonizer* hz) {
    if (!hz) return;
    for (pv_handle* v : hz->voices) pv_destroy(v);
    delete hz;
}

pv_status pv_harmonizer_create(const pv_config* cfg, const float* ratios, int voices, pv_harmonizer** out) {
    if (!cfg || !ratios || !out) return fail(PV_ERR_ARG, "null argument");
    // the version first: no other field of a caller's struct is read before it matches
    if (cfg->abi_version != PV_ABI_VERSION)
        return fail(PV_ERR_ARG, "pv_config.abi_version != PV_ABI_VERSION (caller built against another pv.h)");
    if (cfg->tables_external) return fail(PV_ERR_UNSUPPORTED, "tables_external: batch handles only");
    *out = nullptr;
    if (voices <= 0 || voices > 64) return fail(PV_ERR_ARG, "voices must be in [1, 64]");
    if (cfg->mode != PV_MODE_STANDARD) return fail(PV_ERR_UNSUPPORTED, "the harmoniser runs the STANDARD pipeline");
    pv_harmonizer* hz = new pv_harmonizer();
    for (int k = 0; k < voices; ++k) {
        pv_config c = *cfg;
        c.effect = PV_PITCH_SHIFT;
        c.scale = ratios[k];
        pv_handle* h = nullptr;
        pv_status st = pv_create(&c, &h);
        if (st != PV_OK) {
            pv_harmonizer_destroy(hz);
            return st;
        }
        hz->voices.push_back(h);
    }
    *out = hz;
    return PV_OK;
}

pv_status pv_harmonize(pv_harmonizer* hz, const float* x, long long ldx, long long n_samples,
                       int channels, int frames, pv_float2* spec, long long ld_spec, float* voices_out,
                       long long ldo, long long ld_voice, const float* gains, float* mix,
                       long long ld_mix, void* stream) {
    if (!hz || hz->voices.empty()) return fail(PV_ERR_ARG, "null harmoniser");
    pv_handle* h0 = hz->voices[0];
    pv_status st = check_common(h0, channels, frames);
    if (st != PV_OK) return st;
    if (mix && !gains) return fail(PV_ERR_ARG, "mix needs gains");
    if (channels == 0 || frames == 0) return PV_OK;  // nothing to do (as pv_process)
    if (!voices_out) return fail(PV_ERR_ARG, "null voices_out");
    const int K = (int)hz->voices.size();
    const long long olen = pv_output_length(h0, frames);
    if (K > 1 && ld_voice < (long long)(channels - 1) * ldo + olen)
        return fail(PV_ERR_ARG, "ld_voice smaller than one voice's output block");
    DeviceGuard g(h0->cfg.device);
    hipStream_t s = (hipStream_t)stream;
    st = do_analysis(h0, x, ldx, n_samples, channels, frames, spec, ld_spec, true, s);
    if (st != PV_OK) return st;
    st = do_resynthesis(h0, spec, ld_spec, channels, frames, nullptr, 0, voices_out, ldo, true, s,
                        nullptr, /*force_scan: other voices read h0's carries*/ true);
    if (st != PV_OK) return st;
    for (int k = 1; k < K; ++k) {
        st = do_resynthesis(hz->voices[k], spec, ld_spec, channels, frames, nullptr, 0,
                            voices_out + (long long)k * ld_voice, ldo, true, s, h0->d_carry);
        if (st != PV_OK) return st;
    }
    if (mix && channels > 0 && frames > 0) {
        if (K > 64) return fail(PV_ERR_ARG, "too many voices to mix");
        pv::MixParams mp{};
        mp.src = voices_out;
        mp.ldo = ldo;
        mp.ld_voice = ld_voice;
        mp.voices = K;
        for (int k = 0; k < K; ++k) mp.gain[k] = gains[k];
        mp.dst = mix;
        mp.ld_mix = ld_mix;
        mp.len = olen;
        mp.channels = channels;
        hipError_t e = pv::launch_mix(mp, s);
        if (e != hipSuccess) return fail(PV_ERR_HIP, std::string("mix launch: ") + hipGetErrorString(e));
    }
    return PV_OK;
}

}  // extern "C"
