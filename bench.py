#!/usr/bin/env python3
"""bench.py — STFT frames/s of the MI355X phase-vocoder hot path.

Workload (BASELINE.json configs[2], the batched throughput configuration at the metric's
N=1024 / hop=256): per GPU 1024 synthetic 44.1 kHz mono channels x 10 s (441 000
samples, 1722 frames each), PV_STANDARD time-stretch 0.5 (out hop 128).  A "step" is one
pass of the hot path (analysis -> phase processing -> resynthesis + overlap-add, libpv
pv_process) over that batch, with the input resident in HBM.  Channels shard across
ranks with no data-path collective (weak scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--channels C] [--no-cpu]
  torchrun --nproc-per-node N bench.py --gpus N ...       (one process per GPU, RCCL)

`--gpus N` without a launcher starts the N rank processes itself (launch_ranks); with one
(WORLD_SIZE set) it must equal WORLD_SIZE.  PV_DIST_BACKEND=gloo runs the same N-rank path
over gloo (collectives on host tensors) — how the one-GPU box rehearses it.

The synthetic channels are generated once on the host and uploaded; after the timed
steps the whole output is checked for finiteness and 16 channels spread over the batch
(first and last included) are compared with the CPU oracle (`rms_vs_oracle`, bar 1e-5
RMS per sample), and the CPU baseline is timed on a bounded prefix of the same channels.

Rank 0 prints ONE JSON line (metric, value, roofline{...}, rms_vs_oracle{...},
cpu_baseline{...}, ...).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "phase-vocoder_amd"))

METRIC = "STFT frames/s @ N=1024,hop=256; % HBM roofline; RMS err vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SR = 44100


def cpu_share():
    """(threads the CPU legs use, CPUs in this process's affinity mask).  On the GPU pool
    `nproc`/os.cpu_count() show the whole machine while one GPU's share is 16 CPUs
    (OMP_NUM_THREADS is set to it there), so the share is min(affinity, OMP_NUM_THREADS);
    PV_CPU_THREADS overrides."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = min(aff, omp) if omp > 0 else aff
    return int(os.environ.get("PV_CPU_THREADS", "0") or 0) or share, aff


def _synth_one(c, n, seed0, out):
    t = np.arange(n) / SR
    rng = np.random.default_rng(seed0 + c)
    f = rng.uniform(55, 4000, 3)
    ph = rng.uniform(0, 2 * np.pi, 3)
    acc = sum(0.1 * np.sin(2 * np.pi * f[i] * t + ph[i]) for i in range(3))
    acc = acc + rng.uniform(-1e-3, 1e-3, n)
    out[c] = acc.astype(np.float32)


def synth_channels_np(C, n, seed0, threads=1):
    """configs 2-4 generator: 3 sines f~U[55,4000] Hz, a=0.1, random
    phase, + U(+-1e-3) noise, seed = seed0 + channel.  Built once on the host: the GPU
    batch, the CPU baseline and the oracle check all read this same array."""
    out = np.empty((C, n), np.float32)
    if threads <= 1 or C == 1:
        for c in range(C):
            _synth_one(c, n, seed0, out)
    else:
        from concurrent.futures import ThreadPoolExecutor  # numpy ufuncs release the GIL
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda c: _synth_one(c, n, seed0, out), range(C)))
    return out


def _pvref():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pvref  # test infrastructure: the timed CPU baseline and the checker, never the product
    return pvref


def _oracle_batch(pvref, compat):
    """The oracle's batched path (the checker): (x, N, hop_div, effect, scale, frames,
    threads) -> (out, threads used).  REF_COMPAT: the fp64 restatement of kernel.cu /
    main.cpp; STANDARD: the fp32-contract analysis + fp64 textbook synthesis."""
    if compat:
        return lambda x, N, hd, e, s, fr, th: pvref.compat_process_batch(x, N, hd, fr, th)
    return pvref.std_process_batch


def _port_batch(pvref, compat):
    """What cpu_baseline times: the fp32 CPU ports (oracle/pvport.c, OpenMP over channels).
    STANDARD — the contract's fp32 analysis, the integer phase scan, fp32 sin/cos, fp32
    inverse FFT and overlap-add; REF_COMPAT — kernel.cu's path in fp32 (2N-point real FFT,
    sqrtf / atanf, the y-bug, N-point C2R, /N, swap, window, overlap-add)."""
    if compat:
        return lambda x, N, hd, e, s, fr, th: pvref.port_compat_process_batch(x, N, hd, fr, th)
    return pvref.port_std_process_batch


def cpu_baseline(x, N, hop_div, effect, scale, target_s=10.0, single=False, compat=False):
    """The fp32 CPU port (oracle/pvport.c, STANDARD or REF_COMPAT; OpenMP over channels)
    timed on a bounded sample of
    the SAME host channels the GPU processes (x: [C, n] float32).  A single stream
    (single=True) has no channel parallelism and runs on one core."""
    pvref = _pvref()
    batch = _port_batch(pvref, compat)
    what = ("oracle/pvport.c REF_COMPAT fp32 CPU port" if compat
            else "oracle/pvport.c fp32 CPU port")
    threads, aff = cpu_share()
    C_all, n = x.shape
    frames = pvref.num_frames(n, N // hop_div)
    host = f"{threads} threads = this process's CPU share (affinity {aff}, machine {os.cpu_count()})"
    note = ("fp32 end to end: kernel.cu's path as a CPU port (Hamming window, shift + pad, the "
            "2N-point real FFT, sqrtf / atanf(y/x) over all 2N bins, the y-bug, N-point C2R, /N, "
            "swap halves, window, overlap-add); gcc -O3 -march=x86-64-v3, OpenMP over channels "
            "(pinned to the fp64 restatement <= 1e-6 RMS, tests/test_oracle.py)" if compat else
            "fp32 end to end: the fp32-contract analysis (the GPU's own phases), the integer "
            "phase scan, fp32 sin/cos, fp32 inverse real FFT and overlap-add; gcc -O3 "
            "-march=x86-64-v3, OpenMP over channels (pinned to the fp64 oracle <= 1e-6 RMS, "
            "tests/test_oracle.py)")
    if single:
        t0 = time.perf_counter()
        _, used = batch(x[:1], N, hop_div, effect, scale, frames, 1)
        dt = time.perf_counter() - t0
        # the whole stream takes well under a second: repeat it to ~target_s of CPU work
        reps = max(1, min(100, int(target_s / max(dt, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(reps):
            _, used = batch(x[:1], N, hop_div, effect, scale, frames, 1)
        dt = time.perf_counter() - t0
        return {"value": reps * frames / dt, "unit": "frames/s", "cores": int(used), "kind": "port",
                "sample": f"the whole stream ({n} samples, {frames} frames) x {reps} on 1 core, "
                          f"{what}, {dt:.1f} s wall", "note": note}
    k = min(threads, C_all)
    t0 = time.perf_counter()
    _, used = batch(x[:k], N, hop_div, effect, scale, frames, threads)
    dt = time.perf_counter() - t0
    rate = k * frames / dt
    C = max(k, int(rate * target_s / frames) // threads * threads)
    C = min(C, C_all)
    t0 = time.perf_counter()
    _, used = batch(x[:C], N, hop_div, effect, scale, frames, threads)
    dt = time.perf_counter() - t0
    return {"value": C * frames / dt, "unit": "frames/s", "cores": int(used), "kind": "port",
            "sample": f"channels 0..{C - 1} of the GPU batch x {n} samples ({C * frames} frames), "
                      f"{what}, {dt:.1f} s wall; "
                      f"{host}", "note": note}


def check_channels(C, k=16):
    """k channel indices spread over the batch, first and last included."""
    return sorted(set(int(round(v)) for v in np.linspace(0, C - 1, min(k, C))))


def oracle_check(x, out_rows, idx, N, hop_div, effect, scale, frames, all_finite, compat=False):
    """RMS per sample of the GPU output against the oracle on the sampled channels of
    the timed batch (BASELINE.json metric: "RMS err vs CPU ref"; bar 1e-5)."""
    pvref = _pvref()
    threads, _ = cpu_share()
    ref, _ = _oracle_batch(pvref, compat)(x[idx], N, hop_div, effect, scale, frames, threads)
    got = out_rows[:, :ref.shape[1]]
    rms = np.sqrt(np.mean((got.astype(np.float64) - ref) ** 2, axis=1))
    return {"max": float(rms.max()), "mean": float(rms.mean()), "tol": 1e-5,
            "pass": bool(rms.max() <= 1e-5 and all_finite), "channels": idx,
            "all_finite": bool(all_finite),
            "oracle": ("oracle/pvref.c pvr_compat_process_batch (fp64 restatement of kernel.cu / main.cpp)"
                       if compat else
                       "oracle/pvref.c pvr_std_process_batch (fp32-contract analysis, fp64 synthesis)")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 10; 200 for the 50-us c2 step, 2000 callbacks for rt)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 3; 20 for c2)")
    ap.add_argument("--channels", type=int, default=1024, help="channels per GPU")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--prof-every", type=int, default=None,
                    help="per-kernel hipEvents on every k-th timed step (default 1; a "
                         "single-launch step is timed as one block instead)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the timed CPU baseline")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the oracle check of the timed batch (profiling passes only)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--write-spec", action="store_true",
                    help="hand the spectrum rows back to the caller (by default STANDARD runs do not: "
                         "the single launch keeps them on chip, SURVEY §8(d) fused mode; the split "
                         "path still round-trips every row through HBM)")
    ap.add_argument("--layout", choices=["packed", "natural"], default="packed",
                    help="STANDARD spectrum rows of the pv_process workspace (include/pv.h "
                         "pv_spec_layout): packed (default) folds the real bin N/2 into slot 0 "
                         "so every row store is whole 64-byte segments")
    ap.add_argument("--workload", choices=["c3", "c2", "c4", "compat", "rt", "batch"], default="c3",
                    help="c3 (= batch): configs[2], the headline line (default); c2: configs[1] "
                         "single 60 s stream, pitch 2.0; c4: configs[3] per-GPU slice (1024 ch, "
                         "N=2048 hop=512, pitch 1.5); compat: the reference's own path (REF_COMPAT) "
                         "at configs[2]'s size; rt: configs[4] real-time mode")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.workload == "rt" and args.gpus > 1:
        raise SystemExit("bench.py: the real-time workload runs on one GPU (--gpus 1)")
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} "
                             "(one rank per GPU: the two must agree)")
    elif args.gpus > 1:
        # no launcher: start one rank process per GPU here, before anything touches the GPU
        return launch_ranks(args.gpus)
    # a c2 step is ~50 us: 10 steps would time the barrier/synchronise bracket, not the path
    if args.steps is None:
        args.steps = 200 if args.workload == "c2" else 10
    if args.warmup is None:
        args.warmup = 20 if args.workload == "c2" else 3
    if args.workload == "rt":
        return bench_rt(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; more ranks than GPUs (the one-GPU rehearsal of the N-rank path,
    # PV_DIST_BACKEND=gloo) share the devices round-robin
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    backend = os.environ.get("PV_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI on ROCm
    # under torchrun (or launch_ranks) the process group is always formed, a single rank
    # included: the N = 1 torchrun run exercises the same RCCL init, table broadcast and
    # reductions as N = 8 (tests/test_gpu_bench_dist.py)
    distributed = world > 1 or ("MASTER_ADDR" in os.environ and "WORLD_SIZE" in os.environ)
    if distributed:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local}")
    # the device the few collectives of the bench (timing, check) run on
    cdev = dev if backend == "nccl" else torch.device("cpu")

    from pvamd import PITCH_SHIFT, REF_COMPAT, PhaseVocoder, STANDARD, TIME_SHIFT
    from pvamd._lib import PV_SPEC_NATURAL, PV_SPEC_PACKED, diagnostic_build, lib as _pvlib
    # the loaded library's source hash (pvamd._lib refuses one that is not this tree's)
    lib_sha = _pvlib().pv_sources_sha().decode()
    # a diagnostic build (timing-only ablations: wrong outputs) is for --no-check A/B runs only
    diag = diagnostic_build()
    if diag and not args.no_check:
        raise SystemExit("bench.py: libpv is a diagnostic build (PV_DIAGNOSTIC_BUILD): "
                         "timing-only, run it with --no-check")

    wl = "c3" if args.workload == "batch" else args.workload
    # (N, hop_div, effect, scale, seconds, channels per GPU, description)
    WL = {"c3": (1024, 4, TIME_SHIFT, 0.5, args.seconds, args.channels,
                 "BASELINE configs[2]: 1024 mono ch x 10 s per GPU, N=1024 hop=256, "
                 "PV_STANDARD time-stretch 0.5"),
          "c2": (1024, 4, PITCH_SHIFT, 2.0, 60.0, 1,
                 "BASELINE configs[1]: single mono 44.1 kHz stream x 60 s, N=1024 hop=256, "
                 "PV_STANDARD pitch 2.0"),
          "compat": (1024, 4, TIME_SHIFT, 1.0, args.seconds, args.channels,
                     "the reference's active path (REF_COMPAT: kernel.cu:299-348 analysis to 2N "
                     "{mag, atanf(Im/Re)} bins, kernel.cu:352-432 resynthesis, running OLA), "
                     "1024 mono ch x 10 s per GPU, N=1024 hop=256"),
          "c4": (2048, 4, PITCH_SHIFT, 1.5, args.seconds, args.channels,
                 "BASELINE configs[3] per-GPU slice: 1024 mono ch x 10 s per GPU, N=2048 hop=512, "
                 "PV_STANDARD pitch 1.5 (8192 ch on 8 GPUs)")}
    N, hop_div, effect, scale, seconds, C, wl_desc = WL[wl]
    n = int(round(seconds * SR))
    compat = wl == "compat"
    if compat:
        args.layout = "natural"  # REF_COMPAT rows: the 2N bins of kernel.cu:337
    layout = PV_SPEC_PACKED if args.layout == "packed" else PV_SPEC_NATURAL
    # under a process group only rank 0 builds the constant tables; the other ranks' handles
    # start without any (tables_external) and compute with what the broadcast delivers
    mk = dict(mode=REF_COMPAT if compat else STANDARD, device=local, spec_layout=layout)
    pv = PhaseVocoder(N, effect, scale, hop_div, max_channels=C, max_frames=pv_frames(n, N // hop_div),
                      tables_external=distributed and rank != 0, **mk)
    frames = pv.num_frames(n)
    tables = None
    if distributed:  # init-time RCCL broadcast of rank 0's tables (north_star); not timed
        from pvamd.dist import broadcast_tables
        # the check only: a one-frame handle built locally, compared with what arrived
        ref = PhaseVocoder(N, effect, scale, hop_div, max_channels=1, max_frames=1, **mk) if rank != 0 else None
        same = broadcast_tables(pv, src=0, local=ref)
        t_same = torch.tensor([0.0 if same else 1.0], dtype=torch.float64, device=cdev)
        dist.all_reduce(t_same, op=dist.ReduceOp.MAX)
        tables = {"bytes": pv.tables_bytes(), "built_on": "rank 0 only (the other ranks' handles: tables_external)",
                  "received_by_ranks": world - 1, "bit_identical_to_local": bool(t_same.item() == 0.0)}
        if ref is not None:
            ref.close()
    threads, _ = cpu_share()
    t_gen = time.perf_counter()
    x_host = synth_channels_np(C, n, 20240 + rank * C, threads)
    x = torch.from_numpy(x_host).to(dev)
    t_gen = time.perf_counter() - t_gen
    # STANDARD workloads do not hand the spectrum back (the reference's main.cpp never reads
    # it) unless --write-spec: the single launch (config 2) then consumes it on chip, the
    # split path still writes and re-reads every row (the handle's own buffer; for pitch > 1
    # the bins no output bin reads are neither analysed, written nor read back).
    # REF_COMPAT fills the caller's 2N-bin rows, as kernel.cu does.
    want_spec = args.write_spec or compat
    spec_on_chip = bool(pv.single_launch) and not want_spec
    spec = pv.alloc_spec(C, frames) if want_spec else None
    out = pv.alloc_out(C, frames)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        if distributed:
            dist.barrier()

    for _ in range(args.warmup):
        pv.process(x, spec=spec, out=out, spectrum=want_spec)
    torch.cuda.synchronize(dev)

    # kernel durations for the roofline, on the launch stream (pv launches on torch's current
    # stream).  A single-launch step (the q = 1 fused path, config 2) is timed as a block:
    # one event pair around the timed loop / steps (back-to-back launches, no gaps: the
    # rocprofv3 trace shows 0 us between them).  Otherwise libpv records an event pair around
    # every launch; each event record costs the queue ~5.6 us, nothing at ms-scale kernels
    # but 15 % of a 37-us one (and ~1 % of a 4-ms four-launch step, which keeps them on every
    # step so that every launch of the timed region is accounted for; --prof-every k samples
    # every k-th step instead).
    block = bool(pv.single_launch) and not args.prof_every
    prof_every = 0 if block else (args.prof_every or 1)
    pv.profile(prof_every)
    pv.profile_reset()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        pv.process(x, spec=spec, out=out, spectrum=want_spec)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0
    if block:
        prof = {"fused": (ev0.elapsed_time(ev1), args.steps)}
    else:
        prof = pv.profile_read()
    pv.profile(False)

    dt_t = torch.tensor([dt], dtype=torch.float64, device=cdev)
    if distributed:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_frames = C * frames * world * args.steps
    value = total_frames / dt

    hop_a, hop_s, B = N // hop_div, pv.outHopSize, pv.spec_bins
    # the row slots the analysis writes per frame: all of them, or — no spectrum handed back,
    # pitch > 1, L = 1024 (config 4) — only the lane registers holding a bin some output bin
    # reads (pv_analysis.hip NA instantiations: 64 NA slots).  The roofline counts those for
    # both halves — the bytes the algorithm moves; the synthesis loads the same slots
    # (k_synthesis NR: 12 of 16 registers for pitch 1.5)
    B_full = B
    if not want_spec and not compat and not pv.single_launch and effect == PITCH_SHIFT and scale > 1.0 \
            and N // 2 == 1024 and layout == PV_SPEC_PACKED and hop_a == 512:
        src_hi = max(k for k in range(N // 2 + 1) if math.floor(scale * k + 0.5) <= N // 2)
        B = min(B, 64 * 2 * ((src_hi + 128) // 128))
    dom = max(prof, key=lambda k: prof[k][0])
    ms_tot, launches = prof[dom]
    avg_ms = ms_tot / max(launches, 1)
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            # keyed per workload (and spectrum layout): no number for a workload not measured
            ent = tj.get(wl) if isinstance(tj.get(wl), dict) else (tj if tj.get("_workload", "c3") == wl else None)
            if ent is not None and ent.get("_layout", "natural") == args.layout:
                traffic = ent.get(dom, {}).get("bytes_per_launch")
        except Exception:
            traffic = None
    roof = roofline(dom, avg_ms, wl, N, hop_a, hop_s, B, C * frames, compat, traffic,
                    spec_written=not spec_on_chip)
    achieved = roof["achieved"]
    # the box's measured HBM ceilings: plain streams (scripts/bw_probe.hip ->
    # profiles/r02_bw_probe.jsonl: copy ~6.0, write ~6.0 TB/s against the 8 TB/s spec) and the
    # dominant kernel's own byte mix with no arithmetic, in the product's wave mapping and row
    # layout (scripts/layout_probe.hip -> profiles/r03_layout_probe.jsonl, config 3 only)
    ceiling = None
    try:
        rows = {}
        for f in ("r02_bw_probe.jsonl", "r03_layout_probe.jsonl"):
            for d in map(json.loads, open(os.path.join(ROOT, "profiles", f))):
                rows.setdefault(d["probe"], d["GBps"])
        copy = max(v for k, v in rows.items() if k.startswith("copy"))
        write = max(v for k, v in rows.items() if k.startswith("write"))
        ceiling = {"copy_GBps": copy, "write_GBps": write, "frac_of_copy": achieved / copy,
                   "traffic_frac_of_copy": (traffic / (avg_ms * 1e-3) / 1e9 / copy) if traffic else None,
                   "source": "profiles/r02_bw_probe.jsonl, profiles/r03_layout_probe.jsonl"}
        suffix = "512" if args.layout == "packed" else "520_L"
        pat = {"analysis": f"ana_cmaj_product_{suffix}", "synthesis": f"syn_cmaj_product_{suffix}"}.get(dom)
        if pat in rows and wl == "c3":
            ceiling.update(pattern=pat, pattern_GBps=rows[pat], frac_of_pattern=achieved / rows[pat])
    except Exception:
        ceiling = None
    kernels = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1]} for k, v in prof.items()}

    # parity of the timed batch: every sample finite, sampled channels vs the oracle
    check = None
    if not args.no_check:
        idx = check_channels(C)
        finite = bool(torch.isfinite(out).all().item())
        check = oracle_check(x_host, out[idx].cpu().numpy(), idx, N, hop_div, ord(effect), scale,
                             frames, finite, compat=compat)
        if distributed:  # worst rank
            t = torch.tensor([check["max"], check["mean"], 0.0 if check["pass"] else 1.0,
                              0.0 if finite else 1.0], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            check.update(max=float(t[0]), mean=float(t[1]), ranks=world,
                         channels=f"{len(idx)} per rank (indices as rank 0's, rank-local)")
            check["pass"] = bool(t[2] == 0)
            check["all_finite"] = bool(t[3] == 0)
    B_read = N // 2 + 1 if compat else B
    # HBM bytes of the whole path per frame: input and output samples, plus the spectrum row
    # written and re-read when it goes through HBM (the split path); a single launch that keeps
    # the spectrum on chip moves only the samples (SURVEY §8(d) fused-mode bytes)
    path_bpf = path_bytes_per_frame(hop_a, hop_s, B, B_read, spec_on_chip)
    path_bytes = path_bpf * C * frames * world * args.steps

    cpu = None
    # the CPU baseline is a rank-0, N = 1 figure (the contract's cpu_baseline): an N-rank run
    # reports null rather than time the host while the other ranks wait
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(x_host, N, hop_div, ord(effect), scale, single=(C == 1), compat=compat)
        except Exception as e:  # reported, never fatal for the GPU number
            cpu = {"value": None, "unit": "frames/s", "cores": 0, "kind": "port",
                   "sample": f"failed: {e}"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (3 sines U[55,4000] Hz a=0.1 + U(+-1e-3) noise, seed 20240+ch)",
            "config": {"workload": wl_desc,
                       "channels_per_gpu": C, "frames_per_channel": frames, "N": N, "hop": hop_a,
                       "out_hop": hop_s, "spec_layout": args.layout,
                       "spec_slots_carried": B, "spec_slots": B_full,
                       "spectrum": "kept on chip (single launch, SURVEY §8(d) fused mode)" if spec_on_chip
                                   else ("returned to the caller" if want_spec else
                                         "written to and re-read from HBM, not returned (the handle's own rows)"),
                       "parallelism": f"channel-shard x{world}",
                       "dist_backend": backend if distributed else None},
            "roofline": roof,
            "diagnostic_build": diag,
            "lib_sources_sha": lib_sha,
            "path_hbm_frac": path_bytes / dt / 1e9 / HBM_PEAK_GBS,
            "path_bytes_per_frame": path_bpf,
            "measured_ceiling": ceiling,
            "kernels": kernels,
            "kernel_timing": "block: one event pair around the timed loop" if block
                             else f"per-launch event pairs, every {prof_every}-th step",
            "tables_broadcast": tables,
            "rms_vs_oracle": check,
            "cpu_baseline": cpu,
            "host_gen_s": t_gen,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


VALU_PEAK_TFLOPS = 157.3   # MI355X FP32 vector (dense) peak, MI355X_MICROARCH.md
SIMDS = 1024               # 256 CUs x 4 SIMDs
PEAK_SCLK_GHZ = 2.4


def path_bytes_per_frame(hop_a, hop_s, B, B_read, spec_on_chip):
    """HBM bytes of the whole path per frame (the line's path_hbm_frac): the input and output
    samples, plus the spectrum row written (B slots) and re-read (B_read) when it goes
    through HBM; the single launch that keeps it on chip moves the samples only (SURVEY
    §8(d) fused-mode bytes)."""
    return 4 * hop_a + 4 * hop_s + (0 if spec_on_chip else 8 * B + 8 * B_read)


def alg_bytes_per_frame(kernel, N, hop_a, hop_s, B, compat, spec_written=True):
    """SURVEY §8(d) bytes per frame of each kernel: spectrum row = what the layout stores
    (8 (N/2+1) natural, 8 N/2 packed: bin N/2 rides in slot 0, the smaller figure);
    REF_COMPAT writes 2N bins per frame (kernel.cu:337) and its resynthesis reads the N/2+1
    of them its size-N C2R uses (kernel.cu:363-368)."""
    B_read = N // 2 + 1 if compat else B
    return {"analysis": 4 * hop_a + 8 * B,          # new input + spectrum write
            "compat_analysis": 4 * hop_a + 8 * B,
            "synthesis": 8 * B_read + 4 * hop_s,    # spectrum read + emitted output
            "carry": 0, "runsum": 8 * B, "seam": 0,
            # q = 1 single launch (pv_fused.hip): spectrum written once, never re-read
            # (spec_written=False: the rows stay on chip, SURVEY's fused-mode bytes)
            "fused": 4 * hop_a + (8 * B if spec_written else 0) + 4 * hop_s,
            # real-time push (pv_rt.hip): the callback's new input and emitted output (§8(d)
            # fused-mode bytes; the spectrum is not written)
            "rt": 4 * hop_a + 4 * hop_s}.get(kernel, 0)


def alg_flops_per_frame(kernel, N, compat):
    """SURVEY §8(d) algorithmic flops per frame, split by kernel (the two STANDARD halves sum
    to 5 N log2 N + 5 N + 40 (N/2+1) = 77 kflop at N = 1024, REF_COMPAT's to 148 kflop):
      analysis         2.5 N log2 N (real FFT) + N (window) + 25 (N/2+1) (magnitude 3,
                       atan2 18, unwrap decision 4)
      compat_analysis  5 (2N) log2 (2N) (C2C 2N, kernel.cu:331) + N + 5 (N/2+1)
      synthesis        2.5 N log2 N (inverse real FFT) + 4 N (window, gain, overlap-add) +
                       15 (N/2+1) STANDARD (output phase, sin/cos, polar->rect), 5 (N/2+1)
                       REF_COMPAT"""
    lg = math.log2(N)
    b = N // 2 + 1
    ana = 2.5 * N * lg + N + 25 * b
    syn = 2.5 * N * lg + 4 * N + (5 if compat else 15) * b
    return {"analysis": ana, "compat_analysis": 5 * 2 * N * math.log2(2 * N) + N + 5 * b,
            "synthesis": syn, "fused": ana + syn, "rt": ana + syn}.get(kernel, 0.0)


def kernel_sources_sha():
    """sha256[:16] of the library's sources (pvamd._lib.sources_sha, the hash the Makefile
    compiles into libpv.so and scripts/isa_static.py records)"""
    from pvamd._lib import sources_sha
    return sources_sha()


# a roof "binds" when the kernel reaches this fraction of it; below it on both roofs the
# kernel is latency-bound at its occupancy (the regime named in `bound`)
BIND_FRAC = 0.75


def roofline(kernel, avg_ms, wl, N, hop_a, hop_s, B, frames, compat, traffic,
             isa_path=os.path.join(ROOT, "profiles", "isa_static.json"),
             regime_path=os.path.join(ROOT, "profiles", "regime.json"), spec_written=True):
    """Both roofs of the dominant kernel ("Report both and state which roof
    binds").  HBM: algorithmic bytes per launch / average launch time against 8 TB/s (the
    metric's "% HBM roofline": `achieved`, `peak`, `frac`).  VALU: algorithmic flops against
    the 157.3 TFLOP/s FP32 peak, and the issue-cycle estimate — the kernel's per-frame loop
    priced at the measured issue cost of each instruction form (scripts/isa_static.py ->
    profiles/isa_static.json, used only when its source hash matches this build) as a
    fraction of the SIMD cycles the launch had, at the 2.4 GHz peak clock and at the clock
    the chip was measured to hold on this workload (profiles/regime.json: the 1400 W cap
    holds ~1.8 GHz on config 3).  `bound` is "hbm" when the HBM fraction exceeds BIND_FRAC;
    else "power" when the package was measured at its power cap on this workload
    (`power_evidence`: the clock it holds there, the zero-data and ablation runs); else
    "valu" above BIND_FRAC of the issue, else "latency" — with "latency" and "power",
    `latency_evidence` carries the timing-only ablations that place the kernel's time
    (profiles/regime.json)."""
    t = avg_ms * 1e-3
    alg_bytes = alg_bytes_per_frame(kernel, N, hop_a, hop_s, B, compat, spec_written) * frames
    achieved = alg_bytes / t / 1e9
    hbm_frac = achieved / HBM_PEAK_GBS
    fl = alg_flops_per_frame(kernel, N, compat)
    tflops = fl * frames / t / 1e12
    valu = {"flops_per_frame": fl, "achieved_tflops": tflops, "peak_tflops": VALU_PEAK_TFLOPS,
            "flop_frac": tflops / VALU_PEAK_TFLOPS, "issue_cycles_per_frame": None,
            "issue_frac_at_peak_clock": None, "issue_frac_at_measured_clock": None,
            "measured_clock_ghz": None, "issue_source": None}
    regime = {}
    try:
        regime = json.load(open(regime_path)).get(wl, {})
    except (OSError, ValueError):
        regime = {}
    if regime.get("clock_ghz"):  # the measured clock, whatever the static estimate's state
        valu["measured_clock_ghz"] = float(regime["clock_ghz"])
        valu["clock_source"] = regime.get("clock_source")
    try:
        isa = json.load(open(isa_path))
        ent = isa.get(wl, {}).get(kernel)
        if ent is not None:
            cyc = ent["valu_cycles_per_frame"]
            valu["issue_cycles_per_frame"] = cyc
            if isa.get("_sources_sha16") == kernel_sources_sha():
                valu["issue_frac_at_peak_clock"] = cyc * frames / (SIMDS * t * PEAK_SCLK_GHZ * 1e9)
                if valu["measured_clock_ghz"]:
                    clk = valu["measured_clock_ghz"]
                    valu["issue_frac_at_measured_clock"] = cyc * frames / (SIMDS * t * clk * 1e9)
                valu["issue_source"] = ("profiles/isa_static.json (static count of this build's loop, "
                                        "measured issue costs)")
            else:  # a stale estimate is reported but never used for the regime
                valu["issue_source"] = "profiles/isa_static.json (STALE: sources changed since; not used)"
    except (OSError, ValueError, KeyError):
        pass
    issue = valu["issue_frac_at_measured_clock"]
    if issue is None:
        issue = valu["issue_frac_at_peak_clock"]
    vfrac = max(valu["flop_frac"], issue or 0.0)
    # the package power cap (profiles/regime.json: the power measured on this workload at the
    # cap, with the clock it holds there): below the HBM roof the cap, not a roof, sets the
    # time — the measured clock is what the issue fraction above is priced at
    pw, cap = regime.get("package_power_w"), regime.get("power_cap_w")
    power_capped = bool(pw and cap and float(pw) >= 0.99 * float(cap))
    if hbm_frac > BIND_FRAC and hbm_frac >= vfrac:
        bound = "hbm"
    elif power_capped:
        bound = "power"
    elif vfrac > BIND_FRAC:
        bound = "valu"
    else:
        bound = "latency"
    out = {"bound": bound, "bind_threshold": BIND_FRAC, "kernel": kernel,
           "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_frac,
           "frac_of": "hbm (the metric's % HBM roofline)", "traffic": traffic,
           "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": avg_ms, "valu": valu}
    if bound in ("latency", "power"):
        out["latency_evidence"] = (regime.get(kernel) or {}).get("latency_evidence")
    if bound == "power":
        out["power_evidence"] = (regime.get(kernel) or {}).get("power_evidence")
    return out


def bench_rt(args):
    """BASELINE configs[4]: real-time ring-buffer mode, 256 channels, N=256, hop=64
    (64-sample callbacks at 44.1 kHz: 1.451 ms deadline), PV_STANDARD pitch shift 1.5,
    one hipGraph replay per callback (BASELINE config 5's form; the graph's one kernel node
    reads / writes the pinned host buffers in place).  The same callbacks are then timed with
    a direct launch per callback (`alt_direct_launch`: measured faster on ROCm 7.2).  A step
    = one synchronous callback; latency percentiles are host wall-clock per
    callback (what an RtAudio thread waits for)."""
    import torch
    from pvamd import PITCH_SHIFT, RealTimeVocoder

    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(local)
    C, N, hop_div, scale = args.channels if args.channels != 1024 else 256, 256, 4, 1.5
    rt = RealTimeVocoder(N, PITCH_SHIFT, scale, hop_div, channels=C, device=local)
    hop = rt.hopSize
    steps = args.steps if args.steps != 10 else 2000
    warm = max(args.warmup, 50)
    blocks = synth_channels_np(C, hop * 64, 20240, cpu_share()[0]).reshape(C, 64, hop)

    def run_callbacks(v):
        for j in range(warm):
            v.host_in[:] = blocks[:, j % 64]
            v.callback()
        lat = np.empty(steps)
        t0 = time.perf_counter()
        for j in range(steps):
            a = time.perf_counter_ns()
            v.host_in[:] = blocks[:, j % 64]          # main.cpp:49 memcpy into curr_input
            v.callback()
            lat[j] = (time.perf_counter_ns() - a) * 1e-3
        return lat, time.perf_counter() - t0

    prev = os.environ.pop("PV_RT_LAUNCH", None)
    rt.capture(1)                                  # hipGraph replay per callback (config 5)
    lat, dt = run_callbacks(rt)
    os.environ["PV_RT_LAUNCH"] = "direct"          # the same callbacks, one launch each
    alt = RealTimeVocoder(N, PITCH_SHIFT, scale, hop_div, channels=C, device=local)
    alt.capture(1)
    lat_d, dt_d = run_callbacks(alt)
    alt.close()
    if prev is None:
        os.environ.pop("PV_RT_LAUNCH", None)
    else:
        os.environ["PV_RT_LAUNCH"] = prev
    # device time of the per-callback kernel alone (events on the push stream)
    x = torch.from_numpy(blocks[:, 0].copy()).cuda()
    out = torch.empty((C, rt.outHopSize), device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(20):
        rt.push(x, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(200):
        rt.push(x, out=out)
    e1.record(s)
    torch.cuda.synchronize()
    k_us = e0.elapsed_time(e1) / 200 * 1e3
    deadline_us = hop / SR * 1e6
    frame_bytes = 4 * hop + 4 * rt.outHopSize  # SURVEY.md §8(d) fused-mode bytes per frame
    rt_roof = roofline("rt", k_us * 1e-3, "rt", N, hop, rt.outHopSize, N // 2 + 1, C, False, None)
    assert abs(rt_roof["alg_bytes_per_launch"] - C * frame_bytes) < 1e-6
    # one callback of 256 frames is ~7 us of device time, mostly launch and dependent latency
    rt_roof["bound"] = "latency"
    rt_roof["latency_note"] = ("a callback's kernel moves 256 frames x 512 B: HBM and VALU both idle; "
                               "the host round trip per callback (latency_us) is what the deadline sees")
    line = {
        "metric": METRIC + " [real-time mode]", "value": C * steps / dt, "unit": "frames/s",
        "n_gpus": 1, "steps": steps, "warmup": warm, "ms_per_step": dt / steps * 1e3,
        "higher_is_better": True, "scaling": "replicas only", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (3 sines + noise), 64-sample blocks cycled",
        "config": {"workload": "BASELINE configs[4]: real-time ring buffer, 256 ch, N=256 hop=64, "
                               "PV_STANDARD pitch 1.5, hipGraph replay per callback (zero-copy)",
                   "channels": C, "N": N, "hop": hop, "out_hop": rt.outHopSize},
        "latency_us": {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                       "max": float(lat.max()), "deadline": deadline_us,
                       "missed": int(np.sum(lat > deadline_us))},
        "kernel_us": k_us,
        "alt_direct_launch": {"value": C * steps / dt_d, "p50_us": float(np.percentile(lat_d, 50)),
                              "p99_us": float(np.percentile(lat_d, 99)), "max_us": float(lat_d.max())},
        "roofline": rt_roof,
        "world_size_env": world,
    }
    print(json.dumps(line), flush=True)


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this script
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), as torchrun would.
    This parent never touches the GPU and never re-execs; it waits for the ranks, stops the
    others if one fails, and exits with the first failing rank's status (rank 0 prints the
    JSON line)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


def pv_frames(n, hop):
    from pvamd import frame_count
    return frame_count(n, hop)


if __name__ == "__main__":
    sys.exit(main() or 0)
