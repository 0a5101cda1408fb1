#!/usr/bin/env python3
"""Static VALU issue estimate per frame for the kernels bench.py reports (diagnostic).

Compiles the kernel sources to gfx950 assembly (device only, the Makefile's flags), takes
each reported kernel's per-frame loop (the smallest loop that holds the frame's LDS
permutes and global stores) and prices its VALU instructions with the issue costs measured
on MI355X (cycles per wave-instruction per SIMD at 8 waves/SIMD: profiles/r03_valu_probe2.jsonl,
profiles/r04_valu_probe3.jsonl).  Writes profiles/isa_static.json, which bench.py turns into
`roofline.valu.issue_cycles_per_frame` and the issue fraction of the kernel's time.

  python3 scripts/isa_static.py            # -> profiles/isa_static.json
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "phase-vocoder_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "--cuda-device-only", "-S"]

# (workload, bench kernel key) -> (source, extra flags, mangled-name prefix, transcendental
# instructions per frame: the analysis takes E + 1 square roots, the synthesis E + 1 cosines
# and E sines, E = L / 64 — how many frames one trip of an unrolled loop covers)
KERNELS = {
    ("c3", "analysis"): ("pv_analysis.hip", ["-fno-slp-vectorize"], "_ZN2pv14k_std_analysisILi512ELb0ELi2ELb1E", 9),
    ("c3", "synthesis"): ("pv_kernels.hip", [], "_ZN2pv11k_synthesisILi512ELi0ELi1ELb1ELb1E", 17),
    # config 4 (bench.py: no spectrum handed back, pitch 1.5): the instantiation analysing
    # lane registers 0 .. 11 (bins < 768; 12 square roots, no bin L)
    ("c4", "analysis"): ("pv_analysis.hip", ["-fno-slp-vectorize"], "_ZN2pv14k_std_analysisILi1024ELb0ELi4ELb1ELi12E", 12),
    ("c4", "synthesis"): ("pv_kernels.hip", [], "_ZN2pv11k_synthesisILi1024ELi3ELi4ELb1ELb1ELi12E", 33),
    ("compat", "compat_analysis"): ("pv_analysis.hip", ["-fno-slp-vectorize"], "_ZN2pv17k_compat_analysisILi512E", 9),
    ("compat", "synthesis"): ("pv_kernels.hip", [], "_ZN2pv11k_synthesisILi512ELi1ELi2ELb0ELb0E", 17),
    # config 2's single launch (pitch 2: MODE 4, the half-size resynthesis of X^2 / |X|):
    # analysis + synthesis of a frame in one loop trip; 14 = 6 reciprocal square roots + the
    # 8 square roots of the spectrum-output branch, which the static count includes (bench.py
    # runs without it, so the estimate is an upper bound there)
    ("c2", "fused"): ("pv_fused.hip", [], "_ZN2pv7k_fusedILi512ELi4ELi2EE", 14),
    # config 5's per-callback kernel: one frame per wave and launch, no frame loop — the whole
    # kernel is priced (table staging included, its loops counted once); L = 128: 3 + 5
    ("rt", "rt"): ("pv_rt.hip", [], "_ZN2pv4k_rtILi128ELi2ELb1EE", None),
}

# issue cycles per wave-instruction at 8 waves/SIMD (measured; see the module docstring)
FAST = 2.25    # v_fma/fmac/add/sub/mul_f32 (no source modifiers), v_mov_b32, v_add/sub_u32
SLOW = 4.15    # compares, selects, v_bfi, v_rndne, v_fract, min/max with modifiers, max3, ...
PACKED = 4.33  # v_pk_fma/mul/add_f32
TRANS = 8.2    # v_sqrt, v_sin, v_cos, v_rcp, ...
FAST_OPS = ("v_fma_f32", "v_fmac_f32", "v_fmaak_f32", "v_fmamk_f32", "v_add_f32", "v_sub_f32",
            "v_subrev_f32", "v_mul_f32", "v_mov_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32")
FAST_EXTRA = "profiles/r04_valu_costs.json"  # measured overrides {opcode: cycles}, if present


def sources_sha():
    """the library's source hash (phase-vocoder_amd/pvamd/_lib.py sources_sha, the Makefile's
    SRC_SHA): every *.hip *.hpp *.h *.cpp in csrc/ and the Makefile in byte order, then
    include/pv.h"""
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".h", ".cpp")) or f == "Makefile")
    h = hashlib.sha256()
    for p in [os.path.join(CSRC, f) for f in names] + [os.path.join(ROOT, "include", "pv.h")]:
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def function_body(path, prefix):
    lines, on = [], False
    for line in open(path):
        if not on and re.match(rf"^{re.escape(prefix)}\w*:", line):
            on = True
            continue
        if on:
            if line.startswith("\t.section") or re.match(r"^\.Lfunc_end", line):
                break
            lines.append(line.rstrip("\n"))
    return lines


def cost_of(op, text, extra):
    if op in extra:
        return extra[op]
    if op.startswith(("v_sin", "v_cos", "v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log")):
        return TRANS
    if op.startswith("v_pk_"):
        return PACKED
    if op.startswith(FAST_OPS) and "|" not in text and " div:" not in text and " mul:" not in text:
        return FAST
    return SLOW


def loops_of(asm, prefix):
    """every loop body (backward branch) of the function, as (start, end, instructions)"""
    labels, insts = {}, []
    for line in function_body(asm, prefix):
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")):
            continue
        insts.append((s.split()[0], s))
    out = []
    for i, (op, s) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                out.append((labels[tgt], i, insts[labels[tgt]:i + 1]))
    return out


def price(seg, extra):
    cnt, cyc = Counter(), 0.0
    for op, text in seg:
        if op.startswith("v_"):
            c = cost_of(op, text, extra)
            cyc += c
            cnt["valu_trans" if c == TRANS else "valu_packed" if op.startswith("v_pk_") else "valu"] += 1
        elif op.startswith("ds_"):
            cnt["lds"] += 1
        elif op.startswith(("global_", "buffer_")):
            cnt["vmem"] += 1
    return cnt, cyc


def frame_loop(asm, prefix, trans_pf, extra):
    """The steady-state frame loop: among the innermost loops that hold a frame's work (its
    square roots / sines / cosines and global stores), the one with the fewest VALU cycles per frame (the path every
    full run takes; the bounds-checked variants for the channel ends cost more)."""
    def trans(seg):
        return sum(1 for o, _ in seg if o.startswith(("v_sin", "v_cos", "v_sqrt", "v_rsq")))
    cands = [(a, b, seg) for a, b, seg in loops_of(asm, prefix)
             if trans(seg) >= trans_pf and any(o.startswith("global_store") for o, _ in seg)]
    inner = [c for c in cands if not any(o is not c and c[0] <= o[0] and o[1] <= c[1] for o in cands)]
    best = None
    for a, b, seg in inner:
        cnt, cyc = price(seg, extra)
        fpl = max(1, round(cnt["valu_trans"] / trans_pf))
        if best is None or cyc / fpl < best[2] / best[1]:
            best = (seg, fpl, cyc, cnt)
    return best


def main():
    extra = {}
    p = os.path.join(ROOT, FAST_EXTRA)
    if os.path.exists(p):
        extra = json.load(open(p)).get("cycles", {})
    out = {"_sources_sha16": sources_sha(),
           "_cost_model": {"fast": FAST, "slow": SLOW, "packed": PACKED, "trans": TRANS,
                           "overrides": FAST_EXTRA if extra else None},
           "_note": "VALU issue cycles per frame of each kernel's per-frame loop (static, gfx950 "
                    "assembly of this build), priced at the measured 8-wave issue costs"}
    cache = {}
    with tempfile.TemporaryDirectory() as td:
        for (wl, key), (src, fl, prefix, trans_pf) in KERNELS.items():
            asm = cache.get((src, tuple(fl)))
            if asm is None:
                asm = os.path.join(td, f"{src}{len(cache)}.s")
                subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *fl, "-o", asm, os.path.join(CSRC, src)],
                               check=True, stderr=subprocess.DEVNULL)
                cache[(src, tuple(fl))] = asm
            if trans_pf is None:  # no frame loop: the whole kernel is one frame
                seg = [(ln.strip().split()[0], ln.strip()) for ln in function_body(asm, prefix)
                       if ln.strip() and not ln.strip().startswith((";", ".")) and not ln.endswith(":")]
                cnt, cyc = price(seg, extra)
                out.setdefault(wl, {})[key] = {"symbol": prefix, "kernel_instructions": len(seg),
                                               "frames_per_trip": 1, "scope": "whole kernel (loops counted once)",
                                               "counts_per_trip": dict(cnt),
                                               "valu_cycles_per_frame": round(cyc, 1)}
                continue
            best = frame_loop(asm, prefix, trans_pf, extra)
            if best is None:
                continue
            seg, fpl, cyc, cnt = best
            out.setdefault(wl, {})[key] = {"symbol": prefix, "loop_instructions": len(seg),
                                           "frames_per_trip": fpl,
                                           "counts_per_trip": dict(cnt),
                                           "valu_cycles_per_frame": round(cyc / fpl, 1)}
    dst = os.path.join(ROOT, "profiles", "isa_static.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main())
