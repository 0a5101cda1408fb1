#!/usr/bin/env python3
"""Static instruction mix of a kernel's hottest loop from device assembly (diagnostic).

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
      -o k.s phase-vocoder_amd/csrc/pv_kernels.hip
  python3 scripts/isa_loop_counts.py k.s '_ZN2pv11k_synthesisILi512ELi0ELi1ELb1'

Takes the function whose symbol starts with the given prefix, finds every backward branch
(a loop), and prints the instruction classes of the largest loop body: VALU (packed,
transcendental), DPP / permlane, LDS reads / writes / bpermute, global loads / stores,
SALU, waits.
"""
import re
import sys
from collections import Counter


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


def classify(op, text):
    if op.startswith("v_"):
        if "_dpp" in op or "row_" in text or "quad_perm" in text:
            return "valu_dpp"
        if op.startswith("v_permlane"):
            return "valu_permlane"
        if op.startswith(("v_sin", "v_cos", "v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log")):
            return "valu_trans"
        if op.startswith("v_pk_"):
            return "valu_packed"
        return "valu"
    if op.startswith("ds_bpermute") or op.startswith("ds_permute"):
        return "lds_permute"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "lds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "lds_write"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    body = function_body(path, prefix)
    labels = {}
    insts = []  # (index, op, text)
    for line in body:
        m = re.match(r"^(\.LBB\w+):", line)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        insts.append((op, s))
    loops = []
    for i, (op, s) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                loops.append((labels[tgt], i))
    if not loops:
        print("no loop found; whole function")
        loops = [(0, len(insts) - 1)]
    a, b = max(loops, key=lambda x: x[1] - x[0])
    cnt = Counter(classify(op, s) for op, s in insts[a:b + 1])
    print(f"{prefix}: loop of {b - a + 1} instructions (of {len(insts)}; {len(loops)} loops)")
    for k in sorted(cnt):
        print(f"  {k:14s} {cnt[k]}")
    valu = sum(v for k, v in cnt.items() if k.startswith("valu"))
    print(f"  VALU total     {valu}")


if __name__ == "__main__":
    main()
