#!/usr/bin/env python3
"""Static check of the self-tracked prefetches (pv_device.hpp gload_pairs / gload_tail /
gload_row): their global loads are inline asm, invisible to the compiler's s_waitcnt
insertion, so nothing may read, write or copy a destination register of such a load between
the load and the `s_waitcnt vmcnt(N)` that retires it.  A copy would read the register
before the data lands; a reuse of the register would be overwritten when it does (a later
address in that register then faults).

For every inline-asm `global_load_*` of every kernel in a device assembly file, walk forward
in program order, counting the vector-memory instructions issued after the load, until an
`s_waitcnt vmcnt(N)` with at least N of them (the load has then retired); report any
instruction on the way that names one of its destination registers, along every path of the
control flow (branches followed both ways).

A second check covers inline asm that writes SCC (s_and_b64 exec ... in pv_device.hpp
lane0_mov2): if a block has an SCC-writing scalar instruction, the next SCC reader after it
(s_addc / s_subb / s_cselect / s_cmov / s_cbranch_scc) must follow another SCC writer — the
compiler keeps SCC live across an asm block that does not declare the "scc" clobber (a
64-bit address add split around such a block once took a wrong carry and faulted).

  python3 scripts/prefetch_hazards.py file.s [...]   -> exit status 1 if any hazard
"""
import re
import sys

VMEM = ("global_load", "global_store", "buffer_load", "buffer_store", "flat_load", "flat_store",
        "global_atomic", "buffer_atomic", "flat_atomic")


def regs_of(operand):
    """v5 -> {5}; v[4:7] -> {4,5,6,7}"""
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", operand):
        out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", operand):
        out.add(int(m.group(1)))
    return out


def functions(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur:
            if re.match(r"^\.Lfunc_end", line):
                yield cur, body
                cur, body = None, []
            else:
                body.append(line.rstrip("\n"))
    if cur:
        yield cur, body


def check(path):
    hazards = []
    for fn, body in functions(path):
        insts, labels = [], {}  # (text, in_asm); label -> index of its first instruction
        in_asm = False
        for line in body:
            s = line.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            m = re.match(r"^(\.LBB\w+):", s)
            if m:
                labels[m.group(1)] = len(insts)
                continue
            if not s or s.startswith((";", ".")) or s.endswith(":"):
                continue
            insts.append((s.split(";")[0].strip(), in_asm))
        for i, (t, asm) in enumerate(insts):
            op = t.split()[0]
            if not (asm and op.startswith(("global_load", "buffer_load"))):
                continue
            dst = regs_of(t.split()[1].rstrip(","))
            # every path from the load (following branches) until the load has retired
            stack, seen, found = [(i + 1, 0)], set(), None
            while stack and found is None:
                pc, after = stack.pop()
                while pc < len(insts):
                    key = (pc, min(after, 64))
                    if key in seen:
                        break
                    seen.add(key)
                    t2 = insts[pc][0]
                    op2 = t2.split()[0]
                    if op2 == "s_waitcnt" and "vmcnt(" in t2:
                        n = int(re.search(r"vmcnt\((\d+)\)", t2).group(1))
                        if after >= n:
                            break
                    if op2 == "s_endpgm":
                        break
                    if op2.startswith(VMEM):
                        after += 1
                    if op2.startswith(("v_", "ds_", "global_", "buffer_", "flat_")) and regs_of(t2[len(op2):]) & dst:
                        found = t2
                        break
                    if op2 == "s_branch":
                        pc = labels.get(t2.split()[-1], len(insts))
                        continue
                    if op2.startswith("s_cbranch"):
                        tgt = labels.get(t2.split()[-1])
                        if tgt is not None:
                            stack.append((tgt, after))
                    pc += 1
            if found is not None:
                hazards.append((fn, t, found))
    return hazards


SCC_READERS = ("s_addc", "s_subb", "s_cselect", "s_cmov", "s_cbranch_scc")
SCC_NEUTRAL = ("s_mov", "s_waitcnt", "s_nop", "s_setprio", "s_branch", "s_cbranch_exec", "s_cbranch_vcc",
               "s_barrier", "s_memtime", "s_memrealtime", "s_sleep", "s_getpc", "s_setpc", "s_swappc",
               "s_endpgm", "s_sendmsg", "s_load", "s_buffer_load", "s_store", "s_dcache", "s_icache",
               "s_cbranch_cdbg", "s_trap", "s_setreg", "s_getreg", "s_inst_prefetch")


def writes_scc(op):
    return op.startswith("s_") and not op.startswith(SCC_NEUTRAL + SCC_READERS)


def check_scc(path):
    bad = []
    for fn, body in functions(path):
        lines = [l.strip() for l in body]
        in_asm, asm_scc = False, False
        for i, s in enumerate(lines):
            if s.startswith(";;#ASMSTART"):
                in_asm, asm_scc = True, False
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                if asm_scc:
                    for t in lines[i + 1:i + 400]:
                        if not t or t.startswith((";", ".")) or t.endswith(":"):
                            continue
                        op = t.split()[0]
                        if op.startswith(SCC_READERS):
                            bad.append((fn, t))
                            break
                        if writes_scc(op):
                            break
                continue
            if in_asm and s and not s.startswith((";", ".")):
                if writes_scc(s.split()[0]):
                    asm_scc = True
    return bad


def main():
    bad = 0
    for p in sys.argv[1:]:
        for fn, load, use in check(p):
            bad += 1
            print(f"{p}: {fn[:80]}\n    load: {load}\n    use before its vmcnt: {use}")
        for fn, use in check_scc(p):
            bad += 1
            print(f"{p}: {fn[:80]}\n    SCC read after an inline asm block that writes SCC: {use}")
    print(f"{bad} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
