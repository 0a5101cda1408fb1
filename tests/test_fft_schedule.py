"""Integer proof that the register-blocked Stockham schedule of pv_device.hpp performs
exactly the radix-2 butterflies of the oracle's FFT (pvr_fft_c32 / hpfft.cu:145-167):
same stage, same top/bottom input positions, same twiddle index, same output positions.
Together with identical per-butterfly arithmetic this is why the GPU spectra are
bit-identical to the oracle's."""
import pytest


def radix2_butterflies(L):
    out = set()
    Ns = 1
    while Ns < L:
        for j in range(L // 2):
            idx = j & (Ns - 1)
            pos = (j // Ns) * 2 * Ns + idx
            out.add((Ns, j, j + L // 2, idx, pos, pos + Ns))
        Ns <<= 1
    return out


def bitrev(v, bits):
    r = 0
    for i in range(bits):
        r |= ((v >> i) & 1) << (bits - 1 - i)
    return r


def blocked_butterflies(L):
    """Mirror of fft_pass / pass_store / pass_load in pv_device.hpp (positions tracked)."""
    LOG2L = L.bit_length() - 1
    E = L // 64
    RLOG = E.bit_length() - 1
    npass = (LOG2L + RLOG - 1) // RLOG
    seen = set()
    for P in range(npass):
        S = 1 << (P * RLOG)
        r = min(RLOG, LOG2L - P * RLOG)
        R = 1 << r
        NG = E // R
        for lane in range(64):
            for g in range(NG):
                j = lane + 64 * g
                jm = j & (S - 1)
                # input positions of the pass-stage being processed, per register slot
                pos = [j + q * (L // R) for q in range(R)]
                for st in range(r):
                    Ns = S << st
                    newpos = [None] * R
                    for s in range(R // 2):
                        br = bitrev(s & ((1 << st) - 1), st)
                        tw = jm + S * br
                        top, bot = pos[s], pos[s + R // 2]
                        assert bot == top + L // 2
                        o0 = (top // Ns) * 2 * Ns + (top & (Ns - 1))
                        assert (top & (Ns - 1)) == tw, "twiddle index mismatch"
                        seen.add((Ns, top, bot, tw, o0, o0 + Ns))
                        newpos[2 * s], newpos[2 * s + 1] = o0, o0 + Ns
                    pos = newpos
                # pass_store: slot f goes to J + S*bitrev(f)
                J = (j // S) * R * S + jm
                for f in range(R):
                    assert pos[f] == J + S * bitrev(f, r)
    return seen


@pytest.mark.parametrize("L", [128, 256, 512, 1024, 2048])
def test_blocked_schedule_equals_radix2(L):
    assert blocked_butterflies(L) == radix2_butterflies(L)


# exchange layouts of pv_device.hpp (lay_c / lay_s): slot(p) = p + c * (p >> s)
LAYOUT = {128: [(1, 4), (2, 4), (4, 4), (8, 4), (0, 4), (0, 4)], 256: [(1, 4), (4, 4), (0, 4)],
          512: [(1, 4), (8, 6)], 1024: [(1, 4), (0, 4)], 2048: [(1, 5), (0, 5)]}


def _bank_cycles(slots, write):
    """LDS-array cycles of one wave-instruction on float2 slots (MI355X_MICROARCH.md §LDS):
    ds_write_b64 in 4 x 16 lanes over 32 banks, ds_read_b64 in 2 x 32 lanes over 64 banks."""
    group, nb = (16, 32) if write else (32, 64)
    tot = 0
    for g0 in range(0, 64, group):
        banks = {}
        for lane in range(g0, g0 + group):
            for d in (2 * slots[lane], 2 * slots[lane] + 1):
                banks.setdefault(d % nb, set()).add(d)
        tot += max(len(v) for v in banks.values())
    return tot


@pytest.mark.parametrize("L", [128, 256, 512, 1024, 2048])
def test_lds_layouts_injective_affine_and_conflict_free(L):
    """Each exchange layout is injective, keeps base + compile-time-offset addressing, and
    (L >= 256) the unpadded final image and the exchanges beat one pad every E points."""
    E = L // 64
    RLOG = E.bit_length() - 1
    LOG2L = L.bit_length() - 1
    npass = (LOG2L + RLOG - 1) // RLOG
    assert len(LAYOUT[L]) == npass - 1
    new = old = 0
    for P in range(npass):
        S = 1 << (P * RLOG)
        r = min(RLOG, LOG2L - P * RLOG)
        R = 1 << r
        c, s = LAYOUT[L][P] if P + 1 < npass else (0, 0)
        sl = (lambda p, c=c, s=s: p + c * (p >> s))
        cur = (lambda p: p + (p >> RLOG))
        assert len({sl(p) for p in range(L)}) == L
        writes = []
        for g in range(E // R):
            for f in range(R):
                pts = []
                for lane in range(64):
                    j = lane + 64 * g
                    J = (j // S) * R * S + (j & (S - 1))
                    off = S * bitrev(f, r)
                    assert sl(J + off) == sl(J) + sl(off)
                    pts.append(J + off)
                writes.append(pts)
        reads = []
        if P + 1 < npass:
            r2 = min(RLOG, LOG2L - (P + 1) * RLOG)
            R2 = 1 << r2
            for g in range(E // R2):
                for q in range(R2):
                    off = 64 * g + q * (L // R2)
                    assert all(sl(lane + off) == sl(lane) + sl(off) for lane in range(64))
                    reads.append([lane + off for lane in range(64)])
        else:  # real split: bins k and L - k
            for i in range(E):
                reads.append([lane + 64 * i for lane in range(64)])
                reads.append([(L - lane - 64 * i) % L for lane in range(64)])
        for fn, acc in ((sl, "new"), (cur, "old")):
            cyc = sum(_bank_cycles([fn(p) for p in w], True) for w in writes) + \
                sum(_bank_cycles([fn(p) for p in rd], False) for rd in reads)
            if acc == "new":
                new += cyc
            else:
                old += cyc
    assert new <= old
    if L == 512:
        assert (new, old) == (176, 256)
