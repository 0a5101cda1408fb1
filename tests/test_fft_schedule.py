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


@pytest.mark.parametrize("L", [128, 512, 2048])
def test_lds_padding_is_injective(L):
    E = L // 64
    sh = E.bit_length() - 1
    pads = {p + (p >> sh) for p in range(L + 1)}
    assert len(pads) == L + 1 and max(pads) < L + (L >> sh) + 2
