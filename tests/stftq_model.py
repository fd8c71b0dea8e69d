"""A numpy model of stftq_kernel's FFT schedule (csrc/stftq_kernels.hip, n_fft 256 / 512 / 1024):
rustfft 4.0 Radix4 on a frame held as L lanes x P registers (point m = lane + L * register), the
digits taken from the top of m (the prepare_radix4 order), every digit moved into register bits
before its level by lane-bit <-> register-bit swaps, the same f32 operations in the same order
as the oracle's cfft_tab. schedule() is the rule the kernel's constexpr tables follow
(stftq_sched in the .hip file); tests/test_stftq_model.py checks the model against the oracle
bit for bit. Test infrastructure."""
import numpy as np

from stftr_model import Cx, rbfly, rbfly4

GEOM = {128: (16, 8), 256: (16, 16), 512: (32, 16)}  # NC -> (L lanes, P registers)


def schedule(NC):
    """(L, P, levels, pbit): levels = [{digit, swaps, loc, pstart, radix}], digit = the m bits
    of the level's digit (LSB first), swaps = (lane bit, register bit) pairs done before it, loc
    = m bit -> ('l' | 'r', bit) after them, pbit = m bit -> its bit in the output index p."""
    L, P = GEOM[NC]
    B = NC.bit_length() - 1
    nl, nr = L.bit_length() - 1, P.bit_length() - 1
    if B % 2:  # a radix-8 base (butterfly_8 over m's top 3 bits), then radix-4 digits downwards
        digits = [list(range(B - 3, B))] + [[2 * i, 2 * i + 1] for i in reversed(range((B - 3) // 2))]
    else:
        digits = [[2 * i, 2 * i + 1] for i in reversed(range(B // 2))]
    pbit, pos = {}, 0
    for d in digits:
        for c, b in enumerate(d):
            pbit[b] = pos + c
        pos += len(d)
    loc = {b: ("l", b) if b < nl else ("r", b - nl) for b in range(B)}
    levels = []
    for d in digits:
        swaps = []
        for b in d:
            if loc[b][0] == "l":
                x = loc[b][1]
                y = [r for r in range(nr) if not any(loc[bb] == ("r", r) for bb in d)][0]
                other = [k for k in loc if loc[k] == ("r", y)][0]
                loc[b], loc[other] = ("r", y), ("l", x)
                swaps.append((x, y))
        levels.append(dict(digit=list(d), swaps=swaps, loc=dict(loc), pstart=min(pbit[b] for b in d),
                           radix=1 << len(d)))
    return L, P, levels, pbit


def rbfly8(b, w1, w3):
    """oracle bfly8 (rustfft butterfly_8) on 8 Cx."""
    s = [b[0], b[2], b[4], b[6], b[1], b[3], b[5], b[7]]
    s[0], s[1], s[2], s[3] = rbfly4(s[0], s[1], s[2], s[3])
    s[4], s[5], s[6], s[7] = rbfly4(s[4], s[5], s[6], s[7])
    s[5] = s[5].mul(w1)
    s[6] = Cx(s[6].im, -s[6].re)
    s[7] = s[7].mul(w3)
    for i in range(4):
        s[i], s[i + 4] = s[i] + s[i + 4], s[i] - s[i + 4]
    return s


def fft(z, tw, w8):
    """z: NC complex64 points; tw: rustfft twiddles [NC]; w8: (twiddle(1, 8), twiddle(3, 8)).
    Returns Z[p] (natural order) as the kernel's schedule computes it."""
    NC = z.size
    L, P, levels, pbit = schedule(NC)
    lane = np.arange(L)
    # v[r] = lanes' values of register r (Cx arrays over lanes): point m = lane + L r
    v = [Cx(z.real[lane + L * r], z.imag[lane + L * r]) for r in range(P)]
    twc = Cx(tw.real, tw.imag)

    def T(idx):
        return Cx(twc.re[idx], twc.im[idx])

    for t, lev in enumerate(levels):
        for (x, y) in lev["swaps"]:
            nv = [None] * P
            for r in range(P):
                w = (r >> y) & 1
                src_l = (lane & ~(1 << x)) | (w << x)
                u = (lane >> x) & 1
                src_r = np.where(u == 1, r | (1 << y), r & ~(1 << y))
                re = np.empty(L, np.float32)
                im = np.empty(L, np.float32)
                for rr in (r & ~(1 << y), r | (1 << y)):
                    sel = src_r == rr
                    re[sel] = v[rr].re[src_l[sel]]
                    im[sel] = v[rr].im[src_l[sel]]
                nv[r] = Cx(re, im)
            v = nv
        loc, d = lev["loc"], lev["digit"]
        rbits = [loc[b][1] for b in d]
        R = lev["radix"]
        q = 1 << lev["pstart"]
        tstride = NC // (q * 4)
        for base in range(P):
            if any((base >> rb) & 1 for rb in rbits):
                continue
            regs = [base | sum(((dv >> c) & 1) << rb for c, rb in enumerate(rbits)) for dv in range(R)]
            if t == 0:
                if R == 4:
                    out = rbfly4(*[v[r] for r in regs])
                else:
                    out = rbfly8([v[r] for r in regs], Cx(np.float32(w8[0].real), np.float32(w8[0].imag)),
                                 Cx(np.float32(w8[1].real), np.float32(w8[1].imag)))
            else:
                j = np.zeros(L, np.int64)
                for b, (kind, bit) in loc.items():
                    if pbit[b] >= lev["pstart"]:
                        continue
                    bv = (lane >> bit) & 1 if kind == "l" else np.full(L, (base >> bit) & 1)
                    j += bv << pbit[b]
                out = rbfly(*[v[r] for r in regs], T(j * 1 * tstride), T(j * 2 * tstride), T(j * 3 * tstride))
            for r, o in zip(regs, out):
                v[r] = o
    loc = levels[-1]["loc"]
    Z = np.zeros(NC, np.complex64)
    for r in range(P):
        p = np.zeros(L, np.int64)
        for b, (kind, bit) in loc.items():
            bv = (lane >> bit) & 1 if kind == "l" else np.full(L, (r >> bit) & 1)
            p += bv << pbit[b]
        Z.real[p] = v[r].re
        Z.imag[p] = v[r].im
    return Z
