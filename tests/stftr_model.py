"""A numpy model of stftr_kernel's data flow (csrc/stftr_kernels.hip): the same f32 operations on
the same operands in the same order, with the kernel's lane / register placement made explicit
(lane l, register n), so the index maps -- ring layout, the permlane swaps, the LDS transpose, the
partner exchange of the untangle -- can be checked against the oracle bit for bit on the CPU.
Test infrastructure (tests/test_stftr_model.py)."""
import numpy as np

NC, L, P = 1024, 64, 16
f32 = np.float32


class Cx:
    """Complex as two float32 arrays (no fused operations: numpy f32 ops round once each)."""

    def __init__(self, re, im):
        self.re = np.asarray(re, f32)
        self.im = np.asarray(im, f32)

    def __add__(self, o):
        return Cx(self.re + o.re, self.im + o.im)

    def __sub__(self, o):
        return Cx(self.re - o.re, self.im - o.im)

    def mul(self, w):  # num-complex Mul
        return Cx(self.re * w.re - self.im * w.im, self.re * w.im + self.im * w.re)

    def copy(self):
        return Cx(self.re.copy(), self.im.copy())


def rbfly(d0, d1, d2, d3, w1, w2, w3):
    s0, s1, s2 = d1.mul(w1), d2.mul(w2), d3.mul(w3)
    s5 = d0 - s1
    a = d0 + s1
    s3, s4 = s0 + s2, s0 - s2
    n2 = a - s3
    n0 = a + s3
    n1 = Cx(s5.re + s4.im, s5.im - s4.re)
    n3 = Cx(s5.re - s4.im, s5.im + s4.re)
    return n0, n1, n2, n3


def rbfly4(a0, a1, a2, a3):
    v0, v1, v2, v3 = a0, a1, a2, a3
    v0, v2 = v0 + v2, v0 - v2
    v1, v3 = v1 + v3, v1 - v3
    v3 = Cx(v3.im, -v3.re)
    v0, v1 = v0 + v1, v0 - v1
    v2, v3 = v2 + v3, v2 - v3
    return v0, v2, v1, v3


def frame(z, tw, sc):
    """z: the frame's NC complex points (windowed), complex64 [NC]; tw: rustfft twiddles [NC]
    complex64; sc: realfft (sin, cos) float32 [NC, 2]. Returns the NC + 1 bins as the kernel
    produces them."""
    lane = np.arange(L)
    twc = Cx(tw.real, tw.imag)

    def T(idx):  # twiddle table lookup (per lane or uniform)
        return Cx(twc.re[idx], twc.im[idx])

    # ring layout: v[n][l] = z[l + 64 n]
    v = [Cx(z.real[lane + 64 * n], z.imag[lane + 64 * n]) for n in range(P)]
    for d1 in range(4):  # level 0
        v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12] = rbfly4(v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12])
    for j in range(4):  # level 1
        v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3] = rbfly(
            v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3], T(64 * j), T(128 * j), T(192 * j))
    # permlane16 swap: odd rows (lane bit 4) of v[q] <-> even rows of v[q + 4], q bit 2 = 0
    odd16 = (lane >> 4) & 1 == 1
    for q in range(16):
        if q & 4:
            continue
        x, y = v[q].copy(), v[q + 4].copy()
        src_even = lane ^ 16  # partner lane
        for comp in ("re", "im"):
            xs, ys = getattr(v[q], comp), getattr(v[q + 4], comp)
            nx = np.where(odd16, ys[src_even], xs)
            ny = np.where(~odd16, xs[src_even], ys)
            setattr(x, comp, nx)
            setattr(y, comp, ny)
        v[q], v[q + 4] = x, y
    hi32 = lane >= 32
    for q in range(8):
        x, y = v[q].copy(), v[q + 8].copy()
        p = lane ^ 32
        for comp in ("re", "im"):
            xs, ys = getattr(v[q], comp), getattr(v[q + 8], comp)
            setattr(x, comp, np.where(hi32, ys[p], xs))
            setattr(y, comp, np.where(~hi32, xs[p], ys))
        v[q], v[q + 8] = x, y
    d0s = lane >> 4
    for d1 in range(4):  # level 2
        j = d0s + 4 * d1
        v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12] = rbfly(v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12],
                                                        T(16 * j), T(32 * j), T(48 * j))
    # transpose: lane writes row wrow, column d0 + 4 n; lane reads column col
    grid_re = np.zeros((16, 64), f32)
    grid_im = np.zeros((16, 64), f32)
    wrow = ((lane >> 2) & 3) + 4 * (lane & 3)
    for q in range(P):
        grid_re[wrow, d0s + 4 * q] = v[q].re
        grid_im[wrow, d0s + 4 * q] = v[q].im
    col = np.where(lane <= 32, lane, 96 - lane)
    v = [Cx(grid_re[r, col], grid_im[r, col]) for r in range(P)]
    w3 = (T(col * 4), T(col * 8), T(col * 12))
    for d4 in range(4):  # level 3
        v[4 * d4], v[4 * d4 + 1], v[4 * d4 + 2], v[4 * d4 + 3] = rbfly(
            v[4 * d4], v[4 * d4 + 1], v[4 * d4 + 2], v[4 * d4 + 3], *w3)
    for d3 in range(4):  # level 4
        j = col + 64 * d3
        v[d3], v[d3 + 4], v[d3 + 8], v[d3 + 12] = rbfly(v[d3], v[d3 + 4], v[d3 + 8], v[d3 + 12],
                                                        T(j), T(2 * j), T(3 * j))
    # partner exchange (permlane32 of v[8 + i] with itself)
    lo = lane < 32
    special = (lane == 0) | (lane == 32)
    pr = []
    for i in range(8):
        x = v[8 + i]
        part = lane ^ 32
        t = Cx(x.re[part], x.im[part])
        pr.append(Cx(np.where(special, x.re, t.re), np.where(special, x.im, t.im)))
    out = np.zeros((NC + 1,), np.complex64)
    ore = np.zeros(NC + 1, f32)
    oim = np.zeros(NC + 1, f32)
    scs = np.concatenate([sc, np.zeros((1, 2), f32)])
    lane0 = lane == 0
    half = f32(0.5)

    def pair(b, rr, sck, sckp):
        sre, sim = b.re + rr.re, b.im + rr.im
        dre, dim = b.re - rr.re, b.im - rr.im
        xr = half * ((sre + sck[:, 1] * sim) - sck[:, 0] * dre)
        xi = half * ((dim - sck[:, 0] * sim) - sck[:, 1] * dre)
        xpr = half * ((sre + sckp[:, 1] * sim) - sckp[:, 0] * (-dre))
        xpi = half * (((-dim) - sckp[:, 0] * sim) - sckp[:, 1] * (-dre))
        return Cx(xr, xi), Cx(xpr, xpi)

    for r in range(8):
        k = col + 64 * r
        rr = pr[7 - r]
        alt = v[0] if r == 0 else pr[8 - r]
        rr = Cx(np.where(lane0, alt.re, rr.re), np.where(lane0, alt.im, rr.im))
        kp = NC - k
        xk, xkp = pair(v[r], rr, scs[k], scs[kp])
        if r == 0:
            xkp = Cx(np.where(lane0, v[0].re - v[0].im, xkp.re), np.where(lane0, f32(0), xkp.im))
        ore[k], oim[k] = xk.re, xk.im
        ore[kp], oim[kp] = xkp.re, xkp.im
    xk, _ = pair(v[8], v[8], scs[np.full(L, NC // 2)], scs[np.full(L, NC // 2)])
    ore[NC // 2], oim[NC // 2] = xk.re[0], xk.im[0]
    out.real, out.imag = ore, oim
    return out
