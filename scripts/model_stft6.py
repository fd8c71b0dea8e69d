"""Index model of stft6_kernel's FFT and untangle (numpy, float64): checks that the lane data flow
of the kernel header (16 x 16 x 4 split, two LDS transposes, co-resident untangle pairs, the
row-16 copy for the k1 = 0 partners, lane (0,0)'s special slots) reproduces the real FFT of a
2048-sample frame, and models the LDS bank slots of every transpose access.

    python scripts/model_stft6.py
"""
import numpy as np

NC = 1024
W = lambda n, N: np.exp(-2j * np.pi * n / N)


def dft(x):
    return np.fft.fft(x)


def model(frame):
    z = frame[0::2] + 1j * frame[1::2]  # realfft packing (realfft.rs:126-138), 1/2 in the window
    z = z * 0.5
    # stage 1: lane j holds z[64 n1 + j], n1 < 16; DFT-16 over n1, twiddle W_1024^{j k1}
    Y = np.zeros((64, 16), complex)
    for j in range(64):
        col = z[[64 * n1 + j for n1 in range(16)]]
        Y[j] = dft(col) * W(j * np.arange(16), NC)
    # transpose 1: lane t = (k1 = t // 4, b = t % 4) takes a[a] = Y[4a + b][k1]
    T = np.zeros((16, 4, 16), complex)  # [k1][b][c]
    for t in range(64):
        k1, b = t // 4, t % 4
        a = Y[[4 * aa + b for aa in range(16)], k1]
        Z = dft(a)  # over a -> c
        T[k1, b] = Z * W(b * np.arange(16), 64)
    # transpose 2: row r (0..15: T[r]; row 16: T[0] shifted, position p holds c = (p + 1) % 16)
    rows = np.zeros((17, 4, 16), complex)
    rows[:16] = T
    for p in range(16):
        rows[16, :, p] = T[0, :, (p + 1) % 16]
    X = np.full(NC + 1, np.nan + 0j)
    for t in range(64):
        k1, x = t // 4, t % 4
        z0 = t == 0
        for i in range(4):
            c = 4 * x + i
            own = rows[k1, :, c]                 # T[k1][b][c], b = 0..3
            par = rows[16 - k1, :, 15 - c]       # partner row, position 15 - c
            A, B, C, D = own[0] + own[2], own[1] + own[3], own[0] - own[2], own[1] - own[3]
            d0, d1 = A + B, C - 1j * D
            Ap, Bp, Cp, Dp = par[0] + par[2], par[1] + par[3], par[0] - par[2], par[1] - par[3]
            p3, p2 = Cp + 1j * Dp, Ap - Bp
            slots = [(d0, p3, k1 + 16 * c), (d1, p2, k1 + 16 * c + 256)]
            if z0 and i == 0:
                # bins 0 / N from d0; pair (256, 768); 512 with itself
                e0 = d0
                X[0] = 2 * (e0.real + e0.imag)
                X[NC] = 2 * (e0.real - e0.imag)
                slots = [(d1, p3, 256), (p2, p2, 512)]
            for bv, rv, k in slots:
                s, co = np.sin(np.pi * k / NC), np.cos(np.pi * k / NC)
                ar, ai = bv.real + rv.real, bv.imag - rv.imag
                br, bi = bv.real - rv.real, bv.imag + rv.imag
                p = co * br + s * bi
                q = co * bi - s * br
                x1 = (ar + q) + 1j * (ai - p)
                x2 = (ar - q) + 1j * (-ai - p)
                if k == 512 and z0:
                    x2 = x1
                for kk, val in ((k, x1), (NC - k, x2)):
                    if not np.isnan(X[kk]) and abs(X[kk] - val) > 1e-9:
                        raise AssertionError(("twice", kk))
                    X[kk] = val
    return X


def banks():
    # b128: 16-lane groups (kLdsG + 32 for the upper half); slot = (float offset / 4) % 16
    G = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
         [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
    G = G + [[l + 32 for l in g] for g in G]

    def b128(addr_of, name):
        worst = 0
        for g in G:
            for q in range(8):
                sl = {}
                for l in g:
                    a = addr_of(l, q)
                    if a is None:
                        continue
                    sl.setdefault((a // 4) % 16, set()).add(a)
                worst = max([worst] + [len(v) for v in sl.values()])
        print(f"{name}: worst {worst}-way")

    def b64(addr_of, name, n=16):
        worst = 0
        for half in (range(0, 32), range(32, 64)):
            for q in range(n):
                bk = {}
                for l in half:
                    a = addr_of(l, q)
                    for e in (0, 1):
                        bk.setdefault((a + e) % 64, set()).add(a)
                worst = max([worst] + [len(v) for v in bk.values()])
        print(f"{name}: worst {worst}-way")

    RS1, SEG1 = 132, 32
    # transpose 1 write: lane j = 4a + b writes complex at row k1, segment b, index a ^ 8[b>=2]
    b64(lambda j, k1: k1 * RS1 + (j % 4) * SEG1 + 2 * ((j // 4) ^ (8 if j % 4 >= 2 else 0)), "T1 write")
    b128(lambda t, q: (t // 4) * RS1 + (t % 4) * SEG1 + 4 * (q ^ (4 if t % 4 >= 2 else 0)), "T1 read")
    for RS2, SEG2 in ((136, 32), (132, 32), (140, 36), (144, 36), (148, 36), (136, 36), (152, 36)):
        print("T2", RS2, SEG2)
        # write: lane (k1, b) writes 8 float4 (complex pairs) of its segment
        b128(lambda t, q: (t // 4) * RS2 + (t % 4) * SEG2 + 4 * q, " T2 write")
        # own read: lane (k1, x), for b = q // 2: float4 2x + q % 2
        b128(lambda t, q: (t // 4) * RS2 + (q // 2) * SEG2 + 4 * (2 * (t % 4) + q % 2), " T2 own")
        b128(lambda t, q: (16 - t // 4) * RS2 + (q // 2) * SEG2 + 4 * (6 - 2 * (t % 4) + q % 2), " T2 partner")


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for _ in range(3):
        fr = rng.standard_normal(2 * NC)
        got = model(fr)
        ref = np.fft.rfft(fr)
        assert not np.isnan(got).any(), np.where(np.isnan(got))
        err = np.abs(got - ref).max() / np.abs(ref).max()
        print("max rel err", err)
        assert err < 1e-12
    banks()
