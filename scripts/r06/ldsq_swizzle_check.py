import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from stftq_model import schedule, GEOM
SW = {128: ((5, 10, 0, 0, 0), (4, 0, 0, 0, 0)), 256: ((5, 10, 0, 0, 0), (1, 2, 0, 0, 0)), 512: ((4, 9, 6, 0, 0), (1, 2, 4, 0, 0))}
def swzq(NC, zr, x):
    g = SW[NC][1 if zr else 0]
    o = x
    for h in range(5):
        if (x >> (4 + h)) & 1:
            o ^= g[h]
    return o
def lay_m(loc, j, r, B):
    m = 0
    for b in range(B):
        k, bit = loc[b]
        m |= (((j >> bit) & 1) if k == "l" else ((r >> bit) & 1)) << b
    return m
for NC in (128, 256, 512):
    L, P, levels, pbit = schedule(NC)
    B = NC.bit_length() - 1; nl = L.bit_length() - 1
    init = {b: ("l", b) if b < nl else ("r", b - nl) for b in range(B)}
    prev = init; ok = True
    rbase = 128 * 7
    for t, lev in enumerate(levels):
        sw = lev["swaps"]; perm = len(sw) > 0 and all(x == 4 for x, _ in sw)
        if sw and not perm:
            mem = {}
            for j in range(L):
                lm = 0
                for b in range(B):
                    if prev[b][0] == "l":
                        lm ^= swzq(NC, False, 1 << b) if (j >> prev[b][1]) & 1 else 0
                wb = rbase + 8 * lm
                for r in range(P):
                    rm = sum((((r >> prev[b][1]) & 1) << b) for b in range(B) if prev[b][0] == "r")
                    f = swzq(NC, False, rm)
                    a = (wb ^ (8 * (f & 15))) + 8 * (f & ~15)
                    m = lay_m(prev, j, r, B)
                    assert a not in mem, ("collision", NC, t)
                    mem[a] = m
            new = lev["loc"]
            for j in range(L):
                lm = 0
                for b in range(B):
                    if new[b][0] == "l":
                        lm ^= swzq(NC, False, 1 << b) if (j >> new[b][1]) & 1 else 0
                rb = rbase + 8 * lm
                for r in range(P):
                    rm = sum((((r >> new[b][1]) & 1) << b) for b in range(B) if new[b][0] == "r")
                    f = swzq(NC, False, rm)
                    a = (rb ^ (8 * (f & 15))) + 8 * (f & ~15)
                    if mem.get(a) != lay_m(new, j, r, B):
                        ok = False
        prev = lev["loc"]
    print(NC, "relayouts", ok)
    # Z
    loc = levels[-1]["loc"]; mem = {}
    for j in range(L):
        lp = 0
        for b in range(B):
            if loc[b][0] == "l":
                lp ^= swzq(NC, True, 1 << pbit[b]) if (j >> loc[b][1]) & 1 else 0
        zb = rbase + 8 * lp
        for r in range(P):
            rp = sum((((r >> loc[b][1]) & 1) << pbit[b]) for b in range(B) if loc[b][0] == "r")
            f = swzq(NC, True, rp)
            a = (zb ^ (8 * (f & 15))) + 8 * (f & ~15)
            p = 0
            for b in range(B):
                k, bit = loc[b]
                p |= (((j >> bit) & 1) if k == "l" else ((r >> bit) & 1)) << pbit[b]
            mem[a] = p
    ok = True
    for j in range(L):
        l0 = j == 0
        sm = lambda x: x ^ (SW[NC][1][0] if (x & 16) else 0)
        kb = rbase + 8 * sm(j)
        pb = rbase + 8 * (L if l0 else sm(L - j))
        for i in range(P // 2):
            fk = swzq(NC, True, L * i)
            cp = NC - L * (i + 1)
            xp = 8 * (swzq(NC, True, cp) & 15); xp0 = 8 * (swzq(NC, True, cp + L) & 15)
            ak = (kb ^ (8 * (fk & 15))) + 8 * (fk & ~15)
            ap = (pb ^ (xp0 if l0 else xp)) + 8 * cp
            k = j + L * i; kp = (NC - k) & (NC - 1)
            if mem.get(ak) != k: ok = False; print("k", NC, j, i, mem.get(ak), k)
            if not (l0 and i == 0) and mem.get(ap) != kp: ok = False; print("kp", NC, j, i, mem.get(ap), kp)
    ah = rbase + 8 * swzq(NC, True, NC // 2)
    print(NC, "Z/untangle", ok, mem.get(ah) == NC // 2)
