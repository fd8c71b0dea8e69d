import os
import sys, itertools
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stftq_model import schedule, GEOM
import ldsq_conflict_model as S

def rank2(vecs):
    rows = list(vecs); r = 0
    for bit in range(16):
        piv = [v for v in rows if (v >> bit) & 1]
        if not piv: continue
        p = piv[0]; rows.remove(p); rows = [v ^ p if (v >> bit) & 1 else v for v in rows]; r += 1
    return r

def lin(g, m, nlow=4):
    # f(m) = m ^ sum over high bits h of g[h] (g[h]: 4-bit vector)
    out = m
    hi = m >> nlow
    for h, vec in enumerate(g):
        if (hi >> h) & 1:
            out ^= vec
    return out

def layouts(NC):
    L, P, levels, pbit = schedule(NC)
    B = NC.bit_length() - 1
    nl = L.bit_length() - 1
    init = {b: ("l", b) if b < nl else ("r", b - nl) for b in range(B)}
    rel = []  # (write loc, read loc) per LDS relayout
    prev = init
    for t, lev in enumerate(levels):
        sw = lev["swaps"]
        perm = len(sw) > 0 and all(x == 4 for x, _ in sw)
        if sw and not perm:
            rel.append((prev, lev["loc"]))
        prev = lev["loc"]
    return L, B, rel, levels[-1]["loc"], pbit

def ok_span(g, bitsvecs, nfb):
    # images of the spanning m-vectors under f, projected to the low nfb bits, independent?
    imgs = [lin(g, v) & ((1 << nfb) - 1) for v in bitsvecs]
    return rank2(imgs) == len(bitsvecs)

def search(NC):
    L, B, rel, zloc, pbit = layouts(NC)
    nhi = B - 4
    conds = []
    for wl, rl in rel:
        # write groups: 16 lanes = lane bits 0-3
        conds.append(([1 << b for b in range(B) if wl[b][0] == "l" and wl[b][1] < 4], 4))
        if L == 16:
            conds.append(([1 << b for b in range(B) if rl[b][0] == "l"], 4))
        else:
            conds.append(([1 << b for b in range(B) if rl[b][0] == "l"], 5))
    best = None
    for g in itertools.product(range(16), repeat=nhi):
        if all(ok_span(g, v, n) for v, n in conds):
            best = g; break
    # Z: p-space; write spans = final layout lane bits mapped to p bits (16-lane groups)
    zconds = [([1 << pbit[b] for b in range(B) if zloc[b][0] == "l" and zloc[b][1] < 4], 4)]
    zbest = None
    for g in itertools.product(range(16), repeat=nhi):
        if all(ok_span(g, v, n) for v, n in zconds):
            zbest = g; break
    return best, zbest

if __name__ == "__main__":
    for NC in (128, 256, 512):
        print(NC, search(NC))
