"""The display kernels' grey quotient (csrc/display_common.hpp GreyMap): grey_px's
(db - min) / (max - min) (display.rs:44-54, an f32 division) formed as the f32 difference times
the f64 reciprocal of the f32 span, rounded once to f32, with quotients outside the normal range
divided in f32. The claim is bit equality with the f32 division for every input; this restates
the method in numpy and checks it on random and adversarial inputs (quotients next to f32
rounding midpoints, exact ties below the normal range, zero and non-finite spans)."""
import numpy as np

FLT_MIN = np.float32(1.17549435e-38)


def grey_quotient(a, b):
    """the GreyMap quotient of f32 arrays a (= db - min) and b (= max - min)"""
    with np.errstate(all="ignore"):
        r = 1.0 / b.astype(np.float64)
        q = (a.astype(np.float64) * r).astype(np.float32)
        normal = np.isfinite(q) & (np.abs(q) >= FLT_MIN)
        return np.where(normal, q, a / b)


def _same(x, y):
    return (x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))


def test_grey_quotient_random_and_midpoints():
    rng = np.random.default_rng(7)
    n = 2_000_000
    for it in range(6):
        a = rng.uniform(-5.0, 300.0, n).astype(np.float32)
        if it % 2:
            a = (np.abs(rng.standard_normal(n)) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
        b = rng.uniform(1e-3, 400.0, n).astype(np.float32)
        if it % 3 == 0:
            b = (10.0 ** rng.uniform(-20.0, 20.0, n)).astype(np.float32)
        with np.errstate(all="ignore"):
            ref = a / b
            assert _same(grey_quotient(a, b), ref).all()
            # a = RN(b x m) for the rounding midpoint m above each quotient: a / b lands next to m
            up = np.nextafter(ref, np.float32(np.inf))
            mid = ref.astype(np.float64) / 2 + up.astype(np.float64) / 2
            a2 = (b.astype(np.float64) * mid).astype(np.float32)
            assert _same(grey_quotient(a2, b), a2 / b).all()


def test_grey_quotient_subnormal_ties_and_specials():
    # exact ties exist only below the normal range: a = b x (k + 1/2) 2^-149 with a short b
    k = np.arange(1, 4096, dtype=np.float64)
    b = np.float32(3.0) * np.float32(2.0) ** np.arange(-20, 60, 7).astype(np.float32)
    a = (b[:, None].astype(np.float64) * (k[None, :] + 0.5) * 2.0 ** -149).astype(np.float32)
    bb = np.broadcast_to(b[:, None], a.shape).astype(np.float32)
    with np.errstate(all="ignore"):
        assert _same(grey_quotient(a, bb), a / bb).all()
        specials = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, 3e38], np.float32)
        sa, sb = np.meshgrid(specials, specials)
        assert _same(grey_quotient(sa, sb), sa / sb).all()


def test_dB_range_span():
    # the display's own domain: dB values against a global (max, min) pair
    rng = np.random.default_rng(11)
    db = rng.uniform(-140.0, 10.0, 4_000_000).astype(np.float32)
    for mx, mn in ((0.0, -120.0), (-3.25, -97.5), (7.1, -112.9), (0.0, 0.0)):
        a = db - np.float32(mn)
        b = np.full_like(a, np.float32(mx) - np.float32(mn))
        with np.errstate(all="ignore"):
            assert _same(grey_quotient(a, b), a / b).all()
