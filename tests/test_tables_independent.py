"""libthesia's host tables against an independent float64 numpy restatement of the reference
formulas (windows.rs:7-30, mel.rs:8-99), not the C oracle: the bit-exact tests in
test_tables.py compare two restatements of the same f32 code (the library's and the oracle's),
so this file pins both to the mathematics the reference writes down, within the f32 rounding of
its evaluation order. CPU only."""
import math

import numpy as np
import pytest

import thesia

# mel.rs:8-11
MIN_LOG_MEL, MIN_LOG_HZ, LOGSTEP, LINEARSCALE = 15.0, 1000.0, 0.06875177742094912, 200.0 / 3.0


def _hann64(size, symmetric):
    size2 = size if symmetric else size + 1  # windows.rs:10
    i = np.arange(size2, dtype=np.float64)
    x = math.pi * i / (size2 - 1)
    return (0.5 - 0.5 * np.cos(2.0 * x))[:size]


def _hz_to_mel64(f):
    f = np.asarray(f, np.float64)
    return np.where(f < MIN_LOG_HZ, f / LINEARSCALE,
                    MIN_LOG_MEL + np.log(np.maximum(f, 1e-300) / MIN_LOG_HZ) / LOGSTEP)


def _mel_to_hz64(m):
    m = np.asarray(m, np.float64)
    return np.where(m < MIN_LOG_MEL, LINEARSCALE * m, MIN_LOG_HZ * np.exp(LOGSTEP * (m - MIN_LOG_MEL)))


def _linspace(a, b, n):  # ndarray 0.14 Array::linspace: start + step * i, step = (b - a) / (n - 1)
    step = (b - a) / (n - 1) if n > 1 else 0.0
    return a + step * np.arange(n, dtype=np.float64)


def _mel_fb64(sr, n_fft, n_mel, fmin=0.0, fmax=None, do_norm=True):
    nyq = sr / 2.0
    fmax = nyq if fmax is None else fmax
    lin = _linspace(0.0, nyq, n_fft // 2 + 1)
    mf = _mel_to_hz64(_linspace(float(_hz_to_mel64(fmin)), float(_hz_to_mel64(fmax)), n_mel + 2))
    w = np.zeros((lin.size, n_mel))
    for m in range(n_mel):
        lo, c, hi = mf[m], mf[m + 1], mf[m + 2]
        up = (lin > lo) & (lin < c)
        dn = (lin > c) & (lin < hi)
        w[up, m] = (lin[up] - lo) / (c - lo)
        w[lin == c, m] = 1.0
        w[dn, m] = (hi - lin[dn]) / (hi - c)
        if do_norm:
            w[:, m] /= max(w[:, m].sum(), np.finfo(np.float32).eps)
    return w


@pytest.mark.parametrize("size", [2, 3, 5, 320, 640, 884, 960, 1764, 1920, 2048, 4096])
@pytest.mark.parametrize("sym", [False, True])
def test_hann_vs_float64_formula(size, sym):
    got = thesia.windows.hann(size, sym).astype(np.float64)
    ref = _hann64(size, sym)
    # f32 evaluation of pi * i / (size2 - 1), cos(2x), 0.5 - 0.5 c: a few f32 ulps of 1
    assert np.max(np.abs(got - ref)) <= 4e-7 * max(1.0, size / 2048.0)


def test_hz_mel_vs_float64_formula():
    rng = np.random.default_rng(1)
    f = np.concatenate([rng.uniform(0, 48000, 400), [0.0, 500.0, 999.9, 1000.0, 1000.1, 24000.0]])
    got = np.array([thesia.mel.hz_to_mel(float(np.float32(v))) for v in f])
    ref = _hz_to_mel64(f.astype(np.float32).astype(np.float64))
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)) <= 2e-6
    m = rng.uniform(0, 60, 300)
    got = np.array([thesia.mel.mel_to_hz(float(np.float32(v))) for v in m])
    ref = _mel_to_hz64(m.astype(np.float32).astype(np.float64))
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0)) <= 4e-6


@pytest.mark.parametrize("sr,n_fft,n_mel", [(48000, 2048, 128), (24000, 2048, 80), (8000, 512, 40),
                                            (22050, 1024, 64), (44100, 2048, 347), (16000, 4096, 200)])
def test_mel_fb_vs_float64_formula(sr, n_fft, n_mel):
    got = thesia.mel.calc_mel_fb(sr, n_fft, n_mel).astype(np.float64)
    ref = _mel_fb64(sr, n_fft, n_mel)
    assert got.shape == ref.shape
    # every filter: same support (up to a bin whose f32 weight rounds to or from zero at the
    # triangle's ends), weights within the f32 rounding of the linspace / mel / division chain;
    # the narrowest filters (1-2 bins at n_mel 347) divide by band edges a few Hz apart computed
    # from f32 frequencies of ~1e3 Hz, so their f32 weights carry ~1e-4 relative cancellation
    scale = ref.max(axis=0)
    err = np.abs(got - ref) / scale
    assert err.max() <= 2e-4, float(err.max())
    support_diff = ((got > 0) != (ref > 0)) & (np.maximum(got, ref) > 1e-4 * scale)
    assert not support_diff.any(), np.argwhere(support_diff)[:5]
    # unit-sum normalisation (mel.rs:80-82)
    assert np.allclose(got.sum(axis=0), 1.0, atol=2e-6)


@pytest.mark.parametrize("sr", [8000, 16000, 22050, 24000, 44100, 48000])
@pytest.mark.parametrize("n_fft", [256, 512, 1024, 2048, 4096])
def test_default_n_mel_is_the_largest_without_an_empty_filter(sr, n_fft):
    """mel.rs:87-99 independently: starting from floor(2 mel(sr/2) / mel(sr/n_fft) - 1) capped at
    F, the first n_mel whose float64 filterbank has no empty filter: the library's default table
    has exactly that n_mel at every viewer rate and n_fft 256..4096."""
    got = thesia.mel.calc_mel_fb_default(sr, n_fft).shape[1]
    n = int(2.0 * _hz_to_mel64(sr / 2.0) / _hz_to_mel64(sr / n_fft) - 1.0)
    n = min(n, n_fft // 2 + 1)
    while not (_mel_fb64(sr, n_fft, n).sum(axis=0) > 0).all():
        n -= 1
    assert got == n, (got, n)
