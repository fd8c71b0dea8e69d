"""The reference-order streaming kernel at n_fft 256 / 512 / 1024 (stftq_kernel, batch kernel 7 at
those sizes; the C5 geometry: win = n_fft, hop = n_fft / 4) against the oracle, bit for bit.

stftq runs rustfft 4.0 Radix4 on L lanes x P registers per frame with the digit schedule of
tests/stftq_model.py (checked on the CPU against the oracle's cfft_tab), the realfft untangle
(realfft.rs:142-157), glibc hypotf / log10f (exact_math.hpp) and the k-ascending mel fma chain,
with the streaming data movement (register ring, hop loads, several frame streams per wave that
cross track ends). Every output kind must be array_equal to the oracle on any track layout."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine

pytestmark = pytest.mark.gpu


def _fold(t):  # lib.rs:42 channel sum
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _ref_input(t, fmt):
    x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
    return _fold(x.astype(np.float32))


def _tracks(rng, lens, channels, fmt):
    out = []
    for n in lens:
        if fmt == engine.IN_S16:
            out.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            s = np.float32(10.0) ** rng.uniform(-6, 0)
            out.append((rng.standard_normal((n, channels)) * s).astype(np.float32))
    return out


def _run(n_fft, kind, tracks, channels, fmt, gap=0, max_blocks=0, n_mels=0, sr=48000, kernel=7):
    parts, offs, off = [], [], 0
    for t in tracks:
        offs.append(off)
        parts.append(t.reshape(-1))
        off += t.size
        if gap:
            parts.append(np.zeros(gap, t.dtype))
            off += gap
    flat = np.concatenate(parts)
    lens = [t.shape[0] for t in tracks]
    plan = engine.Plan(n_fft, n_fft, n_fft // 4, kind, sr=sr, n_mels=n_mels)
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    el = 8 if kind == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(max(T * plan.row_bins * el, 4))
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels, fold_mono=True,
                     kernel=kernel, max_blocks=max_blocks)
    assert b.kernel == kernel
    b.run()
    engine.synchronize()
    dt = np.complex64 if kind == engine.OUT_COMPLEX else np.float32
    out = dout.to_host(dt, (T, plan.row_bins))
    rows = [out[int(b.frame0[i]):int(b.frame0[i + 1])] for i in range(len(tracks))]
    b.close()
    plan.close()
    din.close()
    dout.close()
    return rows


def _want(kind, X, fb=None):
    if kind == engine.OUT_COMPLEX:
        return X
    if kind == engine.OUT_MAG:
        return O.norm(X)
    if kind == engine.OUT_POWER:
        return O.norm_sqr(X)
    if kind == engine.OUT_AMP_DB:
        return O.amp_to_db_default(O.norm(X))
    if kind == engine.OUT_POWER_DB:
        return O.power_to_db_default(O.norm_sqr(X))
    if kind == engine.OUT_MEL:
        return O.dot(O.norm(X), fb)
    return O.amp_to_db_default(O.dot(O.norm(X), fb))


def _check(n_fft, kind, tracks, rows, fmt, fb=None):
    w = (O.hann(n_fft) / np.float32(n_fft)).astype(np.float32)
    for i, (t, got) in enumerate(zip(tracks, rows)):
        want = _want(kind, O.perform_stft(_ref_input(t, fmt), n_fft, n_fft // 4, n_fft, window=w), fb)
        assert got.shape == want.shape, (i, got.shape, want.shape)
        bad = got.view(np.uint32) != want.view(np.uint32)
        assert not bad.any(), (i, int(bad.sum()), np.argwhere(bad)[:5].tolist(),
                               float(np.abs(got.astype(np.complex128) - want).max()))


KINDS = [engine.OUT_COMPLEX, engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB]
SIZES = [256, 512, 1024]


@pytest.mark.parametrize("n_fft", SIZES)
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap,max_blocks", [(0, 0), (3, 1)])
def test_linear_kinds_bit_exact(n_fft, kind, channels, fmt, gap, max_blocks):
    rng = np.random.default_rng(n_fft + kind * 17 + channels * 5 + fmt + gap)
    hop = n_fft // 4
    lens = [n_fft - 1, n_fft, n_fft + 3, 5 * n_fft + 7, 97 * hop + 2, 211 * hop + 11, 37 * hop]
    tracks = _tracks(rng, lens, channels, fmt)
    _check(n_fft, kind, tracks, _run(n_fft, kind, tracks, channels, fmt, gap, max_blocks), fmt)


@pytest.mark.parametrize("n_fft", SIZES)
@pytest.mark.parametrize("kind", [engine.OUT_MEL_AMP_DB, engine.OUT_MEL])
@pytest.mark.parametrize("sr,n_mels", [(48000, 64), (22050, 0), (8000, 40)])
@pytest.mark.parametrize("channels,fmt,gap", [(2, engine.IN_F32, 0), (1, engine.IN_S16, 3)])
def test_mel_kinds_bit_exact(n_fft, kind, sr, n_mels, channels, fmt, gap):
    rng = np.random.default_rng(n_fft + sr + n_mels + kind + gap)
    hop = n_fft // 4
    lens = [n_fft - 1, 7 * n_fft + 5, 133 * hop + 9]
    tracks = _tracks(rng, lens, channels, fmt)
    try:
        fb = O.calc_mel_fb(sr, n_fft, n_mels) if n_mels else O.calc_mel_fb_default(sr, n_fft)
    except Exception:
        pytest.skip("no valid mel filterbank at this size")
    if fb.shape[1] == 0:
        pytest.skip("no valid mel filterbank at this size")
    rows = _run(n_fft, kind, tracks, channels, fmt, gap, max_blocks=2, n_mels=n_mels, sr=sr)
    _check(n_fft, kind, tracks, rows, fmt, fb)


@pytest.mark.parametrize("n_fft", SIZES)
def test_equals_stftx_on_long_tracks(n_fft):
    """Streams walking hundreds of frames (16 mono s16 tracks x 10 s at 16 kHz, the C5 track
    shape): kernel 7 equals the one-wave-per-frame reference-order kernel (9) bit for bit."""
    rng = np.random.default_rng(n_fft)
    tracks = _tracks(rng, [160_000] * 16, 1, engine.IN_S16)
    a = _run(n_fft, engine.OUT_AMP_DB, tracks, 1, engine.IN_S16, kernel=7)
    b = _run(n_fft, engine.OUT_AMP_DB, tracks, 1, engine.IN_S16, kernel=9)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def _same_nan_aware(got, want):
    gn, wn = np.isnan(got.view(np.float32)), np.isnan(want.view(np.float32))
    assert np.array_equal(gn, wn), int((gn != wn).sum())
    g, w = got.view(np.uint32), want.view(np.uint32)
    keep = ~gn.reshape(g.shape)
    assert np.array_equal(g[keep], w[keep]), int((g[keep] != w[keep]).sum())


@pytest.mark.parametrize("kernel", [7, 9])
@pytest.mark.parametrize("n_fft", [512, 2048])
@pytest.mark.parametrize("kind", [engine.OUT_COMPLEX, engine.OUT_MAG, engine.OUT_POWER, engine.OUT_MEL])
def test_non_finite_samples(kernel, n_fft, kind):
    """f32 tracks holding +inf / -inf / NaN samples (a float WAV can carry them): the
    reference-order kernels follow glibc's special cases (hypotf of an infinity is +inf even
    beside a NaN) -- equal to the oracle bit for bit wherever the value is not NaN, NaN exactly
    where the oracle's is. (The dB kinds are not compared: such frames hold NaN bins, on which
    the reference's amp_to_db asserts, decibel.rs:34; the engine reports them through the range
    NaN flag instead.)"""
    rng = np.random.default_rng(n_fft + kind)
    tracks = _tracks(rng, [9 * n_fft + 5, 4 * n_fft], 1, engine.IN_F32)
    tracks[0][3 * n_fft // 2, 0] = np.inf
    tracks[0][6 * n_fft, 0] = -np.inf
    tracks[1][n_fft + 7, 0] = np.nan
    fb = O.calc_mel_fb(48000, n_fft, 64) if kind == engine.OUT_MEL else None
    rows = _run(n_fft, kind, tracks, 1, engine.IN_F32, n_mels=64 if fb is not None else 0, kernel=kernel)
    w = (O.hann(n_fft) / np.float32(n_fft)).astype(np.float32)
    for t, got in zip(tracks, rows):
        with np.errstate(invalid="ignore", over="ignore"):
            want = _want(kind, O.perform_stft(_ref_input(t, engine.IN_F32), n_fft, n_fft // 4, n_fft, window=w), fb)
        assert got.shape == want.shape
        _same_nan_aware(np.ascontiguousarray(got), np.ascontiguousarray(want))
