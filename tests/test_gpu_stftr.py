"""The reference-order STREAMING kernel (stftr_kernel, batch kernel 7) against the oracle, bit for
bit, at the canonical n_fft 2048 geometry (win = n_fft, hop = n_fft / 4: BASELINE.json C2-C4).

stftr computes every f32 operation of the reference path in the reference's order -- rustfft
4.0 Radix4 as restated in oracle/thesia_oracle.c (prepare_radix4 positions, Butterfly4 base,
butterfly_4 levels with table twiddles, num-complex products), the realfft untangle
(realfft.rs:142-157), glibc hypotf / log10f (exact_math.hpp), the k-ascending mel fma chain --
with the streaming data movement (register ring, hop loads, streams across track ends). So every
output kind must be array_equal to the oracle, on any track layout: odd element offsets
(per-frame reloads), the shortest legal tracks, streams walking hundreds of frames through one
block, mono / stereo, f32 / s16."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine

pytestmark = pytest.mark.gpu

N_FFT, WIN, HOP = 2048, 2048, 512


def _fold(t):  # lib.rs:42 channel sum
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _ref_input(t, fmt):
    x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
    return _fold(x.astype(np.float32))


def _tracks(rng, lens, channels, fmt, wide=False):
    out = []
    for n in lens:
        if fmt == engine.IN_S16:
            out.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            s = np.float32(10.0) ** rng.uniform(-6, 0) if wide else np.float32(0.3)
            out.append((rng.standard_normal((n, channels)) * s).astype(np.float32))
    return out


def _run(kind, tracks, channels, fmt, gap=0, max_blocks=0, n_mels=0, sr=48000, kernel=7):
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
    plan = engine.Plan(N_FFT, WIN, HOP, kind, sr=sr, n_mels=n_mels)
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


def _check(kind, tracks, rows, fmt, fb=None):
    for i, (t, got) in enumerate(zip(tracks, rows)):
        w = (O.hann(WIN) / np.float32(N_FFT)).astype(np.float32)
        want = _want(kind, O.perform_stft(_ref_input(t, fmt), WIN, HOP, N_FFT, window=w), fb)
        assert got.shape == want.shape, (i, got.shape, want.shape)
        bad = got.view(np.uint32) != want.view(np.uint32)
        assert not bad.any(), (i, int(bad.sum()), np.argwhere(bad)[:5].tolist(),
                               float(np.abs(got.astype(np.complex128) - want).max()))


KINDS = [engine.OUT_COMPLEX, engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap,max_blocks", [(0, 0), (3, 1)])
def test_linear_kinds_bit_exact(kind, channels, fmt, gap, max_blocks):
    rng = np.random.default_rng(kind * 17 + channels * 5 + fmt + gap)
    lens = [WIN - 1, WIN, WIN + 3, 5 * N_FFT + 7, 97 * HOP + 2, 211 * HOP + 11]
    tracks = _tracks(rng, lens, channels, fmt, wide=True)
    _check(kind, tracks, _run(kind, tracks, channels, fmt, gap, max_blocks), fmt)


@pytest.mark.parametrize("kind", [engine.OUT_MEL_AMP_DB, engine.OUT_MEL])
@pytest.mark.parametrize("sr,n_mels", [(48000, 128), (48000, 0), (22050, 40), (44100, 128), (16000, 64)])
@pytest.mark.parametrize("channels,fmt,gap", [(2, engine.IN_F32, 0), (1, engine.IN_S16, 3)])
def test_mel_kinds_bit_exact(kind, sr, n_mels, channels, fmt, gap):
    rng = np.random.default_rng(sr + n_mels + kind + gap)
    lens = [WIN - 1, 7 * N_FFT + 5, 133 * HOP + 9]
    tracks = _tracks(rng, lens, channels, fmt, wide=True)
    fb = O.calc_mel_fb(sr, N_FFT, n_mels) if n_mels else O.calc_mel_fb_default(sr, N_FFT)
    rows = _run(kind, tracks, channels, fmt, gap, max_blocks=2, n_mels=n_mels, sr=sr)
    _check(kind, tracks, rows, fmt, fb)


def test_equals_stftx_on_the_bench_shape():
    """The bench's C4 track shape (stereo f32, 30 s at 48 kHz) on 4 tracks: kernel 7 equals the
    one-wave-per-frame reference-order kernel (9) bit for bit, rows of every frame."""
    rng = np.random.default_rng(9)
    tracks = _tracks(rng, [1_440_000] * 4, 2, engine.IN_F32)
    a = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=128, kernel=7)
    b = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=128, kernel=9)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
