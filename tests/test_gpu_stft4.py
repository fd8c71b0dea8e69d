"""stft4_kernel (one frame stream per wave, n_fft 2048): the balanced mel layout
and the output kinds against the oracle, forced against stft3_kernel on the same inputs.

The mel projection is the k-ascending fma chain of the oracle's dot (oracle/thesia_oracle.c
or_dot_f32, lib.rs:131), so for the kernel's own |X| it must match O.dot bit for bit -- for
every filter count, including several rounds of filter pairs (the default n_mel)."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine
from tolerances import DB_MAX, DB_P9999, STFT_REL, db_clamped_err, stft_frame_err

pytestmark = pytest.mark.gpu


def _run(kind, tracks, channels, fmt, n_mels=0, sr=48000, kernel=4, gap=0):
    parts, offs, off = [], [], 0
    for t in tracks:
        offs.append(off)
        parts.append(t.reshape(-1))
        off += t.size + gap
        if gap:
            parts.append(np.zeros(gap, t.dtype))
    flat = np.concatenate(parts)
    lens = [t.shape[0] for t in tracks]
    plan = engine.Plan(2048, 2048, 512, kind, sr=sr, n_mels=n_mels)
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    esz = 8 if kind == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(T * plan.row_bins * esz)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels)
    assert b.kernel == kernel
    b.run()
    engine.synchronize()
    out = dout.to_host(np.complex64 if esz == 8 else np.float32, (T, plan.row_bins))
    return out, plan


def _tracks(rng, channels, fmt, lens):
    out = []
    for n in lens:
        if fmt == engine.IN_S16:
            out.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            out.append((rng.standard_normal((n, channels)) * 0.3).astype(np.float32))
    return out


@pytest.mark.parametrize("kernel", [3, 4])
@pytest.mark.parametrize("n_mels,sr", [(128, 48000), (40, 48000), (200, 44100), (0, 48000), (0, 22050)])
@pytest.mark.parametrize("channels", [1, 2])
def test_mel_is_the_dot_of_the_kernels_own_magnitude(kernel, n_mels, sr, channels, monkeypatch):
    monkeypatch.setenv("THESIA_STFT_KERNEL", str(kernel))
    monkeypatch.setenv("THESIA_GRID", "5")
    rng = np.random.default_rng(n_mels * 7 + channels + kernel + sr)
    tracks = _tracks(rng, channels, engine.IN_F32, [2047, 2048 * 5 + 17, 512 * 41 + 3, 30000])
    mag, _ = _run(engine.OUT_MAG, tracks, channels, engine.IN_F32, kernel=kernel)
    mel, plan = _run(engine.OUT_MEL, tracks, channels, engine.IN_F32, n_mels=n_mels, sr=sr, kernel=kernel)
    fb = O.calc_mel_fb(sr, 2048, n_mels) if n_mels else O.calc_mel_fb_default(sr, 2048)
    assert plan.row_bins == fb.shape[1]
    np.testing.assert_array_equal(mel, O.dot(mag, fb))


@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap", [0, 1])
def test_mel_db_against_oracle_with_track_edges(channels, fmt, gap, monkeypatch):
    monkeypatch.setenv("THESIA_STFT_KERNEL", "4")
    monkeypatch.setenv("THESIA_GRID", "3")  # long streams: shift + prefetch across track ends
    rng = np.random.default_rng(17 + channels + 5 * fmt + gap)
    lens = [2047, 2048, 2049, 6151, 512 * 37, 20483, 512 * 60 + 5]
    tracks = _tracks(rng, channels, fmt, lens)
    got, _ = _run(engine.OUT_MEL_AMP_DB, tracks, channels, fmt, n_mels=128, gap=gap)
    fb = O.calc_mel_fb(48000, 2048, 128)
    T0 = 0
    for t in tracks:
        x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
        acc = np.zeros(x.shape[0], np.float32)
        for c in range(channels):  # lib.rs:42 channel sum
            acc = (acc + x[:, c]).astype(np.float32)
        ref = O.amp_to_db_default(O.dot(O.norm(O.perform_stft(acc, 2048, 512, 2048)), fb))
        g = got[T0:T0 + ref.shape[0]]
        T0 += ref.shape[0]
        mx, p = db_clamped_err(g, ref)
        assert mx <= DB_MAX and p <= DB_P9999, (t.shape, mx, p)


@pytest.mark.parametrize("kind", [engine.OUT_COMPLEX, engine.OUT_MAG, engine.OUT_POWER_DB, engine.OUT_AMP_DB])
def test_linear_kinds_match_stft3(kind, monkeypatch):
    """stft4 and stft3 on the same batch: both within the oracle tolerance of each other."""
    rng = np.random.default_rng(kind)
    tracks = _tracks(rng, 2, engine.IN_F32, [9000, 2048 * 7 + 5, 48000])
    monkeypatch.setenv("THESIA_STFT_KERNEL", "4")
    a, _ = _run(kind, tracks, 2, engine.IN_F32, kernel=4)
    monkeypatch.setenv("THESIA_STFT_KERNEL", "3")
    b, _ = _run(kind, tracks, 2, engine.IN_F32, kernel=3)
    if kind == engine.OUT_COMPLEX:
        assert stft_frame_err(a, b) <= 2 * STFT_REL
    elif kind == engine.OUT_MAG:
        scale = np.abs(b).max(axis=1, keepdims=True)
        assert (np.abs(a - b) <= 4 * STFT_REL * scale + 1e-30).all()
    else:
        mx, p = db_clamped_err(a, b)
        assert mx <= DB_MAX and p <= DB_P9999


@pytest.mark.parametrize("kernel", [None, 4])
def test_kernel_choice(kernel, monkeypatch):
    """stft3 by default (the faster one); stft4 only when forced."""
    if kernel:
        monkeypatch.setenv("THESIA_STFT_KERNEL", str(kernel))
    x = np.zeros((4096, 2), np.float32)
    _run(engine.OUT_MEL_AMP_DB, [x], 2, engine.IN_F32, n_mels=128, kernel=kernel or 3)
    _run(engine.OUT_POWER_DB, [x[:, :1].copy()], 1, engine.IN_F32, kernel=kernel or 3)
