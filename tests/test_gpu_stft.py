"""GPU parity of the fused STFT kernels against the oracle (through the C ABI)."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import thesia
from thesia import engine
from tolerances import STFT_REL, DB_MAX, DB_P9999, stft_frame_err, db_clamped_err

pytestmark = pytest.mark.gpu


def test_stft_impulse_kat_exact(golden_dir):  # lib.rs:491-514 assert_eq
    k = json.load(open(os.path.join(golden_dir, "kats.json")))["stft_impulse"]
    got = thesia.perform_stft(np.array(k["input"], np.float32), k["win"], k["hop"], k["n_fft"])
    exp = np.array(k["expected"], np.float64)
    assert np.array_equal(got.real, exp[..., 0]) and np.array_equal(got.imag, exp[..., 1])


def test_rfft_impulse_kat_exact():  # utils.rs:117-123: rfft(impulse(4, 0)) == [1, 1, 1]
    x = np.zeros(8, np.float32)
    x[2] = 1.0  # frame 1 of (win 4, hop 4) covers samples 2..5 (lib.rs uniform rule)
    got = thesia.perform_stft(x, 4, 4, 4, window=np.ones(4, np.float32))
    assert got[1].tolist() == [1 + 0j, 1 + 0j, 1 + 0j]


@pytest.mark.parametrize("n_fft", [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096])
def test_perform_stft_random(n_fft):
    rng = np.random.default_rng(n_fft)
    for win, hop in [(n_fft, n_fft // 4 or 1), (max(2, n_fft * 15 // 16), max(1, n_fft // 5)), (max(2, n_fft - 1), 3)]:
        n = int(rng.integers(win, 6 * win + 50))
        x = rng.standard_normal(n).astype(np.float32)
        got = thesia.perform_stft(x, win, hop, n_fft)
        ref = O.perform_stft(x, win, hop, n_fft)
        assert got.shape == ref.shape
        assert stft_frame_err(got, ref) <= STFT_REL, (n_fft, win, hop)


def test_perform_stft_custom_window_and_short_inputs():
    rng = np.random.default_rng(7)
    for n_fft, win, hop, n in [(1024, 1000, 250, 999), (512, 400, 100, 401), (2048, 1920, 480, 1919),
                               (256, 255, 17, 254), (64, 64, 1, 100)]:
        x = rng.standard_normal(n).astype(np.float32)
        w = rng.random(win).astype(np.float32)
        got = thesia.perform_stft(x, win, hop, n_fft, window=w)
        ref = O.perform_stft(x, win, hop, n_fft, window=w)
        assert got.shape == ref.shape and stft_frame_err(got, ref) <= STFT_REL


def _batch(n_fft, win, hop, output, tracks, channels=1, fmt=engine.IN_F32, n_mels=0, sr=48000):
    """Runs one batch over `tracks` (list of [n, ch] arrays) and returns per-track outputs."""
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]])
    lens = [t.shape[0] for t in tracks]
    plan = engine.Plan(n_fft, win, hop, output, sr=sr, n_mels=n_mels)
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    esz = 8 if output == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(T * plan.row_bins * esz)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels)
    b.run()
    engine.synchronize()
    out = dout.to_host(np.complex64 if esz == 8 else np.float32, (T, plan.row_bins))
    return [out[int(b.frame0[i]):int(b.frame0[i + 1])] for i in range(len(tracks))], plan


def _oracle_spec(x_mono, win, hop, n_fft, kind, fb=None):
    X = O.perform_stft(x_mono, win, hop, n_fft)
    if kind == engine.OUT_COMPLEX:
        return X
    if kind in (engine.OUT_POWER, engine.OUT_POWER_DB):
        p = O.norm_sqr(X)
        return O.power_to_db_default(p) if kind == engine.OUT_POWER_DB else p
    m = O.norm(X)
    if kind in (engine.OUT_MEL, engine.OUT_MEL_AMP_DB):
        m = O.dot(m, fb)
        return O.amp_to_db_default(m) if kind == engine.OUT_MEL_AMP_DB else m
    return O.amp_to_db_default(m) if kind == engine.OUT_AMP_DB else m


def _mono_fold(t):  # lib.rs:42 channel sum, (0 + c0) + c1 ...
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


@pytest.mark.parametrize("kind", [engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB])
@pytest.mark.parametrize("n_fft", [256, 512, 1024, 2048])
def test_batch_linear_kinds(kind, n_fft):
    rng = np.random.default_rng(11 + n_fft + kind)
    win, hop = n_fft, n_fft // 4
    tracks = [rng.standard_normal((int(rng.integers(win, 9 * win)), 1)).astype(np.float32) * 0.3 for _ in range(5)]
    outs, _ = _batch(n_fft, win, hop, kind, tracks)
    for t, got in zip(tracks, outs):
        X = O.perform_stft(t[:, 0], win, hop, n_fft)
        ref = _oracle_spec(t[:, 0], win, hop, n_fft, kind)
        if kind in (engine.OUT_MAG, engine.OUT_POWER):
            scale = np.abs(X).max(axis=1, keepdims=True) ** (2 if kind == engine.OUT_POWER else 1)
            assert (np.abs(got - ref) <= 4 * STFT_REL * scale + 1e-30).all()
        else:
            mx, p = db_clamped_err(got, ref)
            assert mx <= DB_MAX and p <= DB_P9999, (mx, p)


def test_batch_stereo_fold_f32_and_s16():
    rng = np.random.default_rng(5)
    n_fft, win, hop = 2048, 2048, 512
    i16 = [rng.integers(-20000, 20000, size=(int(rng.integers(3000, 20000)), 2)).astype(np.int16) for _ in range(4)]
    f32 = [(t.astype(np.float32) / 32768.0) for t in i16]
    outs_f, _ = _batch(n_fft, win, hop, engine.OUT_COMPLEX, f32, channels=2)
    outs_s, _ = _batch(n_fft, win, hop, engine.OUT_COMPLEX, i16, channels=2, fmt=engine.IN_S16)
    for t, gf, gs in zip(f32, outs_f, outs_s):
        ref = O.perform_stft(_mono_fold(t), win, hop, n_fft)
        assert stft_frame_err(gf, ref) <= STFT_REL
        assert np.array_equal(gf, gs)  # s16 / 32768 is exact: identical device inputs


@pytest.mark.parametrize("n_fft,sr,n_mels", [(2048, 48000, 128), (2048, 48000, 0), (1024, 22050, 0),
                                             (512, 8000, 0), (256, 16000, 40), (4096, 96000, 0)])
def test_batch_mel_db(n_fft, sr, n_mels):
    rng = np.random.default_rng(n_fft + n_mels)
    win, hop = n_fft, n_fft // 4
    tracks = [(rng.standard_normal((int(rng.integers(win, 12 * win)), 1)) * 0.2).astype(np.float32) for _ in range(4)]
    outs, plan = _batch(n_fft, win, hop, engine.OUT_MEL_AMP_DB, tracks, sr=sr, n_mels=n_mels)
    fb = O.calc_mel_fb(sr, n_fft, n_mels) if n_mels else O.calc_mel_fb_default(sr, n_fft)
    assert plan.row_bins == fb.shape[1]
    for t, got in zip(tracks, outs):
        ref = _oracle_spec(t[:, 0], win, hop, n_fft, engine.OUT_MEL_AMP_DB, fb)
        mx, p = db_clamped_err(got, ref)
        assert mx <= DB_MAX and p <= DB_P9999, (mx, p)


def test_batch_mel_linear_magnitude_close():
    rng = np.random.default_rng(9)
    n_fft, win, hop = 2048, 1920, 480
    tracks = [(rng.standard_normal((30000, 1))).astype(np.float32)]
    outs, plan = _batch(n_fft, win, hop, engine.OUT_MEL, tracks, sr=48000, n_mels=128)
    fb = O.calc_mel_fb(48000, n_fft, 128)
    ref = O.dot(O.norm(O.perform_stft(tracks[0][:, 0], win, hop, n_fft)), fb)
    rel = np.abs(outs[0] - ref) / (np.abs(ref).max(axis=1, keepdims=True) + 1e-30)
    assert rel.max() <= 4e-6


def test_many_tiny_tracks_and_partial_tiles():
    rng = np.random.default_rng(12)
    n_fft, win, hop = 512, 500, 125
    tracks = [rng.standard_normal((int(rng.integers(win - 1, win + 400)), 1)).astype(np.float32) for _ in range(37)]
    outs, _ = _batch(n_fft, win, hop, engine.OUT_COMPLEX, tracks)
    for t, got in zip(tracks, outs):
        ref = O.perform_stft(t[:, 0], win, hop, n_fft)
        assert got.shape == ref.shape and stft_frame_err(got, ref) <= STFT_REL


def test_full_size_properties_c4_shape():
    """Full-size (BASELINE C4 track: 48 kHz, 30 s stereo, 2048/512) checks that need no oracle
    pass: frame count, silence -> exact floor, linearity in scale by a power of two."""
    n = 1_440_000
    z = np.zeros((n, 2), np.float32)
    outs, _ = _batch(2048, 2048, 512, engine.OUT_MEL_AMP_DB, [z], channels=2, n_mels=128)
    assert outs[0].shape == (2813, 128)
    assert (outs[0] == np.float32(20.0) * np.log10(np.float32(1e-18))).all()
    x = engine.synth_pcm_host(2, 0, n, 48000).astype(np.float32) / 32768.0
    a, _ = _batch(2048, 2048, 512, engine.OUT_COMPLEX, [x], channels=2)
    b, _ = _batch(2048, 2048, 512, engine.OUT_COMPLEX, [x * 4], channels=2)
    assert np.array_equal(a[0] * 4, b[0])  # power-of-two scaling is exact through the FFT
