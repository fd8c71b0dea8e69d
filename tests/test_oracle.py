"""The oracle (oracle/thesia_oracle.c) pinned against the reference's own tests and fp64."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O


@pytest.fixture(scope="module")
def kats(golden_dir):
    with open(os.path.join(golden_dir, "kats.json")) as f:
        return json.load(f)


def test_hann_kat(kats):  # windows.rs:35-38
    assert O.hann(4).tolist() == kats["hann_4_periodic"]


def test_rfft_impulse_kat(kats):  # utils.rs:117-123
    x = np.zeros(4, np.float32)
    x[0] = 1
    got = O.rfft(x)
    assert [[float(v.real), float(v.imag)] for v in got] == kats["rfft_impulse_4_0"]


def test_pad_kats(kats):  # utils.rs:125-140
    k = kats["pad_reflect"]
    assert O.pad_reflect(np.array(k["input"], np.float32), *k["pad"]).tolist() == k["expected"]
    k = kats["pad_constant"]
    row = O.pad_constant(np.array([1.0], np.float32), 1, 2, 10.0)  # axis-0 pad of a 1-row array
    assert row.tolist() == [10.0, 1.0, 10.0, 10.0]
    with pytest.raises(ValueError):
        O.pad_reflect(np.array([1, 2], np.float32), 2, 0)  # ndarray slice panic


def test_stft_impulse_kat(kats):  # lib.rs:491-514 (exact assert_eq)
    k = kats["stft_impulse"]
    got = O.perform_stft(np.array(k["input"], np.float32), k["win"], k["hop"], k["n_fft"])
    exp = np.array(k["expected"], np.float64)
    assert got.shape == exp.shape[:2]
    assert np.array_equal(got.real, exp[..., 0]) and np.array_equal(got.imag, exp[..., 1])


def test_real_to_complex_kat(kats):  # realfft.rs:253-272, eps 1e-15 in f64
    k = kats["real_to_complex"]
    x = np.zeros(k["n"])
    for i, v in k["spikes"]:
        x[i] = v
    a = O.rfft(x, np.float64)
    b = O.cfft(x.astype(np.complex128), np.float64)
    assert np.abs(a - b[: k["n"] // 2 + 1]).max() <= k["eps"]


def test_mel_hz_kat(kats):  # mel.rs:107-113
    k = kats["mel_hz"]
    for f, m in k["hz_to_mel"]:
        assert abs(O.hz_to_mel(f, np.float64) - m) <= k["eps"]
    for m, f in k["mel_to_hz"]:
        assert abs(O.mel_to_hz(m, np.float64) - f) <= k["eps"]


def test_mel_works_is_stale_slaney(kats):
    """mel.rs:115-133's golden matches librosa Slaney normalisation, not the code's unit-sum
    normalisation: the triangle shapes are pinned through the Slaney rescale."""
    k = kats["mel_works_stale_slaney"]
    fb = O.calc_mel_fb(k["sr"], k["n_fft"], k["n_mel"], do_norm=False, dtype=np.float64)
    lo, hi = O.hz_to_mel(0.0, np.float64), O.hz_to_mel(k["sr"] / 2, np.float64)
    mels = lo + (hi - lo) / (k["n_mel"] + 1) * np.arange(k["n_mel"] + 2)
    hz = np.array([O.mel_to_hz(m, np.float64) for m in mels])
    slaney = fb * (2.0 / (hz[2:] - hz[:-2]))[None, :]
    assert np.abs(slaney[:8, 0] - np.array(k["first8_of_filter0"])).max() <= k["eps"]
    unit_sum = O.calc_mel_fb(k["sr"], k["n_fft"], k["n_mel"], dtype=np.float64)
    assert np.abs(unit_sum[:8, 0] - np.array(k["first8_of_filter0"])).max() > 1e-3  # stale


@pytest.mark.parametrize("sr", [400, 800, 1000, 2000, 4000, 8000, 16000, 24000, 44100, 48000,
                                88200, 96000])
def test_mel_default_property(sr, kats):  # mel.rs:135-165: the reference's whole grid
    k = kats["mel_default_property"]
    assert sr in k["srs"]
    for e in range(*k["n_fft_exp"]):  # n_fft 2^5 .. 2^14
        n_fft = 2 ** e
        fb = O.calc_mel_fb_default(sr, n_fft)
        assert (fb.sum(axis=0) > 0).all()
        if fb.shape[1] == fb.shape[0]:
            continue
        fail = O.calc_mel_fb(sr, n_fft, fb.shape[1] + 1)
        assert (fail.sum(axis=0) == 0).any()


@pytest.mark.parametrize("n", [4, 8, 16, 64, 256, 1024, 2048, 4096, 8192])
def test_rfft_vs_fp64(n):
    x = np.random.default_rng(n).standard_normal(n)
    ref = np.fft.rfft(x)
    assert np.abs(O.rfft(x, np.float64) - ref).max() <= 1e-12 * n
    err = np.abs(O.rfft(x.astype(np.float32)) - ref).max() / np.abs(ref).max()
    assert err < 5e-7


def test_uniform_rule_equals_literal_framing():
    """The GPU kernels frame with the uniform reflect rule; it reproduces the reference's
    front / middle / back construction (lib.rs:410-435) exactly."""
    rng = np.random.default_rng(0)
    checked = 0
    for _ in range(2500):
        win = int(rng.integers(2, 96))
        hop = int(rng.integers(1, win + 1))
        n = int(rng.integers(max(win - 1, 1), 400))
        n_fft = win + int(rng.integers(0, 6))
        if O.stft_n_frames(n, win, hop) == 0:
            continue
        x = rng.standard_normal(n).astype(np.float32)
        a = O.frames(x, win, hop, n_fft, rule="literal")
        b = O.frames(x, win, hop, n_fft, rule="uniform")
        assert a.shape == b.shape and np.array_equal(a, b), (n, win, hop, n_fft)
        assert a.shape[0] == (n + 2 * (win // 2) - win) // hop + 1
        checked += 1
    assert checked > 2000


def test_perform_stft_vs_fp64_dft():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(5000).astype(np.float32)
    win, hop, n_fft = 1920, 480, 2048
    got = O.perform_stft(x, win, hop, n_fft)
    fr = O.frames(x, win, hop, n_fft).astype(np.float64)
    ref = np.fft.rfft(fr, axis=1)
    err = (np.abs(got - ref).max(axis=1) / np.abs(ref).max(axis=1)).max()
    assert err < 1e-6


def test_db_and_colormap_semantics():
    x = np.array([0.0, 1e-20, 1e-18, 1.0, 10.0], np.float32)
    db = O.amp_to_db_default(x)
    assert db[0] == db[1] == db[2] == np.float32(20.0) * np.log10(np.float32(1e-18))
    assert db[3] == 0.0 and db[4] == 20.0
    with pytest.raises(ValueError):
        O.amp_to_db_default(np.array([-1.0], np.float32))  # decibel.rs:34 assert
    c, p = O.grey_to_color(0.0)
    assert c.tolist() == [0, 0, 4] and not p
    c, p = O.grey_to_color(0.95)
    assert c.tolist() == [252, 255, 164]
    c, p = O.grey_to_color(-0.1)
    assert p  # display.rs:25 would panic


def test_resize_identity_weights_sum_to_one():
    rng = np.random.default_rng(2)
    img = rng.random((17, 29)).astype(np.float32)
    out = O.resize_lanczos3(img, 11, 40)
    assert out.shape == (40, 11)
    const = np.full((17, 29), 0.5, np.float32)
    assert np.abs(O.resize_lanczos3(const, 13, 7) - 0.5).max() < 1e-6


@pytest.mark.parametrize("channels", [1, 2])
def test_track_spec_is_the_composition(channels):
    """or_track_spec_f32 (the CPU baseline's one call per track, one FFT plan per track as
    lib.rs:459-467) equals the composition of the oracle's functions bit for bit."""
    rng = np.random.default_rng(channels)
    pcm = (rng.standard_normal((30011, channels)) * 0.3).astype(np.float32)
    mono = np.zeros(pcm.shape[0], np.float32)
    for c in range(channels):
        mono = (mono + pcm[:, c]).astype(np.float32)
    X = O.perform_stft(mono, 2048, 512, 2048)
    fb = O.calc_mel_fb(48000, 2048, 128)
    cases = {O.TRACK_MAG: O.norm(X), O.TRACK_MEL_DB: O.amp_to_db_default(O.dot(O.norm(X), fb)),
             O.TRACK_AMP_DB: O.amp_to_db_default(O.norm(X)),
             O.TRACK_POWER_DB: O.power_to_db_default(O.norm_sqr(X))}
    for kind, ref in cases.items():
        got = O.track_spec(pcm, 2048, 512, 2048, kind, fb if kind == O.TRACK_MEL_DB else None)
        assert got.view(np.uint32).tolist() == ref.view(np.uint32).tolist(), kind
