"""libthesia's host tables are bit-identical to the oracle (CPU only, no GPU calls)."""
import numpy as np
import pytest

import oracle_ffi as O
import thesia


@pytest.mark.parametrize("size", [2, 3, 4, 5, 320, 640, 884, 960, 1764, 1920, 2048, 4096])
@pytest.mark.parametrize("sym", [False, True])
def test_hann_bit_exact(size, sym):
    assert np.array_equal(thesia.windows.hann(size, sym), O.hann(size, sym))


def test_proper_n_fft_and_track_params():
    for w in list(range(1, 5000, 7)) + [320, 884, 1920, 1764, 2048, 4096]:
        assert thesia.utils.calc_proper_n_fft(w) == O.calc_proper_n_fft(w)
    for sr in [8000, 11025, 16000, 22050, 24000, 32000, 44100, 48000, 88200, 96000]:
        assert thesia.utils.track_params(sr) == O.track_params(sr)
    assert thesia.utils.track_params(22050) == (884, 221, 1024)  # 220.5 rounds away from 0


def test_hz_mel_bit_exact():
    rng = np.random.default_rng(0)
    for f in np.concatenate([rng.uniform(0, 48000, 500), [0.0, 999.99, 1000.0, 1000.01, 24000.0]]).astype(np.float32):
        assert np.float32(thesia.mel.hz_to_mel(float(f))) == O.hz_to_mel(float(f))
    for m in rng.uniform(0, 60, 300).astype(np.float32):
        assert np.float32(thesia.mel.mel_to_hz(float(m))) == O.mel_to_hz(float(m))


@pytest.mark.parametrize("sr,n_fft,n_mel", [(24000, 2048, 80), (48000, 2048, 128), (8000, 512, 40),
                                            (44100, 1024, 1), (22050, 256, 64), (16000, 4096, 200)])
def test_mel_fb_bit_exact(sr, n_fft, n_mel):
    a = thesia.mel.calc_mel_fb(sr, n_fft, n_mel)
    b = O.calc_mel_fb(sr, n_fft, n_mel)
    assert np.array_equal(a, b)
    a = thesia.mel.calc_mel_fb(sr, n_fft, n_mel, fmin=30.0, fmax=sr / 3, do_norm=False)
    b = O.calc_mel_fb(sr, n_fft, n_mel, fmin=30.0, fmax=sr / 3, do_norm=False)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("sr", [8000, 16000, 22050, 24000, 44100, 48000])
@pytest.mark.parametrize("n_fft", [256, 512, 1024, 2048])
def test_mel_fb_default_bit_exact(sr, n_fft):
    a = thesia.mel.calc_mel_fb_default(sr, n_fft)
    b = O.calc_mel_fb_default(sr, n_fft)
    assert a.shape == b.shape and np.array_equal(a, b)


def test_frame_count_matches_reference_construction():
    rng = np.random.default_rng(3)
    for _ in range(4000):
        win = int(rng.integers(1, 200))
        hop = int(rng.integers(1, 2 * win + 1))
        n = int(rng.integers(0, 600))
        assert thesia.utils.stft_n_frames(n, win, hop) == O.stft_n_frames(n, win, hop), (n, win, hop)


def test_colormap():
    cm = thesia.get_colormap()
    assert len(cm) == 30 and bytes(O.COLORMAP.ravel()) == cm
