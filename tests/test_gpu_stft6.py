"""stft6_kernel (one 64-lane frame per wave, 3 waves/SIMD; mel kinds at n_fft 2048) against the
oracle and against stft5.

stft6 has no |X| output kind, so its linear mel rows are checked against the oracle's dot
(lib.rs:131, the k-ascending chain) of stft5's own |X| within a relative bound: the two kernels
round their FFTs differently (f32, ~1e-7 relative), and a filter wider than stft6's cap runs as
two chains summed at the end. Its dB rows are checked against the oracle's full path with the
same dB tolerances as every other kernel (tolerances.py)."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine
from thesia._lib import ThesiaError
from tolerances import DB_MAX, DB_P9999, db_clamped_err
from test_gpu_mel import _run, _tracks

pytestmark = pytest.mark.gpu

# |mel6 - dot(|X5|, fb)| <= RTOL * dot(|X5|, |fb|) + ATOL * (row max): f32 FFT rounding of two
# different factorisations (each ~1e-7 of the frame's energy per bin) through a positive sum
RTOL, ATOL = 2e-5, 2e-6


# filterbanks whose 64-lane packed stream fits stft6's LDS next to its 12 frame regions (the
# mel-128 headline among them: 4 chunks of 3 steps per frame); the others run stft5 (below)
@pytest.mark.parametrize("n_mels,sr", [(128, 48000), (128, 44100), (200, 44100), (0, 48000), (130, 16000),
                                       (80, 16000), (64, 24000)])
@pytest.mark.parametrize("channels", [1, 2])
def test_stft6_mel_matches_the_dot_of_stft5_magnitude(n_mels, sr, channels):
    rng = np.random.default_rng(n_mels * 11 + channels + sr)
    tracks = _tracks(rng, channels, engine.IN_F32, [2047, 2048 * 5 + 17, 512 * 41 + 3, 30000])
    mag, _ = _run(engine.OUT_MAG, tracks, channels, engine.IN_F32, kernel=5, max_blocks=5)
    mel, plan = _run(engine.OUT_MEL, tracks, channels, engine.IN_F32, n_mels=n_mels, sr=sr,
                     kernel=6, max_blocks=5)
    fb = O.calc_mel_fb(sr, 2048, n_mels) if n_mels else O.calc_mel_fb_default(sr, 2048)
    assert plan.row_bins == fb.shape[1]
    ref = O.dot(mag, fb).astype(np.float64)
    bound = RTOL * (mag.astype(np.float64) @ np.abs(fb).astype(np.float64)) + \
        ATOL * np.abs(ref).max(axis=1, keepdims=True)
    err = np.abs(mel.astype(np.float64) - ref)
    assert np.isfinite(mel).all()
    assert (err <= bound).all(), (err.max(), np.unravel_index(np.argmax(err - bound), err.shape))


@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap", [0, 1])
@pytest.mark.parametrize("max_blocks", [1, 3, 0])
def test_stft6_mel_db_against_oracle_with_track_edges(channels, fmt, gap, max_blocks):
    """Long frame streams (1 or 3 blocks: each wave walks many frames across track ends; the
    ring shift + prefetch, the reflect-padded frames, odd gaps that break the pair alignment) and
    the default grid."""
    rng = np.random.default_rng(29 + channels + 5 * fmt + gap + max_blocks)
    lens = [2047, 2048, 2049, 6151, 512 * 37, 20483, 512 * 60 + 5]
    tracks = _tracks(rng, channels, fmt, lens)
    got, _ = _run(engine.OUT_MEL_AMP_DB, tracks, channels, fmt, n_mels=128, gap=gap,
                  max_blocks=max_blocks, kernel=6)
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


@pytest.mark.parametrize("mel_path", [2, 3])
@pytest.mark.parametrize("out_shift", [0, 4, 8])
def test_stft6_mel_paths_and_output_alignment(mel_path, out_shift):
    """Both chunk widths of stft6's packed stream, aligned rows (8-byte stores) and misaligned
    ones (lane-wise stores): identical bits between the store methods, and within the dB
    tolerance of stft5."""
    rng = np.random.default_rng(7 + mel_path + out_shift)
    tracks = _tracks(rng, 2, engine.IN_F32, [2048 * 7 + 5, 512 * 33 + 1, 30011])
    try:
        db6, _ = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=128, kernel=6,
                      max_blocks=3, mel_path=mel_path, out_shift=out_shift)
    except ThesiaError as e:  # this chunk width does not fit LDS / the filterbank
        pytest.skip(str(e))
    db6a, _ = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=128, kernel=6,
                   max_blocks=3, mel_path=mel_path)
    np.testing.assert_array_equal(db6, db6a)
    db5, _ = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=128, kernel=5, max_blocks=3)
    mx, p = db_clamped_err(db6, db5)
    assert mx <= DB_MAX and p <= DB_P9999, (mx, p)


@pytest.mark.parametrize("n_mels,sr", [(40, 48000), (10, 48000), (0, 22050)])
def test_stft6_declines_filterbanks_beyond_its_lds(n_mels, sr):
    """Few wide filters (40 or 10 over 24 kHz: 12-35 chunks per lane even in two pieces) or many
    filters (the default 617 at 22.05 kHz) make the packed stream too big for the LDS left by
    twelve frame regions: forcing stft6 is an error, and the automatic choice is stft5."""
    x = np.zeros((4096, 2), np.float32)
    with pytest.raises(ThesiaError):
        _run(engine.OUT_MEL, [x], 2, engine.IN_F32, n_mels=n_mels, sr=sr, kernel=6)
    _run(engine.OUT_MEL, [x], 2, engine.IN_F32, n_mels=n_mels, sr=sr, kernel=0)
    from test_gpu_mel import _LAST
    assert _LAST["kernel"] == 5


def test_stft6_declines_what_it_cannot_run():
    """Forcing stft6 on a kind / filterbank it does not cover is an error, not a silent
    fallback: linear kinds, and a custom filterbank whose band is wider than its packed stream."""
    x = np.zeros((4096, 2), np.float32)
    with pytest.raises(ThesiaError):
        _run(engine.OUT_AMP_DB, [x], 2, engine.IN_F32, kernel=6)
    fb = np.zeros((1025, 4), np.float32)
    fb[:, 0] = 1e-3  # 1025 bins in one filter: 129 chunks > 64
    with pytest.raises(ThesiaError):
        _run(engine.OUT_MEL, [x], 2, engine.IN_F32, mel_fb=fb, kernel=6)
