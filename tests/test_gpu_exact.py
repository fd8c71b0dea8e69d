"""The reference-order kernel (stftx_kernel, batch kernel 9) against the oracle, bit for bit.

The oracle restates the reference path in the reference's operation order (rustfft Radix4 as
restated in oracle/thesia_oracle.c, realfft untangle, glibc hypotf / log10f, the k-ascending
mel dot); stftx computes the same operations in the same order on the device, so every output
kind must be array_equal, and MultiTrack images (which use stftx) must equal the oracle
pipeline's bytes end to end (north_star: bit-exact u8 image buffer). Parity of the oracle's
FFT order with rustfft itself stays unpinned beyond the reference's KATs."""
import numpy as np
import pytest

import fixtures
import oracle_ffi as O
import thesia
from thesia import engine, shard

pytestmark = pytest.mark.gpu


def _fold(t):  # lib.rs:42 channel sum, (0 + c0) + c1 ...
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _run(kind, tracks, win, hop, n_fft, channels=1, fmt=engine.IN_F32, n_mels=0, sr=48000, fold=True):
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]]).astype(np.uint64)
    lens = [t.shape[0] for t in tracks]
    plan = engine.Plan(n_fft, win, hop, kind, sr=sr, n_mels=n_mels)
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    el = 8 if kind == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(max(T * plan.row_bins * el, 4))
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels,
                     fold_mono=fold, kernel=9)
    assert b.kernel == 9
    b.run()
    engine.synchronize()
    dt = np.complex64 if kind == engine.OUT_COMPLEX else np.float32
    out = dout.to_host(dt, (T, plan.row_bins))
    return [out[int(b.frame0[i]):int(b.frame0[i + 1])] for i in range(len(tracks))], plan


def _ref_input(t, fmt):
    x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
    return _fold(x.astype(np.float32))


@pytest.mark.parametrize("n_fft,win,hop", [(4, 4, 1), (4, 3, 1), (8, 8, 2), (16, 12, 5), (32, 32, 8),
                                           (64, 50, 13), (256, 256, 64), (512, 320, 80),
                                           (1024, 884, 221), (2048, 1920, 480), (2048, 2048, 512),
                                           (4096, 4096, 1024)])
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16)])
def test_complex_bit_exact(n_fft, win, hop, channels, fmt):
    rng = np.random.default_rng(n_fft * 7 + win + channels + fmt)
    lens = [max(win - 1, win // 2 + 1), win + 3, 5 * n_fft + 7, 17 * hop + 3]
    tracks = []
    for n in lens:
        if fmt == engine.IN_S16:
            tracks.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            tracks.append((rng.standard_normal((n, channels)) * 0.3).astype(np.float32))
    outs, _ = _run(engine.OUT_COMPLEX, tracks, win, hop, n_fft, channels, fmt)
    for t, got in zip(tracks, outs):
        w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
        ref = O.perform_stft(_ref_input(t, fmt), win, hop, n_fft, window=w)
        assert got.shape == ref.shape
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (
            n_fft, int((got != ref).sum()), float(np.abs(got - ref).max()))


def test_win_le_2_refused():
    # win <= 2: the reflect pad of input[..win-1] (lib.rs:413) panics for every track length
    t = np.zeros((64, 1), np.float32)
    with pytest.raises(thesia.ThesiaError):
        _run(engine.OUT_COMPLEX, [t], 2, 1, 2)


@pytest.mark.parametrize("kind", [engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB])
@pytest.mark.parametrize("n_fft,win,hop", [(512, 320, 80), (2048, 2048, 512), (1024, 960, 240)])
def test_linear_kinds_bit_exact(kind, n_fft, win, hop):
    rng = np.random.default_rng(kind * 31 + n_fft)
    # a wide dynamic range (quiet passages near the -120 dB floor) exercises hypot and log10
    tracks = [(rng.standard_normal((n, 1)) * np.float32(10.0) ** rng.uniform(-6, 0)).astype(np.float32)
              for n in (win + 5, 40 * hop + 11)]
    outs, _ = _run(kind, tracks, win, hop, n_fft)
    for t, got in zip(tracks, outs):
        w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
        X = O.perform_stft(_fold(t), win, hop, n_fft, window=w)
        if kind == engine.OUT_MAG:
            ref = O.norm(X)
        elif kind == engine.OUT_POWER:
            ref = O.norm_sqr(X)
        elif kind == engine.OUT_AMP_DB:
            ref = O.amp_to_db_default(O.norm(X))
        else:
            ref = O.power_to_db_default(O.norm_sqr(X))
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), int((got != ref).sum())


@pytest.mark.parametrize("sr,n_fft,win,hop,n_mels", [(48000, 2048, 1920, 480, 0), (8000, 512, 320, 80, 0),
                                                     (48000, 2048, 2048, 512, 128), (22050, 1024, 884, 221, 0)])
def test_mel_db_bit_exact(sr, n_fft, win, hop, n_mels):
    rng = np.random.default_rng(sr + n_mels)
    tracks = [(rng.standard_normal((n, 1)) * 0.2).astype(np.float32) for n in (win + 1, 30 * hop + 7)]
    outs, plan = _run(engine.OUT_MEL_AMP_DB, tracks, win, hop, n_fft, n_mels=n_mels, sr=sr)
    fb = O.calc_mel_fb(sr, n_fft, n_mels) if n_mels else O.calc_mel_fb_default(sr, n_fft)
    assert plan.row_bins == fb.shape[1]
    for t, got in zip(tracks, outs):
        w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
        ref = O.amp_to_db_default(O.dot(O.norm(O.perform_stft(_fold(t), win, hop, n_fft, window=w)), fb))
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), int((got != ref).sum())


@pytest.mark.parametrize("scale", [thesia.FreqScale.Mel, thesia.FreqScale.Linear])
def test_multitrack_images_bit_exact(scale):
    """MultiTrack (lib.rs:170-298, stftx spectrograms) on the reference's sample excerpts + the
    48 kHz substitute: get_spec_image bytes == the all-oracle pipeline from the PCM."""
    z = np.load(fixtures.GOLDEN + "/samples_excerpt.npz")
    tags = ["8k", "16k", "22k05", "24k", "44k1"]
    pcm = [fixtures.s16_to_f32(z[f"pcm_{t}"]) for t in tags] + [fixtures.s16_to_f32(fixtures.c1_substitute()[:72000])]
    srs = [int(z[f"sr_{t}"]) for t in tags] + [48000]
    mt = thesia.MultiTrack(freq_scale=scale)
    mt.add_tracks_pcm(list(range(len(pcm))), pcm, srs)
    dbs = []
    for x, sr in zip(pcm, srs):
        win, hop, n_fft = O.track_params(sr)
        w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
        mag = O.norm(O.perform_stft((np.float32(0.0) + x).astype(np.float32), win, hop, n_fft, window=w))
        if scale == thesia.FreqScale.Mel:
            mag = O.dot(mag, O.calc_mel_fb_default(sr, n_fft))
        dbs.append(O.amp_to_db_default(mag))
    gmax = float(np.float32(min(max(float(d.max()) for d in dbs), 0.0)))
    gmin = float(np.float32(max(min(float(d.min()) for d in dbs), gmax - 120.0)))
    assert mt.get_max_db() == np.float32(gmax) and mt.get_min_db() == np.float32(gmin)
    for i, (x, sr, db) in enumerate(zip(pcm, srs, dbs)):
        up = shard.up_ratio(sr, max(srs), freq_scale_mel=scale == thesia.FreqScale.Mel)
        grey = O.spec_to_grey(db, up, gmax, gmin)
        for nh, pps in ((300, 100.0), (120, 37.5)):
            nwidth = int(np.float32(pps) * np.float32(len(x)) / np.float32(sr))
            img, _ = O.grey_to_rgb(grey, nwidth, nh)
            got = np.frombuffer(mt.get_spec_image(i, pps, nh), np.uint8)
            assert got.size == img.size
            diff = int((got != img.reshape(-1)).sum())
            assert diff == 0, (srs[i], nh, diff)
