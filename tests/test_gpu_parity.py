"""Parity on the exact measured configurations and end to end.

  bench   the headline bench line's own workload and kernel: stft5_kernel on stereo f32
          interleaved tracks from the device generator bench.py uses (whose bytes must equal its
          host twin), 30 s tracks, mel-128 amp dB vs the oracle (lib.rs:112-136).
  C1      BASELINE.json configs[0]: the 48 kHz sample substitute (tests/fixtures.py), n_fft 1024
          / hop 256 / Hann, |X| (lib.rs:124) vs the oracle, the whole 2 113 529-sample track.
  E2E     PCM -> the oracle's full pipeline (STFT, |X| [, mel], dB, global range lib.rs:194-209,
          spec_to_grey display.rs:44-54, Lanczos3 + colormap display.rs:56-61) against the
          device's RGB bytes: SURVEY.md §8c (iv) allows <= 1 LSB on <= 1e-4 of the pixels.
"""
import numpy as np
import pytest

import fixtures
import oracle_ffi as O
import thesia
from thesia import engine, pipeline, shard
from tolerances import DB_MAX, DB_P9999, db_clamped_err

pytestmark = pytest.mark.gpu

E2E_MAX_LSB = 1
E2E_MAX_FRAC = 1e-4


def _rgb_diff(got: np.ndarray, ref: np.ndarray):
    """(max |diff| over channels, fraction of pixels with any channel differing)."""
    d = np.abs(got.reshape(-1, 3).astype(np.int16) - ref.reshape(-1, 3).astype(np.int16))
    per_px = d.max(axis=1)
    return int(per_px.max(initial=0)), float((per_px > 0).mean()) if per_px.size else 0.0


def test_bench_config_exact():
    """bench.py's C4 shard configuration on 3 of its tracks: same generator call, same layout,
    same plan, same kernel."""
    n_tracks, n, sr, ch = 3, 1_440_000, 48000, 2
    din = engine.DeviceBuffer(n_tracks * n * ch * 4)
    engine.synth_pcm_device(din, engine.IN_F32, ch, n_tracks, n, sr, seed=0)
    dev_pcm = din.to_host(np.float32, (n_tracks, n, ch))
    plan = engine.Plan(2048, 2048, 512, engine.OUT_MEL_AMP_DB, sr=sr, n_mels=128)
    offs = np.arange(n_tracks, dtype=np.uint64) * (n * ch)
    T = engine.Batch.frames_for(plan, [n] * n_tracks)
    assert T == 2813 * n_tracks
    dout = engine.DeviceBuffer(T * 128 * 4)
    b = engine.Batch(plan, din, offs, [n] * n_tracks, dout, input_format=engine.IN_F32, channels=ch)
    assert b.kernel == 5  # the bench's kernel (stft5_kernel, the n_fft 2048 default)
    b.run()
    engine.synchronize()
    got = dout.to_host(np.float32, (T, 128))
    fb = O.calc_mel_fb(sr, 2048, 128)
    for k in range(n_tracks):
        host = fixtures.s16_to_f32(engine.synth_pcm_host(ch, k, n, sr, seed=0))
        assert np.array_equal(dev_pcm[k].view(np.uint32), host.view(np.uint32)), k  # generator twin
        ref = O.track_spec(host, 2048, 512, 2048, O.TRACK_MEL_DB, fb)
        mx, p = db_clamped_err(got[2813 * k:2813 * (k + 1)], ref)
        assert mx <= DB_MAX and p <= DB_P9999, (k, mx, p)
    assert np.isfinite(got).all()


def test_c1_48k_substitute_1024_256_magnitude():
    x = fixtures.s16_to_f32(fixtures.c1_substitute())
    n = x.shape[0]
    plan = engine.Plan(1024, 1024, 256, engine.OUT_MAG, sr=48000)
    din = engine.DeviceBuffer.from_host(x)
    T = engine.Batch.frames_for(plan, [n])
    assert T == 8256
    dout = engine.DeviceBuffer(T * 513 * 4)
    b = engine.Batch(plan, din, [0], [n], dout)
    assert b.kernel == 3
    b.run()
    engine.synchronize()
    got = dout.to_host(np.float32, (T, 513))
    ref = O.norm(O.perform_stft(x, 1024, 256, 1024))
    scale = np.abs(ref).max(axis=1, keepdims=True)
    err = np.abs(got - ref) / np.maximum(scale, 1e-30)
    assert float(err.max()) <= 4e-6, float(err.max())  # |X| within the STFT contract (2e-6 x 2)


def _oracle_amp_db(t):
    x = (np.float32(0.0) + fixtures.s16_to_f32(t.pcm)).astype(np.float32)  # lib.rs:42 fold
    return O.track_spec(x, t.n_fft, t.n_fft // 4, t.n_fft, O.TRACK_AMP_DB)


def test_e2e_rgb_c5_generator():
    """Mixed rates and n_fft (the C5 generator): device RGB vs the all-oracle pipeline from
    the same PCM (the oracle's own dB, the oracle's own global range)."""
    tracks = pipeline.c5_tracks(12, seconds=2.0)
    nh = 200
    out = pipeline.render_tracks(tracks, px_per_sec=100.0, nheight=nh)
    ref_db = [_oracle_amp_db(t) for t in tracks]
    gmax, gmin, max_sr = shard.global_db_range(max(float(d.max()) for d in ref_db),
                                               min(float(d.min()) for d in ref_db),
                                               max(t.sr for t in tracks))
    worst, diff_px, total_px = 0, 0.0, 0
    for t, r, db in zip(tracks, out, ref_db):
        grey = O.spec_to_grey(db, shard.up_ratio(t.sr, max_sr, freq_scale_mel=False), gmax, gmin)
        img, _ = O.grey_to_rgb(grey, r.nwidth, nh)
        m, f = _rgb_diff(r.rgb, img)
        worst = max(worst, m)
        diff_px += f * img.size / 3
        total_px += img.size // 3
    assert worst <= E2E_MAX_LSB and diff_px / total_px <= E2E_MAX_FRAC, (worst, diff_px, total_px)


@pytest.mark.parametrize("fast", [False, True])
@pytest.mark.parametrize("scale", [thesia.FreqScale.Mel, thesia.FreqScale.Linear])
def test_e2e_rgb_multitrack_samples(scale, fast):
    """MultiTrack (lib.rs:170-298) on the reference's sample excerpts + the 48 kHz substitute:
    get_spec_image bytes vs the oracle pipeline from the PCM; fast = the streaming kernel at the
    viewer's geometries (thesia_mt_set_fast) instead of the reference-order one."""
    z = np.load(fixtures.GOLDEN + "/samples_excerpt.npz")
    tags = ["8k", "16k", "22k05", "24k", "44k1"]
    pcm = [fixtures.s16_to_f32(z[f"pcm_{t}"]) for t in tags] + [fixtures.s16_to_f32(fixtures.c1_substitute()[:72000])]
    srs = [int(z[f"sr_{t}"]) for t in tags] + [48000]
    mt = thesia.MultiTrack(freq_scale=scale, fast=fast)
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
    max_sr = max(srs)
    nh = 300
    worst, diff_px, total_px = 0, 0.0, 0
    for i, (x, sr, db) in enumerate(zip(pcm, srs, dbs)):
        up = shard.up_ratio(sr, max_sr, freq_scale_mel=scale == thesia.FreqScale.Mel)
        grey = O.spec_to_grey(db, up, gmax, gmin)
        nwidth = int(np.float32(100.0) * np.float32(len(x)) / np.float32(sr))
        img, _ = O.grey_to_rgb(grey, nwidth, nh)
        got = np.frombuffer(mt.get_spec_image(i, 100.0, nh), np.uint8)
        assert got.size == img.size
        m, f = _rgb_diff(got, img)
        worst = max(worst, m)
        diff_px += f * img.size / 3
        total_px += img.size // 3
    assert worst <= E2E_MAX_LSB and diff_px / total_px <= E2E_MAX_FRAC, (worst, diff_px, total_px)
