"""GPU parity on the BASELINE.json configurations at sizes the
oracle finishes in seconds, plus size-independent properties at full size.

  C2  the reference's 6 sample rates (the 5 committed samples whole + the 48 kHz substitute),
      n_fft 2048 / hop 512, power dB, one batch over all tracks (s16 input, audio.rs:16-19)
  C3  48 kHz 10 s mono tracks, n_fft 2048 / hop 512, mel-128 + amp dB
  C5  mixed rates x per-track n_fft in {256..2048}, amp dB -> global range -> grey ->
      Lanczos3 -> colormap RGB (thesia.pipeline), bytes checked against the oracle display
      path run on the device's own dB (bit-exact), dB against the oracle (tolerance)
"""
import os

import numpy as np
import pytest

import fixtures
import oracle_ffi as O
from thesia import engine, pipeline, shard
from tolerances import (DB_MAX, DB_P9999, STFT_REL, db_clamped_err, db_err_relative_to_oracle, stft_f64,
                        stft_frame_err)

pytestmark = pytest.mark.gpu


def _excerpts_s16(golden_dir):
    z = np.load(os.path.join(golden_dir, "samples_excerpt.npz"))
    out = [(z[f"pcm_{t}"], int(z[f"sr_{t}"])) for t in ["8k", "16k", "22k05", "24k", "44k1"]]
    from scipy.signal import resample_poly  # the 48 kHz substitute
    x48 = np.clip(np.round(resample_poly(z["pcm_24k"].astype(np.float64), 2, 1)), -32768, 32767)
    out.append((x48.astype(np.int16), 48000))
    return out


def _c2_batch(tracks, kind):
    """One batch over the C2 tracks (s16 mono, n_fft 2048 / hop 512, the automatic kernel) of
    output kind `kind`; returns (rows [T, row_floats], frame0)."""
    n_fft, hop = 2048, 512
    plan = engine.Plan(n_fft, n_fft, hop, kind)
    flat = np.concatenate([t for t, _ in tracks])
    offs = np.cumsum([0] + [len(t) for t, _ in tracks[:-1]])
    lens = [len(t) for t, _ in tracks]
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    dout = engine.DeviceBuffer(T * plan.row_bins * 4 * (2 if kind == engine.OUT_COMPLEX else 1))
    b = engine.Batch(plan, din, offs, lens, dout, input_format=engine.IN_S16, channels=1)
    b.run()
    engine.synchronize()
    if kind == engine.OUT_COMPLEX:
        got = dout.to_host(np.complex64, (T, plan.row_bins))
    else:
        got = dout.to_host(np.float32, (T, plan.row_bins))
    f0 = [int(v) for v in b.frame0]
    b.close()
    dout.close()
    din.close()
    plan.close()
    return got, f0


def test_c2_six_sample_rates_power_db():
    """C2 at the size BASELINE.json names: the five sample WAVs whole (44.03 s each) + the
    48 kHz substitute (2 113 529 samples), 13 946 frames in one batch.

    Two contracts per track, both against the oracle on the same int16 input:
      * linear domain, kernel vs oracle directly (which does not degrade at
        the -120 dB floor): complex rows per frame |dX| <= STFT_REL * max_k |X_t|; |X|^2 rows
        per frame <= 8e-6 * max_k |X_t|^2 (the bound test_gpu_viewer_geometry uses);
      * power dB: the kernel's clamped-dB error against the float64 spectrum at most
        max(0.25 dB, 2 x the oracle's own) -- the reference's f32 error at the floor of a 44 s
        recording reaches 0.76 dB -- and the kernel-vs-oracle clamped dB max /
        p99.99 printed per rate (recorded in DESIGN.md §3)."""
    tracks = fixtures.samples_full() + [(fixtures.c1_substitute(), 48000)]
    assert sum(engine.Batch.frames_for(engine.Plan(2048, 2048, 512, engine.OUT_POWER_DB), [len(t)]) for t, _ in tracks) == 13946
    n_fft, hop = 2048, 512
    got_db, f0 = _c2_batch(tracks, engine.OUT_POWER_DB)
    got_pw, f0p = _c2_batch(tracks, engine.OUT_POWER)
    got_cx, f0c = _c2_batch(tracks, engine.OUT_COMPLEX)
    assert f0 == f0p == f0c
    w = (O.hann(n_fft) / np.float32(n_fft)).astype(np.float32)
    for k, (pcm, sr) in enumerate(tracks):
        x = (0.0 + pcm.astype(np.float32) / np.float32(32768.0)).astype(np.float32)  # lib.rs:42 fold
        spec = O.perform_stft(x, n_fft, hop, n_fft)
        pw = O.norm_sqr(spec)
        ref = O.power_to_db_default(pw)
        rows = slice(f0[k], f0[k + 1])
        g = got_db[rows]
        assert g.shape == ref.shape
        # (i) complex rows vs the oracle, per frame
        e_cx = stft_frame_err(got_cx[rows], spec)
        assert e_cx <= STFT_REL, (sr, e_cx)
        # |X|^2 rows vs the oracle, per frame (8e-6 x the frame's largest power)
        scale = pw.max(axis=1, keepdims=True)
        d_pw = np.abs(got_pw[rows].astype(np.float64) - pw)
        e_pw = float((d_pw / np.maximum(scale, 1e-30)).max())
        assert np.all(d_pw <= 8e-6 * np.maximum(scale, 1e-30)), (sr, e_pw)
        # power dB vs the float64 spectrum, relative to the oracle's own error
        X = stft_f64(x, n_fft, hop, n_fft, w)
        exact = 10.0 * np.log10(np.maximum(X.real ** 2 + X.imag ** 2, 1e-36))
        ok, ge, oe = db_err_relative_to_oracle(g, ref, exact)
        assert ok, (sr, ge, oe)
        kmx, kp = db_clamped_err(g, ref)
        print(f"C2 {sr} Hz: complex {e_cx:.2e}, power {e_pw:.2e}, kernel-vs-oracle dB max {kmx:.3f} "
              f"p99.99 {kp:.4f}; vs f64 kernel {ge[0]:.3f}/{ge[1]:.4f} oracle {oe[0]:.3f}/{oe[1]:.4f}")


def test_c3_mel128_mono_10s():
    n_tracks, n = 6, 480000
    pcm = [engine.synth_pcm_host(1, i, n, 48000)[:, 0] for i in range(n_tracks)]
    x = np.stack([p.astype(np.float32) / np.float32(32768.0) for p in pcm])
    plan = engine.Plan(2048, 2048, 512, engine.OUT_MEL_AMP_DB, sr=48000, n_mels=128)
    din = engine.DeviceBuffer.from_host(x)
    T = engine.Batch.frames_for(plan, [n] * n_tracks)
    assert T == 938 * n_tracks
    dout = engine.DeviceBuffer(T * 128 * 4)
    b = engine.Batch(plan, din, np.arange(n_tracks) * n, [n] * n_tracks, dout)
    b.run()
    engine.synchronize()
    got = dout.to_host(np.float32, (T, 128))
    fb = O.calc_mel_fb(48000, 2048, 128)
    for k in (0, n_tracks - 1):
        ref = O.amp_to_db_default(O.dot(O.norm(O.perform_stft(x[k], 2048, 512, 2048)), fb))
        mx, p = db_clamped_err(got[938 * k:938 * (k + 1)], ref)
        assert mx <= DB_MAX and p <= DB_P9999, (k, mx, p)
    assert np.isfinite(got).all()


def test_c5_mixed_rate_render_pipeline():
    tracks = pipeline.c5_tracks(12, seconds=1.0)  # every (rate, n_fft) pair of the generator
    out = pipeline.render_tracks(tracks, px_per_sec=100.0, nheight=120, keep_db=True)
    # global range over all tracks (lib.rs:194-209) from the device's own dB
    gmax, gmin, max_sr = shard.global_db_range(max(r.spec_max for r in out),
                                               min(r.spec_min for r in out),
                                               max(t.sr for t in tracks))
    for t, r in zip(tracks, out):
        x = (t.pcm.astype(np.float32) / np.float32(32768.0)).astype(np.float32)
        x = (np.float32(0.0) + x).astype(np.float32)
        ref_db = O.amp_to_db_default(O.norm(O.perform_stft(x, t.n_fft, t.n_fft // 4, t.n_fft)))
        assert r.db.shape == ref_db.shape
        mx, p = db_clamped_err(r.db, ref_db)
        assert mx <= DB_MAX and p <= DB_P9999, (t.sr, t.n_fft, mx, p)
        assert (r.spec_max, r.spec_min) == (float(r.db.max()), float(r.db.min()))
        up = shard.up_ratio(t.sr, max_sr, freq_scale_mel=False)
        grey = O.spec_to_grey(r.db, up, gmax, gmin)
        img, _ = O.grey_to_rgb(grey, r.nwidth, 120)
        assert r.rgb.tobytes() == img.tobytes(), (t.sr, t.n_fft)  # display path bit-exact


# 0: single-pass stripes for groups downsampling >= 3:1 along time, else two kernels; 1: per-track;
# 2: three-stage; 3: two kernels for every group (LDS-DMA horizontal; wide vertical pass for
# upsampling groups); 4: single-pass stripes wherever an instance covers the geometry; 5: as 0, plus
# the stripes' ring mode (exact taps from a per-lane LDS ring) for the groups below 3 frames / column
@pytest.mark.parametrize("path", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("px_per_sec", [73.0, 30.0, 9.0, 2.0])  # 30: 17-64 taps; 9, 2: wider spans
@pytest.mark.parametrize("nheight", [90, 400, 600])  # 400, 600: H -> nheight downsampling ~2.5, taller
def test_render_batch_ragged_groups(path, px_per_sec, nheight):
    """Several tracks of different lengths per geometry group: the batched renders (one launch
    per stage for the whole group: fused grey + vertical with a transposed intermediate, or the
    three-stage one) and the per-track launches produce the oracle's bytes for every image
    (ragged T, nwidth and workspace offsets; staged and direct horizontal spans)."""
    engine.set_render_path(path)
    try:
        _ragged(px_per_sec, nheight)
    finally:
        engine.set_render_path(0)


def _ragged(px_per_sec, nheight):
    base = pipeline.c5_tracks(12, seconds=0.6)
    tracks = []
    # the 12 (rate, n_fft) geometries x 2 lengths: 4 spectrogram batches (one per n_fft) of 3
    # rates each, so every display group is a slice of a batch's rows
    for k, t in enumerate(base * 2):
        n = int(t.pcm.shape[0] * (0.5 + 0.45 * (k // 12))) + 3 * k
        n = max(n, t.n_fft)
        tracks.append(pipeline.Track(t.pcm[:n].copy(), t.sr, t.n_fft))
    out = pipeline.render_tracks(tracks, px_per_sec=px_per_sec, nheight=nheight, keep_db=True)
    _oracle_check(tracks, out, nheight)


def _oracle_check(tracks, out, nheight):
    gmax, gmin, max_sr = shard.global_db_range(max(r.spec_max for r in out),
                                               min(r.spec_min for r in out),
                                               max(t.sr for t in tracks))
    for t, r in zip(tracks, out):
        up = shard.up_ratio(t.sr, max_sr, freq_scale_mel=False)
        grey = O.spec_to_grey(r.db, up, gmax, gmin)
        img, _ = O.grey_to_rgb(grey, r.nwidth, nheight)
        assert r.rgb.tobytes() == img.tobytes(), (t.sr, t.n_fft, t.pcm.shape)


@pytest.mark.parametrize("path", [0, 3, 4, 5])
@pytest.mark.parametrize("mode", ["some_silent", "all_silent"])
def test_render_silent_tracks(path, mode):
    """Silent tracks in a display batch: their dB rows sit at the global minimum, so the grey
    quotient (db - min) / (max - min) is +0 (the kernels' GreyMap takes its f32-division branch
    there); with every track silent the span is 0 and every quotient 0 / 0 (NaN, grey +0 after
    the clamps, as in display.rs). Bytes equal the oracle's on every render path."""
    base = pipeline.c5_tracks(12, seconds=0.6)
    tracks = []
    for k, t in enumerate(base):
        pcm = t.pcm.copy()
        if mode == "all_silent" or k in (0, 5, 7):
            pcm[:] = 0
        tracks.append(pipeline.Track(pcm, t.sr, t.n_fft))
    engine.set_render_path(path)
    try:
        out = pipeline.render_tracks(tracks, px_per_sec=30.0, nheight=400, keep_db=True)
    finally:
        engine.set_render_path(0)
    _oracle_check(tracks, out, 400)


@pytest.mark.parametrize("path", [0, 3, 4, 5])
def test_c5_geometry_500_rows(path):
    """The C5 display geometry (100 px/s x 500 rows, every (rate, n_fft) pair) at 3 s per track:
    the single-pass stripe kernel runs the 3 groups that downsample >= 3:1 along time (path 0) or
    the 7 whose geometry its instances cover (path 4; 8-wave blocks of 512 rows, strips of 64
    columns, dword RGB stores: nwidth 300), the others the two-kernel path; bytes equal the
    oracle display of the device's own dB."""
    engine.set_render_path(path)
    try:
        tracks = pipeline.c5_tracks(12, seconds=3.0)
        out = pipeline.render_tracks(tracks, px_per_sec=100.0, nheight=500, keep_db=True)
    finally:
        engine.set_render_path(0)
    gmax, gmin, max_sr = shard.global_db_range(max(r.spec_max for r in out), min(r.spec_min for r in out),
                                               max(t.sr for t in tracks))
    for t, r in zip(tracks, out):
        up = shard.up_ratio(t.sr, max_sr, freq_scale_mel=False)
        img, _ = O.grey_to_rgb(O.spec_to_grey(r.db, up, gmax, gmin), r.nwidth, 500)
        assert r.rgb.tobytes() == img.tobytes(), (t.sr, t.n_fft)


def test_render_pinned_readback_matches_pageable():
    """RenderPipeline(pinned_output=True) reads the RGB bytes into page-locked host buffers
    (thesia_host_register); the bytes equal the pageable readback's."""
    tracks = pipeline.c5_tracks(6, seconds=0.5)
    outs = []
    for pinned in (False, True):
        p = pipeline.RenderPipeline(tracks, px_per_sec=50.0, nheight=64, pinned_output=pinned)
        try:
            p.run_spectrograms()
            outs.append([r.rgb.tobytes() for r in p.render()])
        finally:
            p.close()
    assert outs[0] == outs[1]


def test_render_rejects_overlapping_rgb_ranges():
    """render_rgb_multi runs its groups concurrently: two tracks whose RGB ranges overlap would
    race, so the call is refused (thesia.h) instead of leaving either image."""
    import ctypes as C
    from thesia._lib import lib, _fp, _u64p
    p = pipeline.RenderPipeline(pipeline.c5_tracks(6, seconds=0.5), px_per_sec=50.0, nheight=64)
    try:
        p.run_spectrograms()
        p.render(want_rgb=False)
        up = next(iter(p._up.values()))
        off = p._off.copy()
        args = lambda o: (p._n_disp, p._c_specs, p._c_row0, p._c_bins, p._c_ns, up.ctypes.data_as(_fp),
                          p._nw.ctypes.data_as(C.POINTER(C.c_uint32)), p.nheight, 0.0, -100.0,
                          p._rgb.ptr, o.ctypes.data_as(_u64p))
        assert lib.thesia_render_rgb_multi(*args(off)) == 0
        off[1] = off[0] + 1
        assert lib.thesia_render_rgb_multi(*args(off)) != 0
        assert "overlap" in lib.thesia_last_error().decode()
    finally:
        p.close()


@pytest.mark.parametrize("path", [0, 3, 4])
def test_device_range_render_equals_host_exchange(path):
    """render(want_rgb=False) on one rank reduces the global range on the device
    (thesia_ranges_global) and the display reads it there (thesia_render_rgb_multi_dev): the
    device range equals the host exchange's (shard.global_db_range, lib.rs:194-209) and the RGB
    bytes equal the host-exchange render's, for every render path that takes it."""
    engine.set_render_path(path)
    try:
        tracks = pipeline.c5_tracks(24, seconds=1.2)
        p = pipeline.RenderPipeline(tracks, px_per_sec=100.0, nheight=300)
        p.run_spectrograms()
        assert p.render(want_rgb=False) is None
        engine.synchronize()
        dev = p._rgb.read(np.uint8, p._rgb_total).copy()
        g2 = p._d_grange.read(np.float32, 2).copy()
        out = p.render(want_rgb=True)
        host = p._rgb.read(np.uint8, p._rgb_total)
        gmax, gmin, _ = shard.global_db_range(max(r.spec_max for r in out), min(r.spec_min for r in out),
                                              max(t.sr for t in tracks))
        assert (float(g2[0]), float(g2[1])) == (gmax, gmin)
        assert dev.tobytes() == host.tobytes()
        p.close()
    finally:
        engine.set_render_path(0)
