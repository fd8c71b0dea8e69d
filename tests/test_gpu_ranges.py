"""Batch range option (THESIA_BATCH_OPT_RANGE): per-track max / min of the output rows
(update_spec_greys' reduction, lib.rs:194-207) left by the spectrogram launch itself -- folded
into stft3's staged-row epilogue for the linear kinds, one pass over the rows otherwise -- must
equal numpy's max / min of the rows the same launch wrote, for ragged tracks, every kernel and
several frame-stream splits (max_blocks: streams crossing track boundaries)."""
import numpy as np
import pytest

from thesia import engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", [engine.OUT_AMP_DB, engine.OUT_POWER_DB, engine.OUT_MAG, engine.OUT_MEL_AMP_DB])
@pytest.mark.parametrize("n_fft", [256, 1024, 2048])
@pytest.mark.parametrize("kernel,max_blocks", [(0, 0), (0, 3), (1, 0), (2, 0)])
def test_batch_ranges_equal_row_reduction(kind, n_fft, kernel, max_blocks):
    rng = np.random.default_rng(n_fft + kind)
    lens = [n_fft * 3 + 17, n_fft * 40 + 5, n_fft + 1, n_fft * 11 + 300, n_fft * 2]
    ch = 2
    tracks = [(rng.standard_normal((n, ch)) * np.float32(10.0) ** rng.uniform(-5, 0)).astype(np.float32)
              for n in lens]
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]]).astype(np.uint64)
    plan = engine.Plan(n_fft, n_fft, n_fft // 4, kind, sr=48000, n_mels=64 if kind == engine.OUT_MEL_AMP_DB else 0)
    T = engine.Batch.frames_for(plan, lens)
    din = engine.DeviceBuffer.from_host(flat)
    dout = engine.DeviceBuffer(T * plan.row_bins * 4)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=engine.IN_F32, channels=ch, fold_mono=True,
                     kernel=kernel, max_blocks=max_blocks)
    drange = engine.DeviceBuffer(12 * len(lens))
    b.set_option(engine.OPT_RANGE, drange.ptr.value)
    for _ in range(2):  # the slots are re-initialised by every run
        b.run()
    engine.synchronize()
    mx, mn, nan = engine.ranges_read(drange, len(lens))
    rows = dout.to_host(np.float32, (T, plan.row_bins))
    for i in range(len(lens)):
        r = rows[int(b.frame0[i]):int(b.frame0[i + 1])]
        assert not nan[i]
        assert mx[i] == r.max() and mn[i] == r.min(), (i, kernel, mx[i], r.max(), mn[i], r.min())


def test_range_option_rejects_complex_rows():
    plan = engine.Plan(512, 512, 128, engine.OUT_COMPLEX, sr=48000)
    din = engine.DeviceBuffer(4 * 4096)
    dout = engine.DeviceBuffer(8 * 257 * 64)
    b = engine.Batch(plan, din, np.zeros(1, np.uint64), [4096], dout)
    with pytest.raises(Exception):
        b.set_option(engine.OPT_RANGE, 1 << 20)


def test_auto_kernel_follows_the_range_option():
    """Mono linear rows at n_fft 2048 run stft5 by default (measured faster); with the range
    option the automatic choice moves to stft3, which folds the ranges into its row epilogue;
    a forced kernel stays. The ranges equal the rows' max / min either way."""
    rng = np.random.default_rng(5)
    lens = [48000, 30011, 2048 * 7 + 1]
    x = np.concatenate([(rng.standard_normal(n) * 0.2).astype(np.float32) for n in lens])
    offs = np.cumsum([0] + lens[:-1]).astype(np.uint64)
    plan = engine.Plan(2048, 2048, 512, engine.OUT_AMP_DB, sr=48000)
    T = engine.Batch.frames_for(plan, lens)
    din = engine.DeviceBuffer.from_host(x)
    outs = []
    for forced in (0, 5):
        dout = engine.DeviceBuffer(T * plan.row_bins * 4)
        b = engine.Batch(plan, din, offs, lens, dout, kernel=forced)
        assert b.kernel == 5
        drange = engine.DeviceBuffer(12 * len(lens))
        b.set_option(engine.OPT_RANGE, drange.ptr.value)
        assert b.kernel == (3 if forced == 0 else 5)
        b.run()
        engine.synchronize()
        mx, mn, nan = engine.ranges_read(drange, len(lens))
        rows = dout.to_host(np.float32, (T, plan.row_bins))
        for i in range(len(lens)):
            r = rows[int(b.frame0[i]):int(b.frame0[i + 1])]
            assert mx[i] == r.max() and mn[i] == r.min() and not nan[i]
        outs.append(rows)


@pytest.mark.parametrize("n_fft", [256, 512, 1024, 2048])
@pytest.mark.parametrize("ch,fmt", [(1, "f32"), (2, "f32"), (1, "s16"), (2, "s16")])
def test_amp_db_fold_instances(n_fft, ch, fmt):
    """Amp dB rows run stft3 instances with the kind and the range fold fixed at compile time
    (stft3_kernel.hpp VAR bits 18-21): with the range option (fold compiled in)
    and without it (fold compiled out) the rows are the same bits, and the folded ranges equal
    the rows' max / min, for every n_fft, channel count and input format."""
    rng = np.random.default_rng(n_fft * 7 + ch)
    lens = [n_fft * 5 + 3, n_fft * 23 + 101, n_fft + 1, n_fft * 9]
    if fmt == "f32":
        tracks = [(rng.standard_normal((n, ch)) * 0.3).astype(np.float32) for n in lens]
        inf = engine.IN_F32
    else:
        tracks = [(rng.standard_normal((n, ch)) * 3000).clip(-32768, 32767).astype(np.int16) for n in lens]
        inf = engine.IN_S16
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]]).astype(np.uint64)
    plan = engine.Plan(n_fft, n_fft, n_fft // 4, engine.OUT_AMP_DB, sr=48000)
    T = engine.Batch.frames_for(plan, lens)
    din = engine.DeviceBuffer.from_host(flat)
    rows = []
    for fold in (False, True):
        dout = engine.DeviceBuffer(T * plan.row_bins * 4)
        b = engine.Batch(plan, din, offs, lens, dout, input_format=inf, channels=ch, fold_mono=True,
                         kernel=3, max_blocks=3)
        drange = engine.DeviceBuffer(12 * len(lens))
        if fold:
            b.set_option(engine.OPT_RANGE, drange.ptr.value)
        b.run()
        engine.synchronize()
        r = dout.to_host(np.float32, (T, plan.row_bins))
        rows.append(r)
        if fold:
            mx, mn, nan = engine.ranges_read(drange, len(lens))
            for i in range(len(lens)):
                ri = r[int(b.frame0[i]):int(b.frame0[i + 1])]
                assert not nan[i] and mx[i] == ri.max() and mn[i] == ri.min(), i
    assert np.array_equal(rows[0], rows[1])


def _k7_rows_and_ranges(plan, din, offs, lens, T, inf, ch, kernel, max_blocks, with_range):
    dout = engine.DeviceBuffer(T * plan.row_bins * 4)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=inf, channels=ch, fold_mono=True, kernel=kernel,
                     max_blocks=max_blocks)
    assert b.kernel == kernel
    drange = engine.DeviceBuffer(12 * len(lens))
    if with_range:
        b.set_option(engine.OPT_RANGE, drange.ptr.value)
    for _ in range(2):  # the slots are re-initialised by every run
        b.run()
    engine.synchronize()
    rows = dout.to_host(np.float32, (T, plan.row_bins))
    rr = engine.ranges_read(drange, len(lens)) if with_range else None
    f0 = [int(v) for v in b.frame0]
    b.close()
    dout.close()
    drange.close()
    return rows, rr, f0


@pytest.mark.parametrize("geo", [(256, 256, 64), (512, 512, 128), (1024, 1024, 256), (2048, 2048, 512),
                                 (1024, 884, 221), (2048, 1920, 480), (2048, 1764, 441)])
@pytest.mark.parametrize("ch,fmt,max_blocks", [(1, "s16", 0), (2, "f32", 3), (1, "f32", 1)])
def test_kernel7_amp_db_range_fold(geo, ch, fmt, max_blocks):
    """Round 6: kernel 7's amp dB rows fold the per-track range into the epilogue (stftq / stftr RG
    instances) instead of the pass over the rows: the rows are the same bits with and without the
    range option, and the (max, min, NaN) triples equal kernel 9's (the separate pass) and the
    rows' max / min -- ragged tracks, streams crossing track boundaries (max_blocks), a track with
    a NaN sample (its |X| is NaN; decibel.rs's amin clamp takes it to the floor: no NaN rows) and a
    silent one."""
    n_fft, win, hop = geo
    if (win, hop) != (n_fft, n_fft // 4) and fmt != "f32":
        pytest.skip("kernel 7 takes the viewer geometries from f32 (MultiTrack's pool)")
    rng = np.random.default_rng(n_fft + win + hop + ch)
    lens = [n_fft * 3 + 17, n_fft * 40 + 5, win - 1, n_fft * 11 + 300, n_fft * 2, n_fft * 6 + 9]
    tracks = []
    for i, n in enumerate(lens):
        t = rng.standard_normal((n, ch)) * np.float32(10.0) ** rng.uniform(-4, -0.5)
        if i == 4:
            t[:] = 0.0  # silent: every row at the dB floor
        tracks.append(t)
    if fmt == "f32":
        tracks = [t.astype(np.float32) for t in tracks]
        tracks[3][n_fft * 5 + 7, 0] = np.nan
        inf = engine.IN_F32
    else:
        tracks = [(t * 32767).clip(-32768, 32767).astype(np.int16) for t in tracks]
        inf = engine.IN_S16
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]]).astype(np.uint64)
    plan = engine.Plan(n_fft, win, hop, engine.OUT_AMP_DB, sr=48000)
    T = engine.Batch.frames_for(plan, lens)
    din = engine.DeviceBuffer.from_host(flat)
    rows0, _, _ = _k7_rows_and_ranges(plan, din, offs, lens, T, inf, ch, 7, max_blocks, False)
    rows7, (mx7, mn7, nan7), f0 = _k7_rows_and_ranges(plan, din, offs, lens, T, inf, ch, 7, max_blocks, True)
    rows9, (mx9, mn9, nan9), _ = _k7_rows_and_ranges(plan, din, offs, lens, T, inf, ch, 9, 0, True)
    assert np.array_equal(rows0.view(np.uint32), rows7.view(np.uint32))
    assert np.array_equal(rows7.view(np.uint32), rows9.view(np.uint32))
    assert np.array_equal(mx7.view(np.uint32), mx9.view(np.uint32))
    assert np.array_equal(mn7.view(np.uint32), mn9.view(np.uint32))
    assert np.array_equal(nan7 != 0, nan9 != 0)
    for i in range(len(lens)):
        r = rows7[f0[i]:f0[i + 1]]
        bad = np.isnan(r)
        assert bool(nan7[i]) == bool(bad.any()), i
        ok = r[~bad]
        if ok.size:
            assert mx7[i] == ok.max() and mn7[i] == ok.min(), (i, mx7[i], ok.max(), mn7[i], ok.min())
    din.close()
    plan.close()
