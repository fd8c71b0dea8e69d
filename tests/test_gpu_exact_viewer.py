"""Round 6: the reference-order streaming kernels (batch kernel 7: stftq at n_fft 512 / 1024, stftr at
2048) at the viewer's own geometries (lib.rs:43-46: win = round(40 ms sr / 4) 4, hop = win / 4,
n_fft = next_pow2(win); 8 kHz 320 / 80 / 512 ... 48 kHz 1920 / 480 / 2048, the odd hops 221 and 441
included) and other even-window geometries, against the oracle bit for bit. There each frame loads
its n_fft samples itself (no register ring), odd starts sample by sample, and the window step keeps
the reference's +0 in the centring pads (lib.rs:377-385). MultiTrack's default path runs them."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine

pytestmark = pytest.mark.gpu

VIEWER_SR = [8000, 16000, 22050, 24000, 44100, 48000]
LINEAR = [engine.OUT_COMPLEX, engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB]


def _fold(t):  # lib.rs:42 channel sum
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _tracks(rng, lens, channels):
    out = []
    for n in lens:
        s = np.float32(10.0) ** rng.uniform(-6, 0)
        out.append((rng.standard_normal((n, channels)) * s).astype(np.float32))
    return out


def _run(geo, kind, tracks, channels, gap=0, max_blocks=0, n_mels=0, sr=48000, kernel=7, fold=True):
    win, hop, n_fft = geo
    parts, offs, off = [], [], 0
    for t in tracks:
        offs.append(off)
        parts.append(t.reshape(-1))
        off += t.size
        if gap:
            parts.append(np.zeros(gap, np.float32))
            off += gap
    flat = np.concatenate(parts)
    lens = [t.shape[0] for t in tracks]
    plan = engine.Plan(n_fft, win, hop, kind, sr=sr, n_mels=n_mels)
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    el = 8 if kind == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(max(T * plan.row_bins * el, 4))
    b = engine.Batch(plan, din, offs, lens, dout, channels=channels, fold_mono=fold, kernel=kernel,
                     max_blocks=max_blocks)
    assert b.kernel == kernel
    b.run()
    engine.synchronize()
    dt = np.complex64 if kind == engine.OUT_COMPLEX else np.float32
    out = dout.to_host(dt, (T, plan.row_bins))
    rows = [out[int(b.frame0[i]):int(b.frame0[i + 1])] for i in range(len(tracks))]
    b.close()
    plan.close()
    din.close()
    dout.close()
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


def _check(geo, kind, tracks, rows, fb=None, fold=True):
    win, hop, n_fft = geo
    w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
    for i, (t, got) in enumerate(zip(tracks, rows)):
        x = _fold(t) if fold else np.ascontiguousarray(t[:, 0])
        want = _want(kind, O.perform_stft(x, win, hop, n_fft, window=w), fb)
        assert got.shape == want.shape, (i, got.shape, want.shape)
        bad = got.view(np.uint32) != want.view(np.uint32)
        assert not bad.any(), (geo, i, int(bad.sum()), np.argwhere(bad)[:5].tolist())


def _lens(geo):
    win, hop, n_fft = geo
    # the shortest legal track (lib.rs:413), a few frames, odd lengths, tracks of hundreds of frames
    return [win - 1, win, n_fft + 3, 9 * hop + 5, 211 * hop + 7, 97 * hop]


@pytest.mark.parametrize("sr", VIEWER_SR)
@pytest.mark.parametrize("kind", LINEAR)
@pytest.mark.parametrize("channels,gap,max_blocks", [(1, 0, 0), (2, 3, 1), (1, 1, 2)])
def test_viewer_geometry_linear_kinds(sr, kind, channels, gap, max_blocks):
    geo = O.track_params(sr)
    rng = np.random.default_rng(sr + 31 * kind + 7 * channels + gap)
    tracks = _tracks(rng, _lens(geo), channels)
    _check(geo, kind, tracks, _run(geo, kind, tracks, channels, gap, max_blocks, sr=sr))


@pytest.mark.parametrize("sr", VIEWER_SR)
@pytest.mark.parametrize("kind", [engine.OUT_MEL_AMP_DB, engine.OUT_MEL])
@pytest.mark.parametrize("n_mels", [0, 128])
def test_viewer_geometry_mel_kinds(sr, kind, n_mels):
    geo = O.track_params(sr)
    win, hop, n_fft = geo
    rng = np.random.default_rng(sr + kind + n_mels)
    tracks = _tracks(rng, _lens(geo), 1)
    fb = O.calc_mel_fb(sr, n_fft, n_mels) if n_mels else O.calc_mel_fb_default(sr, n_fft)
    plan = engine.Plan(n_fft, win, hop, kind, sr=sr, n_mels=n_mels)
    din = engine.DeviceBuffer(16)
    b = engine.Batch(plan, din, [0], [win], din)
    runs7 = True
    try:
        b.set_option(engine.OPT_KERNEL, 7)
    except Exception:
        runs7 = False  # the exact mel tables of this plan do not fit kernel 7's LDS: stftx runs it
    b.close()
    plan.close()
    din.close()
    if not runs7:
        pytest.skip("kernel 7's mel tables do not fit LDS at this filterbank (kernel 9 covers it)")
    _check(geo, kind, tracks, _run(geo, kind, tracks, 1, 1, 2, n_mels=n_mels, sr=sr), fb)


@pytest.mark.parametrize("geo", [(1000, 250, 1024), (1022, 333, 1024), (400, 99, 512), (2000, 501, 2048),
                                 (512, 128, 512), (1536, 384, 2048), (256, 1, 256)])
@pytest.mark.parametrize("kind", [engine.OUT_COMPLEX, engine.OUT_AMP_DB])
def test_other_even_windows(geo, kind):
    """Even windows shorter than n_fft, hops not a quarter of it (odd, 1, longer than the window's
    quarter), and win = n_fft at a non-canonical hop."""
    rng = np.random.default_rng(geo[0] + geo[1] + kind)
    win, hop, n_fft = geo
    lens = [win - 1, n_fft + 11, max(40 * hop + 3, 3 * win + 7)]
    tracks = _tracks(rng, lens, 1)
    _check(geo, kind, tracks, _run(geo, kind, tracks, 1, 1))


@pytest.mark.parametrize("sr", VIEWER_SR)
def test_equals_stftx_on_long_tracks(sr):
    """8 x 60 s tracks at the viewer geometry: kernel 7 equals the one-wave-per-frame kernel 9."""
    geo = O.track_params(sr)
    rng = np.random.default_rng(sr)
    tracks = _tracks(rng, [60 * sr] * 8, 1)
    a = _run(geo, engine.OUT_AMP_DB, tracks, 1, kernel=7, sr=sr)
    b = _run(geo, engine.OUT_AMP_DB, tracks, 1, kernel=9, sr=sr)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


@pytest.mark.parametrize("geo", [(1920, 480, 2048), (640, 160, 1024), (2048, 512, 2048), (1024, 256, 1024),
                                 (256, 64, 256)])
def test_negative_zero_samples_and_silence(geo):
    """-0 samples and silent stretches, unfolded (MultiTrack's mono pool: fold_mono = 0): the pads'
    +0, the window's products and the untangle's partner bins as the reference forms them (complex
    rows: every bit, signs of zeros included), at viewer and canonical geometries."""
    win, hop, n_fft = geo
    x = np.zeros((30 * hop + win, 1), np.float32)
    x[::3] = -0.0
    x[5 * hop: 9 * hop] = np.random.default_rng(1).standard_normal((4 * hop, 1)).astype(np.float32)
    x[12 * hop] = -1e-3
    tracks = [x]
    _check(geo, engine.OUT_COMPLEX, tracks, _run(geo, engine.OUT_COMPLEX, tracks, 1, fold=False), fold=False)
