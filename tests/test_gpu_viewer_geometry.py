"""The streaming kernel at the viewer's own geometries (stft3v_kernels.hip; lib.rs:43-46,93-99:
win = round(40 ms sr / 4) 4, hop = win / 4, n_fft = next_pow2(win), so win < n_fft and the hop is
not a whole number of a lane's rows) against the oracle: streams across track ends, tracks at odd
element offsets (per-frame reloads), the shortest legal tracks (n = win - 1, lib.rs:413), reflect
at both ends, mono / stereo, f32 / s16, every output kind, and a grid small enough that each
stream walks hundreds of frames through the ring's per-lane select shift."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine
from tolerances import DB_MAX, DB_P9999, STFT_REL, db_clamped_err, stft_frame_err

pytestmark = pytest.mark.gpu

# (n_fft, win, hop) of the viewer at 48 / 24 / 16 / 8 kHz (SURVEY.md §8 viewer-defaults row)
VIEW = [(2048, 1920, 480), (1024, 960, 240), (1024, 640, 160), (512, 320, 80)]
# and at 44.1 / 22.05 kHz: odd hops (streams in pairs interleaving the frames)
VIEW_ODD = [(2048, 1764, 441), (1024, 884, 221)]


def _mono_fold(t):  # lib.rs:42 channel sum, (0 + c0) + c1 ...
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _tracks(rng, lens, channels, fmt):
    out = []
    for n in lens:
        if fmt == engine.IN_S16:
            out.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            out.append((rng.standard_normal((n, channels)) * 0.3).astype(np.float32))
    return out


def _run(plan, tracks, channels, fmt, gap, max_blocks=3, kernel=0, row_floats=None):
    parts, offs, off = [], [], 0
    for t in tracks:
        offs.append(off)
        parts.append(t.reshape(-1))
        off += t.size
        if gap:
            parts.append(np.zeros(gap, t.dtype))
            off += gap
    flat = np.concatenate(parts)
    lens = [t.shape[0] for t in tracks]
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    fl = row_floats if row_floats is not None else plan.row_bins
    dout = engine.DeviceBuffer(T * fl * 4)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels,
                     kernel=kernel, max_blocks=max_blocks)
    k = b.kernel
    b.run()
    engine.synchronize()
    res = dout.to_host(np.float32)
    rows = [res[int(b.frame0[i]) * fl:int(b.frame0[i + 1]) * fl] for i in range(len(tracks))]
    b.close()
    dout.close()
    din.close()
    return k, rows


def _x(t, fmt):
    x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
    return _mono_fold(x.astype(np.float32))


@pytest.mark.parametrize("n_fft,win,hop", VIEW + VIEW_ODD)
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap", [0, 3])
def test_viewer_geometry_complex_streams(n_fft, win, hop, channels, fmt, gap):
    rng = np.random.default_rng(n_fft * 7 + hop + channels * 3 + fmt + gap)
    lens = [win - 1, win, n_fft, n_fft + 1, 3 * n_fft + 7, 37 * hop, 10 * n_fft + 3, 60 * hop + 5,
            2 * n_fft, 211 * hop + 11]
    tracks = _tracks(rng, lens, channels, fmt)
    plan = engine.Plan(n_fft, win, hop, engine.OUT_COMPLEX)
    k, rows = _run(plan, tracks, channels, fmt, gap, row_floats=2 * plan.row_bins)
    plan.close()
    # the streaming kernel is the automatic choice at this geometry (odd hops with s16 mono too:
    # 2-byte-aligned sample-pair loads on the shifted grid)
    assert k == 3
    for t, r in zip(tracks, rows):
        ref = O.perform_stft(_x(t, fmt), win, hop, n_fft)
        got = r.view(np.complex64).reshape(ref.shape)
        assert stft_frame_err(got, ref) <= STFT_REL, (len(t), stft_frame_err(got, ref))


_KINDS = [engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB]


def _auto(n_fft, hop, frames=0):
    """The automatic kernel for the mel / linear kinds: stft5 (its viewer column rule,
    stft5_kernels.hip HQ 7) at the 48 kHz geometry for batches of >= 400 000 frames
    (Batch::kView5MinFrames), stft3 otherwise -- these tests' batches are small."""
    return 5 if (n_fft, hop) == (2048, 480) and frames >= 400000 else 3


def _check_kind(kind, g, ref, fb=None):
    if kind == engine.OUT_MEL_AMP_DB:
        want = O.amp_to_db_default(O.dot(O.norm(ref), fb))
    elif kind == engine.OUT_MAG:
        want = O.norm(ref)
    elif kind == engine.OUT_POWER:
        want = O.norm_sqr(ref)
    elif kind == engine.OUT_AMP_DB:
        want = O.amp_to_db_default(O.norm(ref))
    else:
        want = O.power_to_db_default(O.norm_sqr(ref))
    if kind in (engine.OUT_AMP_DB, engine.OUT_POWER_DB, engine.OUT_MEL_AMP_DB):
        mx, p = db_clamped_err(g, want)
        assert mx <= DB_MAX and p <= DB_P9999, (mx, p)
    else:
        scale = np.abs(want).max(axis=1, keepdims=True)
        rel = 4e-6 if kind == engine.OUT_MAG else 8e-6
        assert np.all(np.abs(g - want) <= rel * np.maximum(scale, 1e-30)), float(np.abs(g - want).max())


@pytest.mark.parametrize("kernel", [5, 3])
@pytest.mark.parametrize("kind", _KINDS + [engine.OUT_MEL_AMP_DB])
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap,max_blocks", [(0, 1), (3, 2), (0, 0)])
def test_viewer_48k_stft5_column_rule(kernel, kind, channels, fmt, gap, max_blocks):
    """stft5 at the 48 kHz viewer geometry (win 1920 / hop 480 / n_fft 2048: hop / 2 = 7 rows of
    32 + 16, the ring's per-lane select shift and the column-rotated window, twiddles and
    transpose writes) and stft3 forced at the same inputs, both against the oracle: streams
    across track ends, tracks at odd element offsets (gap 3: per-frame reloads), the shortest
    legal track, one block (every stream walks hundreds of frames through the rotation)."""
    n_fft, win, hop, sr = 2048, 1920, 480, 48000
    rng = np.random.default_rng(kind * 13 + channels * 5 + fmt + gap + 7 * max_blocks)
    lens = [win - 1, 5 * n_fft + 3, 33 * hop + 1, 97 * hop + 2, 211 * hop + 11]
    tracks = _tracks(rng, lens, channels, fmt)
    mel = kind == engine.OUT_MEL_AMP_DB
    plan = engine.Plan(n_fft, win, hop, kind, **({"sr": sr, "n_mels": 128} if mel else {}))
    k, rows = _run(plan, tracks, channels, fmt, gap, max_blocks=max_blocks, kernel=kernel)
    plan.close()
    assert k == kernel
    fb = O.calc_mel_fb(sr, n_fft, 128) if mel else None
    for t, r in zip(tracks, rows):
        ref = O.perform_stft(_x(t, fmt), win, hop, n_fft)
        _check_kind(kind, r.reshape(ref.shape[0], -1), ref, fb)


@pytest.mark.parametrize("win,hop", [(1792, 448), (2040, 510), (2016, 504), (1800, 450), (2048, 496)])
@pytest.mark.parametrize("kind", [engine.OUT_MAG, engine.OUT_AMP_DB, engine.OUT_MEL_AMP_DB])
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_S16)])
@pytest.mark.parametrize("gap,max_blocks", [(3, 1), (0, 0)])
def test_stft5_every_supported_view_hop(win, hop, kind, channels, fmt, gap, max_blocks):
    """stft5_supports takes every even hop with hop / 2 = 7 rows of 32 + rem (rem 0..31) and every
    even win <= 2048: the column rule at rem 0 (hop 448: the shift-by-HQ+1 select
    never taken), rem 31 (hop 510), win 2016 / hop 504 (the viewer's 42 ms window at 48 kHz),
    an odd rem (hop 450: 225 = 7 x 32 + 1) and win = n_fft with a non-canonical hop, forced, against
    the oracle with odd-offset tracks (per-frame reloads) and one-block grids."""
    n_fft, sr = 2048, 48000
    rng = np.random.default_rng(win + hop + 17 * kind + channels + gap)
    lens = [win - 1, 5 * n_fft + 3, 33 * hop + 1, 97 * hop + 2]
    tracks = _tracks(rng, lens, channels, fmt)
    mel = kind == engine.OUT_MEL_AMP_DB
    plan = engine.Plan(n_fft, win, hop, kind, **({"sr": sr, "n_mels": 128} if mel else {}))
    k, rows = _run(plan, tracks, channels, fmt, gap, max_blocks=max_blocks, kernel=5)
    plan.close()
    assert k == 5
    fb = O.calc_mel_fb(sr, n_fft, 128) if mel else None
    for t, r in zip(tracks, rows):
        ref = O.perform_stft(_x(t, fmt), win, hop, n_fft)
        _check_kind(kind, r.reshape(ref.shape[0], -1), ref, fb)


@pytest.mark.parametrize("n_fft,win,hop", VIEW + VIEW_ODD)
@pytest.mark.parametrize("kind", _KINDS)
@pytest.mark.parametrize("max_blocks", [0, 2])
def test_viewer_geometry_linear_kinds(n_fft, win, hop, kind, max_blocks):
    rng = np.random.default_rng(n_fft + hop + 11 * kind + max_blocks)
    lens = [win - 1, 5 * n_fft + 3, 33 * hop + 1, 97 * hop + 2]
    tracks = _tracks(rng, lens, 2, engine.IN_F32)
    plan = engine.Plan(n_fft, win, hop, kind)
    k, rows = _run(plan, tracks, 2, engine.IN_F32, 0, max_blocks=max_blocks)
    plan.close()
    assert k == _auto(n_fft, hop)
    for t, r in zip(tracks, rows):
        ref = O.perform_stft(_x(t, engine.IN_F32), win, hop, n_fft)
        g = r.reshape(ref.shape[0], -1)
        if kind == engine.OUT_MAG:
            want = O.norm(ref)
        elif kind == engine.OUT_POWER:
            want = O.norm_sqr(ref)
        elif kind == engine.OUT_AMP_DB:
            want = O.amp_to_db_default(O.norm(ref))
        else:
            want = O.power_to_db_default(O.norm_sqr(ref))
        if kind in (engine.OUT_AMP_DB, engine.OUT_POWER_DB):
            mx, p = db_clamped_err(g, want)
            assert mx <= DB_MAX and p <= DB_P9999, (mx, p)
        else:
            scale = np.abs(want).max(axis=1, keepdims=True)
            rel = 4e-6 if kind == engine.OUT_MAG else 8e-6
            assert np.all(np.abs(g - want) <= rel * np.maximum(scale, 1e-30)), float(np.abs(g - want).max())


@pytest.mark.parametrize("n_fft,win,hop,sr", [(2048, 1920, 480, 48000), (1024, 960, 240, 24000),
                                              (1024, 640, 160, 16000), (512, 320, 80, 8000),
                                              (2048, 1764, 441, 44100), (1024, 884, 221, 22050)])
@pytest.mark.parametrize("n_mels", [128, 40])
def test_viewer_geometry_mel_db(n_fft, win, hop, sr, n_mels):
    rng = np.random.default_rng(n_fft + n_mels + sr)
    lens = [win - 1, 4 * n_fft + 5, 71 * hop + 3]
    fmt = engine.IN_S16
    tracks = _tracks(rng, lens, 1, fmt)
    plan = engine.Plan(n_fft, win, hop, engine.OUT_MEL_AMP_DB, sr=sr, n_mels=n_mels)
    k, rows = _run(plan, tracks, 1, fmt, 0, max_blocks=2)
    plan.close()
    assert k == _auto(n_fft, hop)
    fb = O.calc_mel_fb(sr, n_fft, n_mels)
    for t, r in zip(tracks, rows):
        ref = O.perform_stft(_x(t, fmt), win, hop, n_fft)
        want = O.amp_to_db_default(O.dot(O.norm(ref), fb))
        mx, p = db_clamped_err(r.reshape(ref.shape[0], -1), want)
        assert mx <= DB_MAX and p <= DB_P9999, (mx, p)


@pytest.mark.parametrize("n_fft,win,hop", VIEW_ODD)
@pytest.mark.parametrize("n_tracks", [1, 2, 7])
def test_odd_hop_pairs_across_track_ends(n_fft, win, hop, n_tracks):
    """Odd hops: a stream pair shares its frames (even / odd ones); with tracks of odd and even
    frame counts the pair's parity relative to each track changes at every track end, and with
    max_blocks 1 every stream pair crosses several tracks."""
    rng = np.random.default_rng(n_fft + hop + n_tracks)
    lens = [int(v) for v in rng.integers(win - 1, 60 * hop, n_tracks)]
    tracks = _tracks(rng, lens, 2, engine.IN_F32)
    plan = engine.Plan(n_fft, win, hop, engine.OUT_AMP_DB)
    for mb in (1, 2, 0):
        k, rows = _run(plan, tracks, 2, engine.IN_F32, 1, max_blocks=mb)
        assert k == 3
        for t, r in zip(tracks, rows):
            ref = O.perform_stft(_x(t, engine.IN_F32), win, hop, n_fft)
            mx, p = db_clamped_err(r.reshape(ref.shape[0], -1), O.amp_to_db_default(O.norm(ref)))
            assert mx <= DB_MAX and p <= DB_P9999, (len(t), mb, mx, p)
    plan.close()
