"""The streaming kernel (stft3_kernel) and the general kernels against the
oracle on the cases their register ring makes special: streams that cross track ends, tracks that start at odd element
offsets (no 8/16-byte alignment: per-frame reloads), the shortest legal tracks (n = win - 1,
lib.rs:413), frames that reflect at both ends, mono / stereo, f32 / s16, and a grid small enough
that each stream walks hundreds of frames (the shift + prefetch path)."""
import os

import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine
from tolerances import DB_MAX, DB_P9999, STFT_REL, db_clamped_err, stft_frame_err

pytestmark = pytest.mark.gpu


def _mono_fold(t):  # lib.rs:42 channel sum, (0 + c0) + c1 ...
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _run(n_fft, tracks, channels, fmt, gap, kernel, max_blocks=3):
    """tracks packed with `gap` elements between them (odd gaps break the alignment)."""
    hop = n_fft // 4
    parts, offs, off = [], [], 0
    for t in tracks:
        offs.append(off)
        parts.append(t.reshape(-1))
        off += t.size
        if gap:
            parts.append(np.zeros(gap, t.dtype))
            off += gap
    flat = np.concatenate(parts)
    plan = engine.Plan(n_fft, n_fft, hop, engine.OUT_COMPLEX)
    lens = [t.shape[0] for t in tracks]
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    dout = engine.DeviceBuffer(T * plan.row_bins * 8)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels,
                     kernel=kernel, max_blocks=max_blocks)
    assert b.kernel == kernel
    b.run()
    engine.synchronize()
    out = dout.to_host(np.complex64, (T, plan.row_bins))
    return [out[int(b.frame0[i]):int(b.frame0[i + 1])] for i in range(len(tracks))]


@pytest.mark.parametrize("n_fft,kernel", [(256, 3), (1024, 3), (2048, 5), (2048, 3), (2048, 2), (512, 1)])
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap", [0, 3])
def test_streams_across_tracks_edges_and_alignment(n_fft, kernel, channels, fmt, gap):
    # at most 3 blocks: every stream of the streaming kernel walks many frames
    rng = np.random.default_rng(n_fft * 10 + channels * 3 + fmt + gap)
    hop = n_fft // 4
    lens = [n_fft - 1, n_fft, n_fft + 1, 3 * n_fft + 7, 37 * hop, 10 * n_fft + 3, 60 * hop + 5, 2 * n_fft]
    tracks = []
    for n in lens:
        if fmt == engine.IN_S16:
            tracks.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            tracks.append((rng.standard_normal((n, channels)) * 0.3).astype(np.float32))
    outs = _run(n_fft, tracks, channels, fmt, gap, kernel)
    for t, got in zip(tracks, outs):
        x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
        ref = O.perform_stft(_mono_fold(x.astype(np.float32)), n_fft, hop, n_fft)
        assert got.shape == ref.shape
        assert stft_frame_err(got, ref) <= STFT_REL, (len(t), stft_frame_err(got, ref))


_LIN_KINDS = [engine.OUT_MAG, engine.OUT_POWER, engine.OUT_AMP_DB, engine.OUT_POWER_DB]


@pytest.mark.parametrize("n_fft", [256, 2048])
@pytest.mark.parametrize("kind", _LIN_KINDS + [engine.OUT_COMPLEX])
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
@pytest.mark.parametrize("row_store,kernel", [(0, 3), (1, 3), (2, 3), (3, 3), (0, 5)])
def test_row_stores_any_output_alignment(n_fft, kind, shift, row_store, kernel):
    """Output rows of F floats / F float2 are not 16-byte aligned; the LDS-staged float4 row
    stores (stft3 store_row_b128: linear kinds by default, complex with the ROW_STORE option) must write
    exactly the row whatever the output pointer's alignment, and nothing outside the batch's
    rows (guard floats on both sides stay untouched)."""
    if kind == engine.OUT_COMPLEX and shift % 2:
        pytest.skip("complex rows are float2: 8-byte aligned output")
    if (row_store or kernel == 5) and n_fft != 2048:
        pytest.skip("the other store method / stft5_kernel: n_fft 2048 only")
    if row_store >= 2 and kind != engine.OUT_COMPLEX:
        pytest.skip("whole-line / lane-wise row store options: complex rows only")
    rng = np.random.default_rng(n_fft + 7 * kind + shift)
    hop = n_fft // 4
    lens = [n_fft - 1, 5 * n_fft + 3, 33 * hop + 1, 2 * n_fft]
    tracks = [(rng.standard_normal((n, 2)) * 0.3).astype(np.float32) for n in lens]
    plan = engine.Plan(n_fft, n_fft, hop, kind)
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]])
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    fl = plan.row_bins * (2 if kind == engine.OUT_COMPLEX else 1)
    guard = 8
    sentinel = np.float32(-12345.5)
    host = np.full(T * fl + 2 * guard + 4, sentinel, np.float32)
    dout = engine.DeviceBuffer.from_host(host)
    ptr = dout.ptr.value + (guard + shift) * 4
    b = engine.Batch(plan, din, offs, lens, ptr, input_format=engine.IN_F32, channels=2,
                     max_blocks=3, row_store=row_store, kernel=kernel)
    assert b.kernel == kernel
    b.run()
    engine.synchronize()
    res = dout.to_host(np.float32)
    assert np.all(res[:guard + shift] == sentinel)
    assert np.all(res[guard + shift + T * fl:] == sentinel)
    got = res[guard + shift:guard + shift + T * fl]
    for i, t in enumerate(tracks):
        ref = O.perform_stft(_mono_fold(t), n_fft, hop, n_fft)
        rows = got[int(b.frame0[i]) * fl:int(b.frame0[i + 1]) * fl]
        if kind == engine.OUT_COMPLEX:
            g = rows.view(np.complex64).reshape(ref.shape)
            assert stft_frame_err(g, ref) <= STFT_REL
            continue
        g = rows.reshape(ref.shape)
        if kind == engine.OUT_MAG:
            r = O.norm(ref)
        elif kind == engine.OUT_POWER:
            r = O.norm_sqr(ref)
        elif kind == engine.OUT_AMP_DB:
            r = O.amp_to_db_default(O.norm(ref))
        else:
            r = O.power_to_db_default(O.norm_sqr(ref))
        if kind in (engine.OUT_AMP_DB, engine.OUT_POWER_DB):
            mx, p = db_clamped_err(g, r)
            assert mx <= DB_MAX and p <= DB_P9999, (mx, p)
        else:
            scale = np.abs(r).max(axis=1, keepdims=True)
            rel = 4e-6 if kind == engine.OUT_MAG else 8e-6
            assert np.all(np.abs(g - r) <= rel * np.maximum(scale, 1e-30)), float(np.abs(g - r).max())


@pytest.mark.parametrize("shift", [0, 2, 6, 30])
@pytest.mark.parametrize("max_blocks", [0, 5])
def test_line_rows_equal_lane_rows(shift, max_blocks):
    """ROW_STORE 2 (complex rows as whole 128-byte lines, the line two rows share carried from
    frame to frame of a stream; the default) computes the same values as the lane-wise stores
    (ROW_STORE 3); only the store
    pattern differs, so the whole output buffer -- guard floats around the rows included -- is
    bit-identical, at every line offset of the output pointer and with many streams (every
    stream's first head line and last tail line are partial)."""
    rng = np.random.default_rng(100 + shift + max_blocks)
    n_fft, hop = 2048, 512
    lens = [int(v) for v in rng.integers(n_fft - 1, 40 * n_fft, 37)]
    tracks = [(rng.standard_normal((n, 2)) * 0.3).astype(np.float32) for n in lens]
    plan = engine.Plan(n_fft, n_fft, hop, engine.OUT_COMPLEX)
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]])
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    fl = plan.row_bins * 2
    guard = 64
    host = np.full(T * fl + 2 * guard, np.float32(-777.25), np.float32)
    outs = []
    for rs in (3, 2, 0):
        dout = engine.DeviceBuffer.from_host(host)
        b = engine.Batch(plan, din, offs, lens, dout.ptr.value + (guard - 32 + shift) * 4,
                         input_format=engine.IN_F32, channels=2, max_blocks=max_blocks, row_store=rs,
                         kernel=3)
        b.run()
        engine.synchronize()
        outs.append(dout.to_host(np.float32))
        b.close()
        dout.close()
    assert outs[0].view(np.uint32).tobytes() == outs[1].view(np.uint32).tobytes() == outs[2].view(np.uint32).tobytes()


@pytest.mark.parametrize("n_fft", [256, 512, 1024])
@pytest.mark.parametrize("max_blocks", [0, 2])
def test_line_rows_all_sizes(n_fft, max_blocks):
    """The whole-line complex row stores at every streaming size (a frame on L = 8 / 16 / 32
    lanes, the carried line spread over 32 / L floats per lane): rows equal the oracle's
    perform_stft within the STFT tolerance, guard floats on both sides untouched, with many
    streams and with few long ones."""
    rng = np.random.default_rng(n_fft + max_blocks)
    hop = n_fft // 4
    lens = [int(v) for v in rng.integers(n_fft - 1, 30 * n_fft, 23)]
    tracks = [(rng.standard_normal((n, 2)) * 0.3).astype(np.float32) for n in lens]
    plan = engine.Plan(n_fft, n_fft, hop, engine.OUT_COMPLEX)
    flat = np.concatenate([t.reshape(-1) for t in tracks])
    offs = np.cumsum([0] + [t.size for t in tracks[:-1]])
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    fl = plan.row_bins * 2
    guard, shift = 64, 14  # rows start 56 bytes into a 128-byte line
    sentinel = np.float32(-4321.5)
    dout = engine.DeviceBuffer.from_host(np.full(T * fl + 2 * guard, sentinel, np.float32))
    b = engine.Batch(plan, din, offs, lens, dout.ptr.value + (guard - 32 + shift) * 4,
                     input_format=engine.IN_F32, channels=2, max_blocks=max_blocks, kernel=3)
    b.run()
    engine.synchronize()
    res = dout.to_host(np.float32)
    lo = guard - 32 + shift
    assert np.all(res[:lo] == sentinel) and np.all(res[lo + T * fl:] == sentinel)
    got = res[lo:lo + T * fl]
    for i, t in enumerate(tracks):
        ref = O.perform_stft(_mono_fold(t), n_fft, hop, n_fft)
        rows = got[int(b.frame0[i]) * fl:int(b.frame0[i + 1]) * fl].view(np.complex64).reshape(ref.shape)
        assert stft_frame_err(rows, ref) <= STFT_REL, i
