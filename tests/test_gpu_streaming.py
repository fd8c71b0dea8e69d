"""The streaming kernels (stft3_kernel; stft4_kernel at n_fft 2048) against the
oracle on the cases their register ring makes special: streams that cross track ends, tracks that start at odd element
offsets (no 8/16-byte alignment: per-frame reloads), the shortest legal tracks (n = win - 1,
lib.rs:413), frames that reflect at both ends, mono / stereo, f32 / s16, and a grid small enough
that each stream walks hundreds of frames (the shift + prefetch path)."""
import os

import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine
from tolerances import STFT_REL, stft_frame_err

pytestmark = pytest.mark.gpu


def _mono_fold(t):  # lib.rs:42 channel sum, (0 + c0) + c1 ...
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(t.shape[1]):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def _run(n_fft, tracks, channels, fmt, gap, kernel):
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
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=channels)
    assert b.kernel == kernel  # a streaming kernel runs these geometries
    b.run()
    engine.synchronize()
    out = dout.to_host(np.complex64, (T, plan.row_bins))
    return [out[int(b.frame0[i]):int(b.frame0[i + 1])] for i in range(len(tracks))]


@pytest.mark.parametrize("n_fft,kernel", [(256, 3), (1024, 3), (2048, 3), (2048, 4)])
@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap", [0, 3])
def test_streams_across_tracks_edges_and_alignment(n_fft, kernel, channels, fmt, gap, monkeypatch):
    monkeypatch.setenv("THESIA_GRID", "3")  # 3 blocks: every stream walks many frames
    monkeypatch.setenv("THESIA_STFT_KERNEL", str(kernel))
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
