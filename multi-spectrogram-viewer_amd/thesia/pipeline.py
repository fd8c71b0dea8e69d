"""Batched spectrogram + display pipeline (BASELINE.json configs[4], "C5": mixed sample rates,
per-track n_fft, dB + colormap render) over the HBM-resident engine.

The reference computes this one track at a time inside MultiTrack (lib.rs:112-136 for the
spectrogram, lib.rs:193-263 for the global range and grey images, lib.rs:294-298 for the RGB
image). Here tracks are grouped by geometry -- (sample rate, n_fft): one Plan (window, tables)
and one Batch (one kernel launch over all the group's tracks) per group -- and the spectrograms
never leave HBM: the per-track max/min, grey image, Lanczos3 resize and colormap run on the
device, and only the RGB bytes come back.

Semantics follow the viewer with FreqScale::Linear (the C5 config names no mel): amp dB
(decibel.rs:79-88), global range max = min(max, 0), min = max(min, max - db_range) over ALL
tracks (lib.rs:194-209; with torch.distributed initialised, over all ranks -- thesia.shard),
up_ratio = max_sr / sr (lib.rs:231-248), nwidth = (px_per_sec * n / sr) as u32 (lib.rs:296).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ._lib import lib, check
from . import engine, shard


@dataclass
class Track:
    pcm: np.ndarray      # [n] or [n, ch]: f32 (open_audio_file scale) or int16 PCM
    sr: int
    n_fft: int
    win_length: int = 0  # 0 => n_fft
    hop_length: int = 0  # 0 => n_fft // 4


@dataclass
class Rendered:
    db: Optional[np.ndarray]  # [T, n_fft/2+1] amp dB (only when keep_db)
    rgb: bytes                # [nheight, nwidth, 3] (display.rs:56-61)
    nwidth: int
    spec_max: float
    spec_min: float


def _geometry(t: Track):
    win = t.win_length or t.n_fft
    hop = t.hop_length or t.n_fft // 4
    ch = 1 if t.pcm.ndim == 1 else t.pcm.shape[1]
    fmt = engine.IN_S16 if t.pcm.dtype == np.int16 else engine.IN_F32
    return (t.sr, t.n_fft, win, hop, ch, fmt)


def render_tracks(tracks: Sequence[Track], px_per_sec: float = 100.0, nheight: int = 500,
                  db_range: float = 120.0, keep_db: bool = False, group=None) -> List[Rendered]:
    """Spectrogram (amp dB) + global range + grey + Lanczos3 + colormap for every track; one
    kernel launch per geometry group. `group`: torch.distributed group for the range exchange
    when tracks are sharded over ranks (None = default group if initialised)."""
    groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
    for i, t in enumerate(tracks):
        groups.setdefault(_geometry(t), []).append(i)

    specs = {}   # track index -> (device buffer, row offset, T, bins) kept alive below
    keep = []
    ranges = {}
    for (sr, n_fft, win, hop, ch, fmt), idx in groups.items():
        plan = engine.Plan(n_fft, win, hop, engine.OUT_AMP_DB, sr=sr)
        flat = np.concatenate([np.ascontiguousarray(tracks[i].pcm).reshape(-1) for i in idx])
        lens = [tracks[i].pcm.shape[0] for i in idx]
        offs = np.cumsum([0] + [tracks[i].pcm.size for i in idx[:-1]]).astype(np.uint64)
        din = engine.DeviceBuffer.from_host(flat)
        T_all = engine.Batch.frames_for(plan, lens)
        dout = engine.DeviceBuffer(T_all * plan.row_bins * 4)
        b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=ch)
        b.run()
        engine.synchronize()
        keep += [plan, din, dout, b]
        for k, i in enumerate(idx):
            f0, f1 = int(b.frame0[k]), int(b.frame0[k + 1])
            specs[i] = (dout, f0 * plan.row_bins, f1 - f0, plan.row_bins)
            ptr = C.c_void_p(dout.ptr.value + f0 * plan.row_bins * 4)
            mx, mn, nan = C.c_float(), C.c_float(), C.c_int()
            check(lib.thesia_minmax_device(ptr, (f1 - f0) * plan.row_bins, C.byref(mx), C.byref(mn),
                                           C.byref(nan)))
            # ndarray-stats max/min error on NaN -> unwrap_or(-inf / +inf) (lib.rs:198-199)
            ranges[i] = (-np.inf, np.inf) if nan.value else (mx.value, mn.value)

    lmx, lmn = shard.local_range([r[0] for r in ranges.values()], [r[1] for r in ranges.values()])
    lsr = max((t.sr for t in tracks), default=0)
    gmax, gmin, max_sr = shard.global_db_range(lmx, lmn, lsr, db_range=db_range, group=group)

    out: List[Rendered] = []
    for i, t in enumerate(tracks):
        dbuf, row0, T, bins = specs[i]
        up = shard.up_ratio(t.sr, max_sr, freq_scale_mel=False)
        H = C.c_uint32()
        check(lib.thesia_spec_grey_height(bins, up, C.byref(H)))
        n = t.pcm.shape[0]
        nwidth = int(np.float32(px_per_sec) * np.float32(n) / np.float32(t.sr))  # lib.rs:296
        grey = engine.DeviceBuffer(max(1, H.value * T) * 4)
        rgb = engine.DeviceBuffer(max(1, nwidth * nheight * 3))
        check(lib.thesia_spec_to_grey_device(C.c_void_p(dbuf.ptr.value + row0 * 4), T, bins, up,
                                             gmax, gmin, grey.ptr))
        check(lib.thesia_grey_to_rgb_device(grey.ptr, T, H.value, nwidth, nheight, rgb.ptr))
        img = rgb.to_host(np.uint8)[: nwidth * nheight * 3].tobytes()
        db = dbuf.read(np.float32, T * bins, row0).reshape(T, bins) if keep_db else None
        out.append(Rendered(db, img, nwidth, *ranges[i]))
        grey.close()
        rgb.close()
    for k in keep[::-1]:
        k.close()
    return out


def c5_tracks(n_tracks: int, seconds: float = 10.0, seed: int = 0, channels: int = 1,
              first: int = 0) -> List[Track]:
    """The C5 generator: rates cycle {8000, 16000, 22050, 24000, 44100, 48000},
    n_fft cycles {256, 512, 1024, 2048}, hop = n_fft/4, win = n_fft; int16-quantised chirp +
    noise from the engine's deterministic generator (track index = seed of the track)."""
    rates = [8000, 16000, 22050, 24000, 44100, 48000]
    ffts = [256, 512, 1024, 2048]
    out = []
    for i in range(first, first + n_tracks):
        sr = rates[i % len(rates)]
        n = int(round(seconds * sr))
        pcm = engine.synth_pcm_host(channels, i, n, sr, seed)
        out.append(Track(pcm[:, 0].copy() if channels == 1 else pcm, sr, ffts[i % len(ffts)]))
    return out
