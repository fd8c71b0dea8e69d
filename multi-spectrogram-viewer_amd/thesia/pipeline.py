"""Batched spectrogram + display pipeline (BASELINE.json configs[4], "C5": mixed sample rates,
per-track n_fft, dB + colormap render) over the HBM-resident engine.

The reference computes this one track at a time inside MultiTrack (lib.rs:112-136 for the
spectrogram, lib.rs:193-263 for the global range and grey images, lib.rs:294-298 for the RGB
image). Here tracks are grouped by geometry -- n_fft / win / hop: one Plan (window, tables)
and one Batch (one kernel launch over all the group's tracks) per group -- and the spectrograms
never leave HBM: the per-track max/min, grey image, Lanczos3 resize and colormap run on the
device, and only the RGB bytes come back. (Amp dB rows do not depend on the rate, so the
spectrogram batches are per (n_fft, win, hop, layout) with every rate inside; the display
groups are per batch and rate.)

Semantics follow the viewer with FreqScale::Linear (the C5 config names no mel): amp dB
(decibel.rs:79-88), global range max = min(max, 0), min = max(min, max - db_range) over ALL
tracks (lib.rs:194-209; with torch.distributed initialised, over all ranks -- thesia.shard),
up_ratio = max_sr / sr (lib.rs:231-248), nwidth = (px_per_sec * n / sr) as u32 (lib.rs:296).
"""
from __future__ import annotations

import ctypes as C
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ._lib import lib, check, _fp, _u64p
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
    rgb: np.ndarray           # u8 [nheight * nwidth * 3] (display.rs:56-61; a view of the
                              # call's one device-to-host copy)
    nwidth: int
    spec_max: float
    spec_min: float


def _geometry(t: Track):
    """The spectrogram batch a track joins: amp dB rows do not depend on the sample rate (the
    window is hann(win) / n_fft, lib.rs:138-140; the rate only picks the mel filterbank), so
    tracks of every rate with one n_fft / win / hop / layout share one launch."""
    win = t.win_length or t.n_fft
    hop = t.hop_length or t.n_fft // 4
    ch = 1 if t.pcm.ndim == 1 else t.pcm.shape[1]
    fmt = engine.IN_S16 if t.pcm.dtype == np.int16 else engine.IN_F32
    return (t.n_fft, win, hop, ch, fmt)


class RenderPipeline:
    """The C5 pipeline with its inputs resident in HBM: `prepare` uploads the tracks and builds
    one Plan + Batch per geometry group; `run_spectrograms` is one launch per group; `render`
    runs the global-range exchange and the device display path for every track. `render` with
    want_rgb=False and keep_db=False on one rank is asynchronous and returns None (the images
    stay in HBM); otherwise it returns one Rendered per track."""

    def __init__(self, tracks: Sequence[Track], px_per_sec: float = 100.0, nheight: int = 500,
                 db_range: float = 120.0, pinned_output: bool = False, kernel: int = 0):
        """pinned_output: read the RGB images back into one page-locked host buffer (one
        DMA-rate copy per render); the returned images are then views that the next
        render() overwrites. Default: fresh pageable arrays per render().
        kernel: the spectrogram kernel of every batch (0 = automatic; 7 = the streaming
        reference-order kernels (stftr / stftq), 9 = the one-wave-per-frame one: images equal to
        the oracle pipeline's bytes; thesia_batch_set_option)."""
        self.tracks = list(tracks)
        self.pinned_output = pinned_output
        self._pinned = {}  # group -> registered host array
        self.px_per_sec, self.nheight, self.db_range = px_per_sec, nheight, db_range
        groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
        for i, t in enumerate(self.tracks):
            groups.setdefault(_geometry(t), []).append(i)
        self.groups = []  # spectrogram batches: (plan, din, dout, batch), one launch each
        self.where = {}  # track -> (group index, row offset, T, bins)
        # display groups: the tracks of one batch and one sample rate (contiguous in the batch:
        # tracks are ordered by rate inside it), so the display's tap counts follow the rate
        disp = []  # (batch index, first track in the batch, count)
        for (n_fft, win, hop, ch, fmt), idx in groups.items():
            idx.sort(key=lambda i: (self.tracks[i].sr, i))
            plan = engine.Plan(n_fft, win, hop, engine.OUT_AMP_DB, sr=self.tracks[idx[0]].sr)
            flat = np.concatenate([np.ascontiguousarray(self.tracks[i].pcm).reshape(-1) for i in idx])
            lens = [self.tracks[i].pcm.shape[0] for i in idx]
            offs = np.cumsum([0] + [self.tracks[i].pcm.size for i in idx[:-1]]).astype(np.uint64)
            din = engine.DeviceBuffer.from_host(flat)
            T_all = engine.Batch.frames_for(plan, lens)
            dout = engine.DeviceBuffer(T_all * plan.row_bins * 4)
            b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=ch, kernel=kernel)
            g = len(self.groups)
            self.groups.append((plan, din, dout, b))
            k0 = 0
            for k, i in enumerate(idx):
                f0, f1 = int(b.frame0[k]), int(b.frame0[k + 1])
                self.where[i] = (g, f0 * plan.row_bins, f1 - f0, plan.row_bins)
                if k + 1 == len(idx) or self.tracks[idx[k + 1]].sr != self.tracks[i].sr:
                    disp.append((g, k0, k + 1 - k0))
                    k0 = k + 1
        self._batch_order = [i for idx in groups.values() for i in idx]
        self.total_frames = sum(grp[3].total_frames for grp in self.groups)
        # display geometry, fixed for the pipeline's life: every group in one library call
        # (thesia_minmax_segments_multi / thesia_render_rgb_multi), tracks in group order
        self._geo = []
        for i, t in enumerate(self.tracks):
            self._geo.append(int(np.float32(px_per_sec) * np.float32(t.pcm.shape[0]) / np.float32(t.sr)))
        self._order = np.array(self._batch_order, np.int64)  # = display groups in order
        ng = len(disp)
        self._row0 = [np.ascontiguousarray(b.frame0, np.uint64) for _, _, _, b in self.groups]
        self._c_specs = (C.c_void_p * max(ng, 1))(*[self.groups[g][2].ptr.value for g, _, _ in disp])
        self._c_row0 = (_u64p * max(ng, 1))(*[C.cast(self._row0[g].ctypes.data + 8 * k0, _u64p)
                                             for g, k0, _ in disp])
        self._c_bins = (C.c_size_t * max(ng, 1))(*[self.groups[g][0].row_bins for g, _, _ in disp])
        self._c_ns = (C.c_size_t * max(ng, 1))(*[n for _, _, n in disp])
        self._n_disp = ng
        self._nw = np.array([self._geo[i] for i in self._order], np.uint32)
        self._sizes = self._nw.astype(np.uint64) * nheight * 3
        self._off = np.concatenate([[0], np.cumsum(self._sizes)[:-1]]).astype(np.uint64)
        self._rgb_total = int(self._sizes.sum())
        self._rgb = engine.DeviceBuffer(max(self._rgb_total, 1))
        # per-track dB ranges left by the spectrogram launches themselves (Batch range option,
        # folded into the streaming kernel's row epilogue): 3 int32 per track, call order
        self._d_range = engine.DeviceBuffer(12 * max(len(self._order), 1))
        self._d_grange = engine.DeviceBuffer(8)  # the device-side global (max, min), render()
        t0 = 0
        for _, _, _, b in self.groups:
            b.set_option(engine.OPT_RANGE, self._d_range.ptr.value + 12 * t0)
            t0 += len(b.frame0) - 1
        self._up = {}  # max_sr -> up_ratio per track (call order)
        self._max_sr = max((t.sr for t in self.tracks), default=0)

    def run_spectrograms(self) -> None:
        """One kernel launch per geometry group, the launches overlapped on the library's
        streams (thesia_batches_run; asynchronous, ordered before later library calls)."""
        engine.run_batches([b for _, _, _, b in self.groups])

    def _up_for(self, max_sr):
        up = self._up.get(max_sr)
        if up is None:
            up = np.array([shard.up_ratio(self.tracks[i].sr, max_sr, freq_scale_mel=False)
                           for i in self._order.tolist()], np.float32)
            self._up[max_sr] = up
        return up

    def _spec_ptr(self, i):
        g, row0, T, bins = self.where[i]
        return C.c_void_p(self.groups[g][2].ptr.value + row0 * 4), T, bins

    def _range_arrays(self):
        """(max, min) dB per track in call order (group order), NaN-holding tracks as -inf /
        +inf (ndarray-stats max/min error on NaN -> unwrap_or, lib.rs:198-199): the ranges the
        last run_spectrograms() left (one readback)."""
        mx, mn, nan = engine.ranges_read(self._d_range, len(self._order))
        bad = nan != 0
        return np.where(bad, -np.inf, mx.astype(np.float64)), np.where(bad, np.inf, mn.astype(np.float64))

    def ranges(self):
        """Per-track (max, min) dB (lib.rs:194-207), indexed like self.tracks."""
        mx, mn = self._range_arrays()
        out = [None] * len(self.tracks)
        for k, i in enumerate(self._order.tolist()):
            out[i] = (float(mx[k]), float(mn[k]))
        return out

    def _single_rank(self, group) -> bool:
        try:
            import torch.distributed as dist
            return not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1)
        except ImportError:  # pragma: no cover - torch is in the image
            return True

    def render(self, group=None, keep_db: bool = False, want_rgb: bool = True) -> Optional[List[Rendered]]:
        """The global-range exchange and the display of every track. want_rgb=False and
        keep_db=False on one rank: the range is reduced on the device (thesia_ranges_global)
        and the display reads it there (thesia_render_rgb_multi_dev), so nothing waits for the
        spectrograms on the host; the images stay in HBM and None is returned (asynchronous).
        Otherwise the ranges come back to the host (the multi-rank exchange, the per-track
        results) and the rendered tracks are returned."""
        # (THESIA_HOST_RANGE=1 in the environment keeps the host exchange: A/B)
        if (not want_rgb and not keep_db and engine.render_path() in (0, 3, 4) and self._single_rank(group)
                and os.environ.get("THESIA_HOST_RANGE") != "1"):
            check(lib.thesia_ranges_global(self._d_range.ptr, len(self._order), self.db_range, self._d_grange.ptr))
            up = self._up_for(self._max_sr)
            check(lib.thesia_render_rgb_multi_dev(
                self._n_disp, self._c_specs, self._c_row0, self._c_bins, self._c_ns,
                up.ctypes.data_as(_fp), self._nw.ctypes.data_as(C.POINTER(C.c_uint32)), self.nheight,
                self._d_grange.ptr, self._rgb.ptr, self._off.ctypes.data_as(_u64p)))
            return None
        # (the range readback is ordered on the library stream after the spectrogram batches,
        # which thesia_batches_run joins back into it, and waits for it: no device-wide sync)
        mx, mn = self._range_arrays()
        lmx = float(mx.max()) if mx.size else -np.inf  # shard.local_range over numpy arrays
        lmn = float(mn.min()) if mn.size else np.inf
        gmax, gmin, max_sr = shard.global_db_range(lmx, lmn, self._max_sr, db_range=self.db_range, group=group)
        up = self._up_for(max_sr)
        check(lib.thesia_render_rgb_multi(
            self._n_disp, self._c_specs, self._c_row0, self._c_bins, self._c_ns,
            up.ctypes.data_as(_fp), self._nw.ctypes.data_as(C.POINTER(C.c_uint32)), self.nheight,
            gmax, gmin, self._rgb.ptr, self._off.ctypes.data_as(_u64p)))
        total = self._rgb_total
        if want_rgb and self.pinned_output:
            rgb_all = self._pinned_host(0, total)
            check(lib.thesia_memcpy_d2h(rgb_all.ctypes.data_as(C.c_void_p), self._rgb.ptr, total))
            rgb_all = rgb_all[:total]
        else:
            rgb_all = self._rgb.read(np.uint8, total) if want_rgb else None
        out: List[Optional[Rendered]] = [None] * len(self.tracks)
        for k, i in enumerate(self._order.tolist()):
            o, sz = int(self._off[k]), int(self._sizes[k])
            img = rgb_all[o:o + sz] if want_rgb else None
            db = None
            if keep_db:
                g, row_el, T, bins = self.where[i]
                db = self.groups[g][2].read(np.float32, T * bins, row_el).reshape(T, bins)
            out[i] = Rendered(db, img, self._geo[i], float(mx[k]), float(mn[k]))
        return out

    def display_bytes(self) -> dict:
        """HBM bytes of one display pass (DESIGN.md §4 'Display roofline'). `total` is the
        algorithmic minimum: the dB spectrogram read once and the RGB bytes written once. The
        separable resize's f32 intermediate [nheight, T] (image 0.23's vertical-then-horizontal
        order) is an implementation's choice, reported apart as an upper bound (the fused path
        neither forms nor reads the rows whose taps reach only the zero fill)."""
        spec = tmp = rgb = 0
        for i, t in enumerate(self.tracks):
            _, _, T, bins = self.where[i]
            spec += T * bins * 4
            tmp += T * self.nheight * 4
            rgb += self._geo[i] * self.nheight * 3
        return {"spec_read": spec, "rgb_write": rgb, "total": spec + rgb,
                "intermediate_write_read_upper_bound": 2 * tmp}

    def display_timed(self, iters: int = 3) -> dict:
        """Device time of the display path (range + grey + Lanczos3 + colormap, no host copy),
        HIP events on the library stream, and its HBM-roofline fraction on the algorithmic
        bytes (spectrogram read + RGB written once)."""
        engine.synchronize()
        self.render(want_rgb=False)  # warm (workspaces, tap tables)
        with engine.EventTimer() as tm:
            for _ in range(iters):
                self.render(want_rgb=False)
        ms = tm.ms / iters
        b = self.display_bytes()
        ach = b["total"] / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0,
                "traffic": None,
                "display_ms": ms, "algorithmic_bytes": b,
                "kernel": "per-track range + grey/vertical Lanczos3 + horizontal Lanczos3 + colormap"}

    def _pinned_host(self, g: int, total: int) -> np.ndarray:
        buf = self._pinned.get(g)
        if buf is None or buf.nbytes < total:
            if buf is not None:
                check(lib.thesia_host_unregister(buf.ctypes.data_as(C.c_void_p)))
            buf = np.empty(max(total, 1), np.uint8)
            check(lib.thesia_host_register(buf.ctypes.data_as(C.c_void_p), buf.nbytes))
            self._pinned[g] = buf
        return buf

    def close(self):
        for buf in self._pinned.values():
            lib.thesia_host_unregister(buf.ctypes.data_as(C.c_void_p))
        self._pinned = {}
        for plan, din, dout, b in self.groups[::-1]:
            b.close()
            dout.close()
            din.close()
            plan.close()
        self.groups = []
        self._rgb.close()
        self._d_range.close()


def render_tracks(tracks: Sequence[Track], px_per_sec: float = 100.0, nheight: int = 500,
                  db_range: float = 120.0, keep_db: bool = False, group=None, kernel: int = 0) -> List[Rendered]:
    """Spectrogram (amp dB) + global range + grey + Lanczos3 + colormap for every track; one
    kernel launch per geometry group. `group`: torch.distributed group for the range exchange
    when tracks are sharded over ranks (None = default group if initialised). `kernel`: as
    RenderPipeline's (7 / 9: the reference-order kernels, images equal to the oracle's bytes)."""
    p = RenderPipeline(tracks, px_per_sec, nheight, db_range, kernel=kernel)
    try:
        p.run_spectrograms()
        return p.render(group=group, keep_db=keep_db)
    finally:
        p.close()


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
