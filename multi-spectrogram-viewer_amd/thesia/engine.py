"""Batched device engine: HBM buffers, plans (per-geometry tables) and batches (many tracks,
one kernel launch per pass). This is the path bench.py measures."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import lib, check, PlanDesc, BatchDesc, _fp, _u64p

OUT_COMPLEX, OUT_MAG, OUT_POWER, OUT_AMP_DB, OUT_POWER_DB, OUT_MEL, OUT_MEL_AMP_DB = range(7)
IN_F32, IN_S16 = 0, 1
OPT_KERNEL, OPT_MAX_BLOCKS, OPT_ROW_STORE, OPT_RANGE, OPT_MEL_PATH = 1, 2, 3, 4, 5


def device_count() -> int:
    n = C.c_int()
    check(lib.thesia_device_count(C.byref(n)))
    return n.value


def set_device(d: int) -> None:
    check(lib.thesia_set_device(d))


def current_device() -> int:
    """The device the library's calls from this thread use (thesia_get_device)."""
    d = C.c_int()
    check(lib.thesia_get_device(C.byref(d)))
    return d.value


def synchronize() -> None:
    check(lib.thesia_device_synchronize())


def device_info():
    name = C.create_string_buffer(128)
    n = C.c_int()
    check(lib.thesia_device_info(name, 128, C.byref(n)))
    return name.value.decode(), n.value


class EventTimer:
    """HIP events on the library stream: `with EventTimer() as t: ...; t.ms` (device time of the
    work enqueued in between)."""

    def __init__(self):
        self._e0, self._e1 = C.c_void_p(), C.c_void_p()
        check(lib.thesia_event_create(C.byref(self._e0)))
        check(lib.thesia_event_create(C.byref(self._e1)))
        self.ms = 0.0

    def __enter__(self):
        check(lib.thesia_event_record(self._e0, None))
        return self

    def __exit__(self, *exc):
        check(lib.thesia_event_record(self._e1, None))
        ms = C.c_float()
        check(lib.thesia_event_elapsed_ms(self._e0, self._e1, C.byref(ms)))
        self.ms = ms.value
        return False

    def close(self):
        for e in (self._e0, self._e1):
            if e and e.value:
                lib.thesia_event_destroy(e)
        self._e0 = self._e1 = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    """An HBM allocation owned by Python (freed on close / GC)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = C.c_void_p()
        check(lib.thesia_device_malloc(C.byref(self.ptr), max(self.nbytes, 16)))

    @classmethod
    def from_host(cls, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes)
        if arr.nbytes:
            check(lib.thesia_memcpy_h2d(b.ptr, arr.ctypes.data_as(C.c_void_p), arr.nbytes))
        return b

    def to_host(self, dtype, shape=None) -> np.ndarray:
        n = self.nbytes // np.dtype(dtype).itemsize
        out = np.empty(n, dtype)
        if out.nbytes:
            check(lib.thesia_memcpy_d2h(out.ctypes.data_as(C.c_void_p), self.ptr, out.nbytes))
        return out if shape is None else out.reshape(shape)

    def read(self, dtype, count: int, offset_elems: int = 0) -> np.ndarray:
        it = np.dtype(dtype).itemsize
        out = np.empty(count, dtype)
        src = C.c_void_p(self.ptr.value + offset_elems * it)
        check(lib.thesia_memcpy_d2h(out.ctypes.data_as(C.c_void_p), src, count * it))
        return out

    def zero(self):
        check(lib.thesia_memset_device(self.ptr, 0, self.nbytes))

    def close(self):
        if self.ptr and self.ptr.value:
            lib.thesia_device_free(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    """Per-geometry tables resident in HBM (window, twiddles, mel filterbank tiles)."""

    def __init__(self, n_fft: int, win_length: int, hop_length: int, output: int = OUT_AMP_DB,
                 sr: int = 48000, n_mels: int = 0, fmin: float = 0.0, fmax=None, window=None,
                 mel_fb=None):
        d = PlanDesc()
        d.sr, d.win_length, d.hop_length, d.n_fft = sr, win_length, hop_length, n_fft
        self._window = None if window is None else np.ascontiguousarray(window, np.float32)
        self._mel_fb = None if mel_fb is None else np.ascontiguousarray(mel_fb, np.float32)
        d.window = self._window.ctypes.data_as(_fp) if self._window is not None else None
        d.output = output
        d.n_mels = n_mels if mel_fb is None else self._mel_fb.shape[1]
        d.fmin = fmin
        d.fmax = -1.0 if fmax is None else fmax
        d.mel_fb = self._mel_fb.ctypes.data_as(_fp) if self._mel_fb is not None else None
        self.handle = C.c_void_p()
        check(lib.thesia_plan_create(C.byref(d), C.byref(self.handle)))
        self.n_fft, self.win_length, self.hop_length, self.output = n_fft, win_length, hop_length, output
        b = C.c_size_t()
        check(lib.thesia_plan_row_bins(self.handle, C.byref(b)))
        self.row_bins = b.value

    def close(self):
        if self.handle and self.handle.value:
            lib.thesia_plan_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    """Many tracks of one input buffer processed by one plan; output rows packed track after
    track ([total_frames, row_bins])."""

    def __init__(self, plan: Plan, d_input: DeviceBuffer, track_offset, track_len, d_output,
                 input_format: int = IN_F32, channels: int = 1, fold_mono: bool = False,
                 kernel: int = 0, max_blocks: int = 0, row_store: int = 0, mel_path: int = 0):
        """kernel / max_blocks / row_store / mel_path: thesia_batch_set_option (0 = defaults)."""
        self.plan = plan
        self._off = np.ascontiguousarray(track_offset, np.uint64)
        self._len = np.ascontiguousarray(track_len, np.uint64)
        d = BatchDesc()
        d.input_format, d.channels, d.fold_mono = input_format, channels, int(fold_mono)
        d.d_input = d_input.ptr
        d.track_offset = self._off.ctypes.data_as(_u64p)
        d.track_len = self._len.ctypes.data_as(_u64p)
        d.n_tracks = len(self._off)
        d.d_output = d_output.ptr if isinstance(d_output, DeviceBuffer) else d_output
        self.handle = C.c_void_p()
        check(lib.thesia_batch_create(plan.handle, C.byref(d), C.byref(self.handle)))
        tot = C.c_uint64()
        f0 = np.zeros(len(self._off) + 1, np.uint64)
        check(lib.thesia_batch_frames(self.handle, C.byref(tot), f0.ctypes.data_as(_u64p)))
        self.total_frames = tot.value
        self.frame0 = f0
        for opt, v in ((OPT_KERNEL, kernel), (OPT_MAX_BLOCKS, max_blocks), (OPT_ROW_STORE, row_store),
                       (OPT_MEL_PATH, mel_path)):
            if v:
                self.set_option(opt, v)

    def set_option(self, option: int, value: int) -> None:
        check(lib.thesia_batch_set_option(self.handle, option, int(value)))

    @staticmethod
    def frames_for(plan: Plan, track_len) -> int:
        return int(sum(lib.thesia_stft_n_frames(int(n), plan.win_length, plan.hop_length) for n in track_len))

    def run(self, stream=None) -> None:
        check(lib.thesia_batch_run(self.handle, stream))

    def run_timed(self, iters: int = 1, stream=None) -> float:
        ms = C.c_float()
        check(lib.thesia_batch_run_timed(self.handle, stream, iters, C.byref(ms)))
        return ms.value

    def kernel_info(self):
        lds, tile, grid = C.c_int(), C.c_int(), C.c_int()
        check(lib.thesia_batch_kernel_info(self.handle, C.byref(lds), C.byref(tile), C.byref(grid)))
        return {"lds_bytes": lds.value, "tile_frames": tile.value}

    @property
    def kernel(self) -> int:
        """1 stft_kernel, 2 stft2_kernel, 3 stft3_kernel (streaming)."""
        k = C.c_int()
        check(lib.thesia_batch_kernel(self.handle, C.byref(k)))
        return k.value

    def close(self):
        if self.handle and self.handle.value:
            lib.thesia_batch_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ranges_read(d_range: "DeviceBuffer", n: int, offset_tracks: int = 0):
    """THESIA_BATCH_OPT_RANGE slots of n tracks -> (max, min, has_nan) arrays (one readback)."""
    mx = np.empty(n, np.float32)
    mn = np.empty(n, np.float32)
    nan = np.empty(n, np.int32)
    check(lib.thesia_batch_ranges_read(C.c_void_p(d_range.ptr.value + 12 * offset_tracks), n,
                                       mx.ctypes.data_as(C.POINTER(C.c_float)),
                                       mn.ctypes.data_as(C.POINTER(C.c_float)),
                                       nan.ctypes.data_as(C.POINTER(C.c_int))))
    return mx, mn, nan


def run_batches(batches, stream=None) -> None:
    """One pass of every batch, the launches spread over the library's streams and joined back
    to `stream` (thesia_batches_run): the results of calling run() on each."""
    arr = (C.c_void_p * max(len(batches), 1))(*[b.handle.value for b in batches])
    check(lib.thesia_batches_run(arr, len(batches), stream))


def set_batches_policy(policy: int) -> None:
    """thesia_set_batches_policy: 0 (default) = each batch sized for the whole device, the
    batches concurrent on the library streams; 1 = concurrent batches share one occupancy wave by
    work (measured slower); 2 = the batches one after another on the caller's stream."""
    check(lib.thesia_set_batches_policy(policy))


def set_render_path(path: int) -> None:
    """thesia_set_render_path: 0 the fused display with the single-pass kernel where it pays
    (default); 1 per-track launches; 2 three-stage launches; 3 two kernels for every group; 4 the
    single-pass kernel wherever its instances cover the geometry; 5 as 0, plus the single-pass
    kernel's ring mode for the groups below 3 frames per column (all byte-identical)."""
    check(lib.thesia_set_render_path(path))


def render_path() -> int:
    """The library's render path (thesia_get_render_path: whatever set it, this binding or
    another one)."""
    return int(lib.thesia_get_render_path())


def synth_pcm_device(buf: DeviceBuffer, fmt: int, channels: int, n_tracks: int, n_samples: int,
                     sr: int, seed: int = 0) -> None:
    check(lib.thesia_synth_pcm_device(buf.ptr, fmt, channels, n_tracks, n_samples, sr, seed))


def synth_pcm_host(channels: int, track: int, n_samples: int, sr: int, seed: int = 0) -> np.ndarray:
    out = np.empty(n_samples * channels, np.int16)
    check(lib.thesia_synth_pcm_host(out.ctypes.data_as(C.POINTER(C.c_int16)), channels, track,
                                    n_samples, sr, seed))
    return out.reshape(n_samples, channels)
