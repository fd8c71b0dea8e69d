"""lib.rs surface: MultiTrack, perform_stft, get_colormap (device-backed)."""
from __future__ import annotations

import ctypes as C
import enum
from typing import Optional, Sequence

import numpy as np

from ._lib import lib, check, _fp, _u8p, _u64p, ERR_BUFFER_TOO_SMALL, ERR_PANIC


class FreqScale(enum.IntEnum):  # lib.rs:25-28
    Linear = 0
    Mel = 1


def get_colormap() -> bytes:
    """lib.rs:473-480: the 10 colormap stops as 30 RGB bytes."""
    buf = (C.c_uint8 * 30)()
    lib.thesia_get_colormap(buf)
    return bytes(buf)


def perform_stft(input, win_length: int, hop_length: int, n_fft: int, window=None,
                 fft_module=None, parallel: bool = False) -> np.ndarray:
    """lib.rs:388-471 on the GPU: [T, n_fft/2+1] complex64. `fft_module` and `parallel` are
    accepted for signature parity; they do not change the numbers (lib.rs:442-468)."""
    x = np.ascontiguousarray(input, np.float32)
    if window is not None:
        window = np.ascontiguousarray(window, np.float32)
        if len(window) != win_length:  # lib.rs:404 assert_eq!
            raise ValueError("window length must equal win_length (lib.rs:404)")
    T = int(lib.thesia_stft_n_frames(len(x), win_length, hop_length))
    out = np.empty((max(T, 1), n_fft // 2 + 1), np.complex64)
    nf = C.c_size_t()
    check(lib.thesia_perform_stft(x.ctypes.data_as(_fp), len(x), win_length, hop_length, n_fft,
                                  window.ctypes.data_as(_fp) if window is not None else None,
                                  out.ctypes.data_as(_fp), out.shape[0], C.byref(nf)))
    return out[: nf.value]


def open_audio_file(path: str):
    """audio.rs:9-37 (WAV, hound semantics): (wav [channels, n] f32, sr)."""
    n, sr, ch = C.c_size_t(), C.c_uint32(), C.c_uint32()
    check(lib.thesia_open_audio_file(path.encode(), None, 0, C.byref(n), C.byref(sr), C.byref(ch)))
    buf = np.empty(n.value, np.float32)
    check(lib.thesia_open_audio_file(path.encode(), buf.ctypes.data_as(_fp), buf.size, C.byref(n),
                                     C.byref(sr), C.byref(ch)))
    return buf.reshape(-1, ch.value).T, sr.value


class MultiTrack:
    """lib.rs:72-365. Tracks, spectrograms and grey images live in HBM."""

    def __init__(self, freq_scale: FreqScale = FreqScale.Mel, win_ms: float = 40.0,
                 t_overlap: int = 4, f_overlap: int = 1, db_range: float = 120.0, fast: bool = False):
        """fast: spectrograms from the streaming kernel (thesia_mt_set_fast; SURVEY §8c's
        end-to-end contract) instead of the reference-order kernel (the oracle's bytes)."""
        self.h = C.c_void_p()
        check(lib.thesia_mt_create(C.byref(self.h)))
        if (freq_scale, win_ms, t_overlap, f_overlap, db_range) != (FreqScale.Mel, 40.0, 4, 1, 120.0):
            check(lib.thesia_mt_set_setting(self.h, win_ms, t_overlap, f_overlap, int(freq_scale), db_range))
        if fast:
            check(lib.thesia_mt_set_fast(self.h, 1))
        self.freq_scale = freq_scale

    def close(self) -> None:
        """Destroy the handle now (wasm-bindgen's free()): its device buffers return to the
        library pool, whose unused reserve is then handed back to the device."""
        if self.h and self.h.value:
            lib.thesia_mt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_tracks(self, id_list: Sequence[int], path_list: str) -> bool:
        """lib.rs:170-191: path_list is '\\n'-separated; returns `changed`."""
        ids = np.ascontiguousarray(id_list, np.uint64)
        ch = C.c_int()
        check(lib.thesia_mt_add_tracks(self.h, ids.ctypes.data_as(_u64p), len(ids),
                                       path_list.encode(), C.byref(ch)))
        return bool(ch.value)

    def add_tracks_pcm(self, id_list: Sequence[int], pcm: Sequence[np.ndarray], sr: Sequence[int],
                       paths: Optional[Sequence[str]] = None) -> bool:
        """add_tracks from decoded audio: each pcm is [n] (mono) or [n, ch] interleaved f32."""
        ids = np.ascontiguousarray(id_list, np.uint64)
        arrs = [np.ascontiguousarray(p if p.ndim == 2 else p[:, None], np.float32) for p in pcm]
        ptrs = (_fp * len(arrs))(*[a.ctypes.data_as(_fp) for a in arrs])
        ns = np.array([a.shape[0] for a in arrs], np.uint64)
        chs = (C.c_uint32 * len(arrs))(*[a.shape[1] for a in arrs])
        srs = (C.c_uint32 * len(arrs))(*sr)
        pl = "\n".join(paths) if paths else ""
        ch = C.c_int()
        check(lib.thesia_mt_add_tracks_pcm(self.h, ids.ctypes.data_as(_u64p), len(ids), ptrs,
                                           ns.ctypes.data_as(_u64p), chs, srs, pl.encode(), C.byref(ch)))
        return bool(ch.value)

    def remove_track(self, id: int) -> bool:
        """lib.rs:265-292."""
        ch = C.c_int()
        check(lib.thesia_mt_remove_track(self.h, id, C.byref(ch)))
        return bool(ch.value)

    def _bytes(self, fn, *args) -> bytes:
        need = C.c_size_t()
        rc = fn(self.h, *args, None, 0, C.byref(need))
        if rc not in (0, -7):
            check(rc)
        buf = (C.c_uint8 * max(need.value, 1))()
        check(fn(self.h, *args, buf, need.value, C.byref(need)))
        return bytes(buf)[: need.value]

    def get_spec_image(self, id: int, px_per_sec: float, nheight: int) -> bytes:
        """lib.rs:294-298: RGB bytes, row-major [nheight][nwidth][3]."""
        return self._bytes(lib.thesia_mt_get_spec_image, id, px_per_sec, nheight)

    def get_wav_image(self, id: int, px_per_sec: float, nheight: int, amp_min: float, amp_max: float,
                      allow_panic: bool = False) -> bytes:
        """lib.rs:300-313: RGBA bytes. Where the reference panics (display.rs:95-108) this
        raises ThesiaError(ERR_PANIC) unless allow_panic (then the clamped image is returned)."""
        need = C.c_size_t()
        rc = lib.thesia_mt_get_wav_image(self.h, id, px_per_sec, nheight, amp_min, amp_max, None, 0,
                                         C.byref(need))
        if rc not in (0, ERR_BUFFER_TOO_SMALL):
            check(rc)
        buf = (C.c_uint8 * max(need.value, 1))()
        rc = lib.thesia_mt_get_wav_image(self.h, id, px_per_sec, nheight, amp_min, amp_max, buf,
                                         need.value, C.byref(need))
        if not (allow_panic and rc == ERR_PANIC):
            check(rc)
        return bytes(buf)[: need.value]

    def get_wav(self, id: int) -> np.ndarray:
        """The track's mono wav as held on the device (audio.rs:9-37 decode + lib.rs:42 sum)."""
        n = C.c_size_t()
        check(lib.thesia_mt_get_wav(self.h, id, None, 0, C.byref(n)))
        out = np.empty(n.value, np.float32)
        check(lib.thesia_mt_get_wav(self.h, id, out.ctypes.data_as(_fp), out.size, C.byref(n)))
        return out

    def get_frequency_hz(self, id: int, relative_freq: float) -> float:
        out = C.c_float()
        check(lib.thesia_mt_get_frequency_hz(self.h, id, relative_freq, C.byref(out)))
        return out.value

    def get_max_db(self) -> float:
        return lib.thesia_mt_get_max_db(self.h)

    def get_min_db(self) -> float:
        return lib.thesia_mt_get_min_db(self.h)

    def get_max_sec(self) -> float:
        return lib.thesia_mt_get_max_sec(self.h)

    def get_sec(self, id: int) -> float:
        out = C.c_float()
        check(lib.thesia_mt_get_sec(self.h, id, C.byref(out)))
        return out.value

    def get_sr(self, id: int) -> int:
        out = C.c_uint32()
        check(lib.thesia_mt_get_sr(self.h, id, C.byref(out)))
        return out.value

    def _str(self, fn, id):
        need = C.c_size_t()
        fn(self.h, id, None, 0, C.byref(need))
        buf = C.create_string_buffer(max(need.value, 1))
        check(fn(self.h, id, buf, need.value, C.byref(need)))
        return buf.value.decode()

    def get_path(self, id: int) -> str:
        return self._str(lib.thesia_mt_get_path, id)

    def get_filename(self, id: int) -> str:
        return self._str(lib.thesia_mt_get_filename, id)

    # -- introspection for parity tests (not part of the reference surface) --
    def get_spec(self, id: int) -> np.ndarray:
        T, B = C.c_size_t(), C.c_size_t()
        check(lib.thesia_mt_get_spec(self.h, id, None, 0, C.byref(T), C.byref(B)))
        out = np.empty((T.value, B.value), np.float32)
        check(lib.thesia_mt_get_spec(self.h, id, out.ctypes.data_as(_fp), out.size, C.byref(T), C.byref(B)))
        return out

    def get_grey(self, id: int) -> np.ndarray:
        w, h = C.c_uint32(), C.c_uint32()
        check(lib.thesia_mt_get_grey(self.h, id, None, 0, C.byref(w), C.byref(h)))
        out = np.empty((h.value, w.value), np.float32)
        check(lib.thesia_mt_get_grey(self.h, id, out.ctypes.data_as(_fp), out.size, C.byref(w), C.byref(h)))
        return out

    def device_bytes(self) -> int:
        """HBM the tracks hold (thesia_mt_device_bytes)."""
        n = C.c_size_t()
        check(lib.thesia_mt_device_bytes(self.h, C.byref(n)))
        return n.value

    def __len__(self):
        n = C.c_size_t()
        check(lib.thesia_mt_track_count(self.h, C.byref(n)))
        return n.value
