"""mel.rs -- mel scale and filterbank (host tables, bit-exact f32 restatement)."""
import ctypes as C

import numpy as np

from ._lib import lib, check, _fp


def hz_to_mel(freq: float) -> float:
    """mel.rs:23-31 (f32)."""
    return float(lib.thesia_hz_to_mel(freq))


def mel_to_hz(mel: float) -> float:
    """mel.rs:13-21 (f32)."""
    return float(lib.thesia_mel_to_hz(mel))


def calc_mel_fb(sr: int, n_fft: int, n_mel: int, fmin: float = 0.0, fmax=None, do_norm: bool = True):
    """mel.rs:33-85 -> [n_fft/2+1, n_mel] f32 (unit-sum normalised filters)."""
    F = n_fft // 2 + 1
    out = np.empty((F, n_mel), np.float32)
    check(lib.thesia_calc_mel_fb(sr, n_fft, n_mel, fmin, -1.0 if fmax is None else fmax,
                                 int(do_norm), out.ctypes.data_as(_fp)))
    return out


def calc_mel_fb_default(sr: int, n_fft: int):
    """mel.rs:87-99: the largest n_mel with no empty filter."""
    n = C.c_size_t()
    check(lib.thesia_calc_mel_fb_default(sr, n_fft, C.byref(n), None, 0))
    F = n_fft // 2 + 1
    out = np.empty((F, n.value), np.float32)
    check(lib.thesia_calc_mel_fb_default(sr, n_fft, C.byref(n), out.ctypes.data_as(_fp), out.size))
    return out
