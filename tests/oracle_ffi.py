"""ctypes wrapper over oracle/build/liboracle.so -- the CPU restatement of the reference.

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the parity checker. The product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB_PATH = os.path.join(_ROOT, "oracle", "build", "liboracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_sz = C.c_size_t


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(_ROOT, "oracle")])
        L = C.CDLL(_LIB_PATH)
        sigs = {
            "or_hann_f32": (None, [_sz, C.c_int, _f32p]),
            "or_hann_f64": (None, [_sz, C.c_int, _f64p]),
            "or_calc_proper_n_fft": (_sz, [_sz]),
            "or_pad_reflect_f32": (C.c_int, [_f32p, _sz, _sz, _sz, _f32p]),
            "or_pad_constant_f32": (C.c_int, [_f32p, _sz, _sz, _sz, C.c_float, _f32p]),
            "or_cfft_radix4_f32": (C.c_int, [_f32p, _sz, _f32p]),
            "or_cfft_radix4_f64": (C.c_int, [_f64p, _sz, _f64p]),
            "or_rfft_f32": (C.c_int, [_f32p, _sz, _f32p]),
            "or_rfft_f64": (C.c_int, [_f64p, _sz, _f64p]),
            "or_irfft_f32": (C.c_int, [_f32p, _sz, _f32p]),
            "or_irfft_f64": (C.c_int, [_f64p, _sz, _f64p]),
            "or_rfft_sin_cos_f32": (None, [_sz, _f32p]),
            "or_stft_n_frames": (_sz, [_sz, _sz, _sz]),
            "or_perform_stft_f32": (_sz, [_f32p, _sz, _sz, _sz, _sz, C.c_void_p, _f32p]),
            "or_frames_uniform_f32": (_sz, [_f32p, _sz, _sz, _sz, _sz, C.c_void_p, _f32p]),
            "or_frames_literal_f32": (_sz, [_f32p, _sz, _sz, _sz, _sz, C.c_void_p, _f32p]),
            "or_norm_f32": (None, [_f32p, _sz, _f32p]),
            "or_norm_sqr_f32": (None, [_f32p, _sz, _f32p]),
            "or_amp_to_db_default_f32": (C.c_int, [_f32p, _sz]),
            "or_power_to_db_default_f32": (C.c_int, [_f32p, _sz]),
            "or_hz_to_mel_f32": (C.c_float, [C.c_float]),
            "or_mel_to_hz_f32": (C.c_float, [C.c_float]),
            "or_hz_to_mel_f64": (C.c_double, [C.c_double]),
            "or_mel_to_hz_f64": (C.c_double, [C.c_double]),
            "or_calc_mel_fb_f32": (None, [C.c_uint32, _sz, _sz, C.c_float, C.c_float, C.c_int, _f32p]),
            "or_calc_mel_fb_f64": (None, [C.c_uint32, _sz, _sz, C.c_double, C.c_double, C.c_int, _f64p]),
            "or_calc_mel_fb_default_f32": (_sz, [C.c_uint32, _sz, C.c_void_p]),
            "or_dot_f32": (None, [_f32p, _f32p, _sz, _sz, _sz, _f32p]),
            "or_grey_to_color": (C.c_int, [C.c_float, _u8p]),
            "or_spec_grey_height": (C.c_uint32, [_sz, C.c_float]),
            "or_spec_to_grey": (None, [_f32p, _sz, _sz, C.c_float, C.c_float, C.c_float, _f32p]),
            "or_resize_lanczos3_f32": (None, [_f32p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _f32p]),
            "or_grey_to_rgb": (_sz, [_f32p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _u8p]),
            "or_wav_to_image": (C.c_int, [_f32p, _sz, C.c_uint32, C.c_uint32, C.c_float, C.c_float, _u8p]),
            "or_track_spec_f32": (_sz, [C.c_void_p, _sz, _sz, _sz, _sz, _sz, C.c_int, C.c_void_p, _sz,
                                        C.c_void_p]),
            "or_rfft_mag_rows_f32": (C.c_int, [C.c_void_p, _sz, _sz, _sz, C.c_int, C.c_void_p]),
            "or_track_params": (None, [C.c_uint32, C.c_float, _sz, _sz, C.POINTER(_sz), C.POINTER(_sz), C.POINTER(_sz)]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _c32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def hann(size, symmetric=False, dtype=np.float32):
    if dtype == np.float64:
        out = np.empty(size, np.float64)
        lib().or_hann_f64(size, int(symmetric), out)
    else:
        out = np.empty(size, np.float32)
        lib().or_hann_f32(size, int(symmetric), out)
    return out


def calc_proper_n_fft(win):
    return lib().or_calc_proper_n_fft(win)


def pad_reflect(x, left, right):
    x = _c32(x)
    out = np.empty(len(x) + left + right, np.float32)
    if lib().or_pad_reflect_f32(x, len(x), left, right, out) != 0:
        raise ValueError("reference panics (reflect pad longer than input)")
    return out


def pad_constant(x, left, right, c):
    x = _c32(x)
    out = np.empty(len(x) + left + right, np.float32)
    lib().or_pad_constant_f32(x, len(x), left, right, c, out)
    return out


def cfft(x, dtype=np.float32):
    x = np.ascontiguousarray(np.asarray(x, np.complex128 if dtype == np.float64 else np.complex64))
    n = len(x)
    if dtype == np.float64:
        xin = x.view(np.float64).copy()
        out = np.empty(2 * n, np.float64)
        assert lib().or_cfft_radix4_f64(xin, n, out) == 0
        return out.view(np.complex128)
    xin = x.view(np.float32).copy()
    out = np.empty(2 * n, np.float32)
    assert lib().or_cfft_radix4_f32(xin, n, out) == 0
    return out.view(np.complex64)


def rfft(x, dtype=np.float32):
    n = len(x)
    if dtype == np.float64:
        xin = np.ascontiguousarray(x, np.float64)
        out = np.empty(2 * (n // 2 + 1), np.float64)
        if lib().or_rfft_f64(xin, n, out) != 0:
            raise ValueError("RealFFT length error")
        return out.view(np.complex128)
    xin = _c32(x)
    out = np.empty(2 * (n // 2 + 1), np.float32)
    if lib().or_rfft_f32(xin, n, out) != 0:
        raise ValueError("RealFFT length error")
    return out.view(np.complex64)


def irfft(X, n, dtype=np.float32):
    """InvRealFFT (realfft.rs:167-241): X [n/2+1] complex -> [n] real, unnormalised."""
    if dtype == np.float64:
        xin = np.ascontiguousarray(np.asarray(X, np.complex128)).view(np.float64)
        out = np.empty(n, np.float64)
        if lib().or_irfft_f64(xin, n, out) != 0:
            raise ValueError("InvRealFFT length error")
        return out
    xin = np.ascontiguousarray(np.asarray(X, np.complex64)).view(np.float32)
    out = np.empty(n, np.float32)
    if lib().or_irfft_f32(xin, n, out) != 0:
        raise ValueError("InvRealFFT length error")
    return out


def rfft_sin_cos(n):
    out = np.empty(n, np.float32)
    lib().or_rfft_sin_cos_f32(n, out)
    return out.reshape(-1, 2)


def stft_n_frames(n, win, hop):
    return lib().or_stft_n_frames(n, win, hop)


def perform_stft(x, win, hop, n_fft, window=None):
    """lib.rs:388-471 (literal framing, one RealFFT per frame). Returns [T, F] complex64."""
    x = _c32(x)
    T = lib().or_stft_n_frames(len(x), win, hop)
    if T == 0:
        raise ValueError("reference panics for this (n, win, hop)")
    F = n_fft // 2 + 1
    out = np.empty(T * F * 2, np.float32)
    w = None if window is None else _c32(window)
    wp = None if w is None else w.ctypes.data_as(C.c_void_p)
    got = lib().or_perform_stft_f32(x, len(x), win, hop, n_fft, wp, out)
    assert got == T, (got, T)
    return out.view(np.complex64).reshape(T, F)


def frames(x, win, hop, n_fft, window=None, rule="literal"):
    x = _c32(x)
    fn = lib().or_frames_literal_f32 if rule == "literal" else lib().or_frames_uniform_f32
    w = None if window is None else _c32(window)
    wp = None if w is None else w.ctypes.data_as(C.c_void_p)
    # count first (literal count is data independent)
    T = lib().or_stft_n_frames(len(x), win, hop) if rule == "literal" else (len(x) + 2 * (win // 2) - win) // hop + 1
    out = np.empty(max(T, 1) * n_fft, np.float32)
    got = fn(x, len(x), win, hop, n_fft, wp, out)
    return out[: got * n_fft].reshape(got, n_fft)


def norm(c):
    c = np.ascontiguousarray(c, np.complex64)
    out = np.empty(c.shape, np.float32)
    lib().or_norm_f32(c.view(np.float32).ravel(), c.size, out.ravel())
    return out


def norm_sqr(c):
    c = np.ascontiguousarray(c, np.complex64)
    out = np.empty(c.shape, np.float32)
    lib().or_norm_sqr_f32(c.view(np.float32).ravel(), c.size, out.ravel())
    return out


def amp_to_db_default(x):
    y = _c32(x).copy()
    if lib().or_amp_to_db_default_f32(y.ravel(), y.size) != 0:
        raise ValueError("reference asserts x >= 0")
    return y


def power_to_db_default(x):
    y = _c32(x).copy()
    if lib().or_power_to_db_default_f32(y.ravel(), y.size) != 0:
        raise ValueError("reference asserts x >= 0")
    return y


def hz_to_mel(f, dtype=np.float32):
    return lib().or_hz_to_mel_f64(f) if dtype == np.float64 else np.float32(lib().or_hz_to_mel_f32(f))


def mel_to_hz(m, dtype=np.float32):
    return lib().or_mel_to_hz_f64(m) if dtype == np.float64 else np.float32(lib().or_mel_to_hz_f32(m))


def calc_mel_fb(sr, n_fft, n_mel, fmin=0.0, fmax=None, do_norm=True, dtype=np.float32):
    F = n_fft // 2 + 1
    fm = -1.0 if fmax is None else fmax
    if dtype == np.float64:
        out = np.empty(F * n_mel, np.float64)
        lib().or_calc_mel_fb_f64(sr, n_fft, n_mel, fmin, fm, int(do_norm), out)
    else:
        out = np.empty(F * n_mel, np.float32)
        lib().or_calc_mel_fb_f32(sr, n_fft, n_mel, fmin, fm, int(do_norm), out)
    return out.reshape(F, n_mel)


def calc_mel_fb_default(sr, n_fft):
    F = n_fft // 2 + 1
    n_mel = lib().or_calc_mel_fb_default_f32(sr, n_fft, None)  # size query
    buf = np.empty(F * max(n_mel, 1), np.float32)
    got = lib().or_calc_mel_fb_default_f32(sr, n_fft, buf.ctypes.data_as(C.c_void_p))
    assert got == n_mel
    return buf[: F * n_mel].reshape(F, n_mel)


def dot(a, b):
    a = _c32(a)
    b = _c32(b)
    T, K = a.shape
    K2, M = b.shape
    assert K == K2
    out = np.empty((T, M), np.float32)
    lib().or_dot_f32(a, b, T, K, M, out)
    return out


COLORMAP = np.array([[0, 0, 4], [27, 12, 65], [74, 12, 107], [120, 28, 109], [165, 44, 96],
                     [207, 68, 70], [237, 105, 37], [251, 155, 6], [247, 209, 61],
                     [252, 255, 164]], np.uint8)


def grey_to_color(x):
    out = np.empty(3, np.uint8)
    panicked = lib().or_grey_to_color(x, out)
    return out, bool(panicked)


def spec_to_grey(spec, up_ratio, max_db, min_db):
    spec = _c32(spec)
    T, bins = spec.shape
    H = lib().or_spec_grey_height(bins, up_ratio)
    grey = np.empty(H * T, np.float32)
    lib().or_spec_to_grey(spec, T, bins, up_ratio, max_db, min_db, grey)
    return grey.reshape(H, T)


def resize_lanczos3(img, nw, nh):
    img = _c32(img)
    h, w = img.shape
    out = np.empty(nh * nw, np.float32)
    lib().or_resize_lanczos3_f32(img, w, h, nw, nh, out)
    return out.reshape(nh, nw)


def grey_to_rgb(grey, nw, nh):
    grey = _c32(grey)
    h, w = grey.shape
    out = np.empty(nh * nw * 3, np.uint8)
    panics = lib().or_grey_to_rgb(grey, w, h, nw, nh, out)
    return out.reshape(nh, nw, 3), panics


def wav_to_image(wav, nwidth, nheight, amp_min, amp_max):
    wav = _c32(wav)
    out = np.empty(nheight * nwidth * 4, np.uint8)
    rc = lib().or_wav_to_image(wav, len(wav), nwidth, nheight, amp_min, amp_max, out)
    return out.reshape(nheight, nwidth, 4), rc != 0


def track_params(sr, win_ms=40.0, t_overlap=4, f_overlap=1):
    win, hop, nfft = _sz(), _sz(), _sz()
    lib().or_track_params(sr, win_ms, t_overlap, f_overlap, C.byref(win), C.byref(hop), C.byref(nfft))
    return win.value, hop.value, nfft.value


TRACK_MAG, TRACK_MEL_DB, TRACK_AMP_DB, TRACK_POWER_DB = 0, 1, 2, 3


def track_spec(pcm, win, hop, n_fft, kind, mel_fb=None):
    """or_track_spec_f32: interleaved f32 PCM [n, ch] (or [n]) through the whole spectrogram
    stage in one C call (the GIL is released: the CPU baseline runs these on a thread pool)."""
    pcm = _c32(pcm)
    n = pcm.shape[0]
    ch = 1 if pcm.ndim == 1 else pcm.shape[1]
    T = lib().or_stft_n_frames(n, win, hop)
    if T == 0:
        raise ValueError("reference panics for this (n, win, hop)")
    fb = None if mel_fb is None else _c32(mel_fb)
    cols = fb.shape[1] if kind == TRACK_MEL_DB else n_fft // 2 + 1
    out = np.empty((T, cols), np.float32)
    got = lib().or_track_spec_f32(pcm.ctypes.data, n, ch, win, hop, n_fft, kind,
                                  None if fb is None else fb.ctypes.data, 0 if fb is None else fb.shape[1],
                                  out.ctypes.data)
    assert got == T, (got, T)
    return out


def rfft_mag_rows(frames, t0, t1, out, replan=True):
    """|rfft| of frames[t0:t1] into out[t0:t1] (frames [T, n_fft], out [T, F] f32, C-contiguous;
    one C call, the GIL released)."""
    assert frames.flags.c_contiguous and out.flags.c_contiguous and frames.dtype == np.float32
    rc = lib().or_rfft_mag_rows_f32(frames.ctypes.data, frames.shape[1], t0, t1, int(replan), out.ctypes.data)
    assert rc == 0
