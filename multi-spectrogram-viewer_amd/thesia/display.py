"""display.rs -- grey images, Lanczos3 resize + colormap, waveform raster (on the GPU)."""
import ctypes as C

import numpy as np

from ._lib import lib, check, _fp, _u8p, ERR_PANIC

COLORMAP = np.array([[0, 0, 4], [27, 12, 65], [74, 12, 107], [120, 28, 109], [165, 44, 96],
                     [207, 68, 70], [237, 105, 37], [251, 155, 6], [247, 209, 61],
                     [252, 255, 164]], np.uint8)  # display.rs:10-21
WAVECOLOR = np.array([200, 21, 103, 255], np.uint8)  # display.rs:22


def spec_to_grey(spec: np.ndarray, up_ratio: float, max: float, min: float) -> np.ndarray:
    """display.rs:44-54: [T, bins] dB -> [H, T] grey, H = round(bins * up_ratio)."""
    spec = np.ascontiguousarray(spec, np.float32)
    T, bins = spec.shape
    h = C.c_uint32()
    check(lib.thesia_spec_grey_height(bins, up_ratio, C.byref(h)))
    out = np.empty((h.value, T), np.float32)
    check(lib.thesia_spec_to_grey(spec.ctypes.data_as(_fp), T, bins, up_ratio, max, min,
                                  out.ctypes.data_as(_fp), out.size))
    return out


def grey_to_rgb(grey: np.ndarray, nwidth: int, nheight: int) -> np.ndarray:
    """display.rs:56-61: Lanczos3 resize to (nwidth, nheight) then colormap -> RGB u8."""
    grey = np.ascontiguousarray(grey, np.float32)
    h, w = grey.shape
    out = np.empty((nheight, nwidth, 3), np.uint8)
    check(lib.thesia_grey_to_rgb(grey.ctypes.data_as(_fp), w, h, nwidth, nheight,
                                 out.ctypes.data_as(_u8p), out.size))
    return out


def wav_to_image(wav: np.ndarray, nwidth: int, nheight: int, amp_range, return_panic: bool = False):
    """display.rs:63-115: min/max envelope in WAVECOLOR -> RGBA u8 [nheight, nwidth, 4]. Where
    the reference panics (display.rs:95-108) this raises ThesiaError(ERR_PANIC); with
    return_panic it returns (image, panicked) instead."""
    wav = np.ascontiguousarray(wav, np.float32)
    out = np.empty((nheight, nwidth, 4), np.uint8)
    rc = lib.thesia_wav_to_image(wav.ctypes.data_as(_fp), wav.size, nwidth, nheight,
                                 float(amp_range[0]), float(amp_range[1]),
                                 out.ctypes.data_as(_u8p), out.size)
    if return_panic and rc == ERR_PANIC:
        return out, True
    check(rc)
    return (out, False) if return_panic else out
