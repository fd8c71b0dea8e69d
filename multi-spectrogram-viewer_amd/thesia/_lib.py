"""ctypes binding of libthesia.so (include/thesia.h).

The product path: every compute call below lands in the HIP kernels of libthesia. There is
no CPU fallback -- if the shared library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("THESIA_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libthesia.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libthesia.so not found at {LIB_PATH}: build it with `make -C multi-spectrogram-viewer_amd` "
        "or `python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")

lib = C.CDLL(LIB_PATH)

_sz = C.c_size_t
_u64 = C.c_uint64
_u32 = C.c_uint32
_f = C.c_float
_i = C.c_int
_vp = C.c_void_p
_fp = C.POINTER(C.c_float)
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)


class PlanDesc(C.Structure):
    _fields_ = [("sr", _u32), ("win_length", _sz), ("hop_length", _sz), ("n_fft", _sz),
                ("window", _fp), ("output", _i), ("n_mels", _sz), ("fmin", _f), ("fmax", _f),
                ("mel_fb", _fp)]


class BatchDesc(C.Structure):
    _fields_ = [("input_format", _i), ("channels", _u32), ("fold_mono", _i), ("d_input", _vp),
                ("track_offset", _u64p), ("track_len", _u64p), ("n_tracks", _sz),
                ("d_output", _vp)]


_SIGS = {
    "thesia_last_error": (C.c_char_p, []),
    "thesia_version": (C.c_char_p, []),
    "thesia_device_count": (_i, [C.POINTER(_i)]),
    "thesia_set_device": (_i, [_i]),
    "thesia_get_device": (_i, [C.POINTER(_i)]),
    "thesia_device_malloc": (_i, [C.POINTER(_vp), _sz]),
    "thesia_device_free": (_i, [_vp]),
    "thesia_memcpy_h2d": (_i, [_vp, _vp, _sz]),
    "thesia_memcpy_d2h": (_i, [_vp, _vp, _sz]),
    "thesia_host_register": (_i, [_vp, _sz]),
    "thesia_host_unregister": (_i, [_vp]),
    "thesia_memset_device": (_i, [_vp, _i, _sz]),
    "thesia_device_synchronize": (_i, []),
    "thesia_pool_trim": (_i, []),
    "thesia_pool_bytes": (_i, [_u64p, _u64p]),
    "thesia_device_info": (_i, [C.c_char_p, _sz, C.POINTER(_i)]),
    "thesia_event_create": (_i, [C.POINTER(_vp)]),
    "thesia_event_destroy": (_i, [_vp]),
    "thesia_event_record": (_i, [_vp, _vp]),
    "thesia_event_elapsed_ms": (_i, [_vp, _vp, _fp]),
    "thesia_hbm_ceiling": (_i, [_vp, _sz, _vp, _sz, _i, _fp, _fp]),
    "thesia_hann": (_i, [_sz, _i, _fp]),
    "thesia_calc_proper_n_fft": (_sz, [_sz]),
    "thesia_hz_to_mel": (_f, [_f]),
    "thesia_mel_to_hz": (_f, [_f]),
    "thesia_calc_mel_fb": (_i, [_u32, _sz, _sz, _f, _f, _i, _fp]),
    "thesia_calc_mel_fb_default": (_i, [_u32, _sz, C.POINTER(_sz), _fp, _sz]),
    "thesia_get_colormap": (None, [_u8p]),
    "thesia_track_params": (_i, [_u32, _f, _sz, _sz, C.POINTER(_sz), C.POINTER(_sz), C.POINTER(_sz)]),
    "thesia_stft_n_frames": (_sz, [_sz, _sz, _sz]),
    "thesia_perform_stft": (_i, [_fp, _sz, _sz, _sz, _sz, _fp, _fp, _sz, C.POINTER(_sz)]),
    "thesia_plan_create": (_i, [C.POINTER(PlanDesc), C.POINTER(_vp)]),
    "thesia_plan_destroy": (_i, [_vp]),
    "thesia_plan_row_bins": (_i, [_vp, C.POINTER(_sz)]),
    "thesia_batch_create": (_i, [_vp, C.POINTER(BatchDesc), C.POINTER(_vp)]),
    "thesia_batch_destroy": (_i, [_vp]),
    "thesia_batch_frames": (_i, [_vp, _u64p, _u64p]),
    "thesia_batch_output_bytes": (_i, [_vp, _u64p]),
    "thesia_batch_run": (_i, [_vp, _vp]),
    "thesia_batches_run": (_i, [_vp, C.c_size_t, _vp]),
    "thesia_batch_run_timed": (_i, [_vp, _vp, _i, _fp]),
    "thesia_batch_kernel_info": (_i, [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i)]),
    "thesia_synth_pcm_device": (_i, [_vp, _i, _u32, _u64, _u64, _u32, _u64]),
    "thesia_synth_pcm_host": (_i, [C.POINTER(C.c_int16), _u32, _u64, _u64, _u32, _u64]),
    "thesia_spec_grey_height": (_i, [_sz, _f, C.POINTER(_u32)]),
    "thesia_spec_to_grey": (_i, [_fp, _sz, _sz, _f, _f, _f, _fp, _sz]),
    "thesia_grey_to_rgb": (_i, [_fp, _u32, _u32, _u32, _u32, _u8p, _sz]),
    "thesia_wav_to_image": (_i, [_fp, _sz, _u32, _u32, _f, _f, _u8p, _sz]),
    "thesia_batch_kernel": (_i, [_vp, C.POINTER(C.c_int)]),
    "thesia_batch_set_option": (_i, [_vp, _i, C.c_int64]),
    "thesia_batch_ranges_read": (_i, [C.c_void_p, _sz, _fp, _fp, C.POINTER(C.c_int)]),
    "thesia_set_batches_policy": (_i, [_i]),
    "thesia_set_render_path": (_i, [_i]),
    "thesia_get_render_path": (_i, []),
    "thesia_minmax_device": (_i, [C.c_void_p, C.c_uint64, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                  C.POINTER(C.c_int)]),
    "thesia_spec_to_grey_device": (_i, [C.c_void_p, _sz, _sz, _f, _f, _f, C.c_void_p]),
    "thesia_grey_to_rgb_device": (_i, [C.c_void_p, _u32, _u32, _u32, _u32, C.c_void_p]),
    "thesia_minmax_segments_device": (_i, [C.c_void_p, _u64p, _sz, _sz, _fp, _fp, C.POINTER(C.c_int)]),
    "thesia_render_rgb_batch_device": (_i, [C.c_void_p, _u64p, _sz, _sz, _fp, C.POINTER(C.c_uint32),
                                            _u32, _f, _f, C.c_void_p, _u64p]),
    "thesia_minmax_segments_multi": (_i, [_sz, C.POINTER(C.c_void_p), C.POINTER(_u64p), C.POINTER(_sz),
                                          C.POINTER(_sz), _fp, _fp, C.POINTER(C.c_int)]),
    "thesia_render_rgb_multi": (_i, [_sz, C.POINTER(C.c_void_p), C.POINTER(_u64p), C.POINTER(_sz),
                                     C.POINTER(_sz), _fp, C.POINTER(C.c_uint32), _u32, _f, _f, C.c_void_p,
                                     _u64p]),
    "thesia_ranges_global": (_i, [C.c_void_p, _sz, _f, C.c_void_p]),
    "thesia_render_rgb_multi_dev": (_i, [_sz, C.POINTER(C.c_void_p), C.POINTER(_u64p), C.POINTER(_sz),
                                         C.POINTER(_sz), _fp, C.POINTER(C.c_uint32), _u32, C.c_void_p,
                                         C.c_void_p, _u64p]),
    "thesia_mt_get_wav": (_i, [_vp, _u64, _fp, _sz, C.POINTER(_sz)]),
    "thesia_inv_real_fft": (_i, [_fp, _sz, _sz, _fp]),
    "thesia_inv_real_fft_device": (_i, [C.c_void_p, _sz, _sz, C.c_void_p]),
    "thesia_open_audio_file": (_i, [C.c_char_p, _fp, _sz, C.POINTER(_sz), C.POINTER(_u32), C.POINTER(_u32)]),
    "thesia_mt_create": (_i, [C.POINTER(_vp)]),
    "thesia_mt_destroy": (None, [_vp]),
    "thesia_mt_set_fast": (_i, [_vp, _i]),
    "thesia_mt_set_setting": (_i, [_vp, _f, _sz, _sz, _i, _f]),
    "thesia_mt_add_tracks": (_i, [_vp, _u64p, _sz, C.c_char_p, C.POINTER(_i)]),
    "thesia_mt_add_tracks_pcm": (_i, [_vp, _u64p, _sz, C.POINTER(_fp), _u64p, C.POINTER(_u32),
                                      C.POINTER(_u32), C.c_char_p, C.POINTER(_i)]),
    "thesia_mt_remove_track": (_i, [_vp, _u64, C.POINTER(_i)]),
    "thesia_mt_get_spec_image": (_i, [_vp, _u64, _f, _u32, _u8p, _sz, C.POINTER(_sz)]),
    "thesia_mt_get_wav_image": (_i, [_vp, _u64, _f, _u32, _f, _f, _u8p, _sz, C.POINTER(_sz)]),
    "thesia_mt_get_frequency_hz": (_i, [_vp, _u64, _f, _fp]),
    "thesia_mt_get_max_db": (_f, [_vp]),
    "thesia_mt_get_min_db": (_f, [_vp]),
    "thesia_mt_get_max_sec": (_f, [_vp]),
    "thesia_mt_get_sec": (_i, [_vp, _u64, _fp]),
    "thesia_mt_get_sr": (_i, [_vp, _u64, C.POINTER(_u32)]),
    "thesia_mt_get_path": (_i, [_vp, _u64, C.c_char_p, _sz, C.POINTER(_sz)]),
    "thesia_mt_get_filename": (_i, [_vp, _u64, C.c_char_p, _sz, C.POINTER(_sz)]),
    "thesia_mt_get_spec": (_i, [_vp, _u64, _fp, _sz, C.POINTER(_sz), C.POINTER(_sz)]),
    "thesia_mt_get_grey": (_i, [_vp, _u64, _fp, _sz, C.POINTER(_u32), C.POINTER(_u32)]),
    "thesia_mt_track_count": (_i, [_vp, C.POINTER(_sz)]),
    "thesia_mt_device_bytes": (_i, [_vp, C.POINTER(_sz)]),
}

for _name, (_res, _args) in _SIGS.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = tuple(_SIGS)

# status codes (thesia.h)
OK = 0
ERR_INVALID_ARG = -1
ERR_IO = -2
ERR_UNKNOWN_ID = -3
ERR_TOO_SHORT = -4
ERR_UNSUPPORTED = -5
ERR_DEVICE = -6
ERR_BUFFER_TOO_SMALL = -7
ERR_NEGATIVE = -8
ERR_PANIC = -9  # the reference panics for these arguments (the output is still written)


class ThesiaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def check(rc: int) -> None:
    if rc != OK:
        raise ThesiaError(rc, lib.thesia_last_error().decode(errors="replace"))
