"""The C-ABI library loads and exports every symbol include/thesia.h declares (CPU only)."""
import ctypes as C
import os
import re

import pytest

import thesia
from thesia import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "thesia.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(thesia_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    syms = declared_symbols()
    assert len(syms) > 50
    L = C.CDLL(_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    assert set(declared_symbols()) <= set(_lib.EXPORTED)


def test_library_is_in_tree_and_not_a_fallback():
    assert _lib.LIB_PATH.startswith(ROOT)
    assert thesia.LIB_PATH == _lib.LIB_PATH
    assert b"gfx950" in _lib.lib.thesia_version()


def test_validation_errors_before_device_work():
    from thesia import engine
    with pytest.raises(thesia.ThesiaError) as e:
        engine.Plan(n_fft=1000, win_length=1000, hop_length=250)  # not a power of two
    assert e.value.code == _lib.ERR_UNSUPPORTED
    with pytest.raises(thesia.ThesiaError) as e:
        engine.Plan(n_fft=1024, win_length=2048, hop_length=256)
    assert e.value.code == _lib.ERR_INVALID_ARG
    with pytest.raises(thesia.ThesiaError):
        thesia.windows.hann(1)  # windows.rs:8 assert size > 1
    with pytest.raises(thesia.ThesiaError) as e:
        thesia.perform_stft([0.0, 1.0], 8, 2, 8)  # n < win - 1: lib.rs:413 panic
    assert e.value.code == _lib.ERR_TOO_SHORT


def test_product_library_has_no_experiment_hooks():
    """The shipped library reads no environment variable that changes a kernel: the ablation /
    A-B variants (THESIA_STFT_VARIANT, some of which write wrong output by design) and the
    launch-shape knobs exist only in lib/libthesia_exp.so (`make exp`, -DTHESIA_EXPERIMENTS)."""
    blob = open(_lib.LIB_PATH, "rb").read()
    for name in (b"THESIA_STFT_VARIANT", b"THESIA_GRID", b"THESIA_STFT_KERNEL", b"THESIA_STFT_V1",
                 b"THESIA_RENDER_PER_TRACK", b"THESIA_RENDER_RY", b"THESIA_RENDER_ABL"):
        assert name not in blob, name
