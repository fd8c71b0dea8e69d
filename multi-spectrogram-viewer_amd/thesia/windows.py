"""windows.rs -- periodic / symmetric Hann (host table, bit-exact f32 restatement)."""
import numpy as np

from ._lib import lib, check, _fp
import ctypes as C


def hann(size: int, symmetric: bool = False) -> np.ndarray:
    """windows::hann (windows.rs:21-30); size > 1 (windows.rs:8 assert)."""
    out = np.empty(size, np.float32)
    check(lib.thesia_hann(size, int(symmetric), out.ctypes.data_as(_fp)))
    return out
