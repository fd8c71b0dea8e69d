"""realfft.rs on the GPU: InvRealFFT (realfft.rs:167-241), complex-to-real inverse FFT.

The forward RealFFT (realfft.rs:80-160) runs inside every spectrogram kernel; the inverse is
exposed on its own. Computed in the reference's operation order (rustfft 4.0 Radix4, inverse),
so results equal the reference's f32 arithmetic bit for bit (tests/test_gpu_irfft.py)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import lib, check, _fp


class InvRealFFT:
    """InvRealFFT::new(length): length even (else ValueError, "Length must be even") and a
    power of two (Radix4; the reference panics otherwise)."""

    def __init__(self, length: int):
        if length % 2 > 0:
            raise ValueError("Length must be even")
        self.length = int(length)

    def get_length(self) -> int:
        return self.length

    def process(self, input: np.ndarray) -> np.ndarray:
        """input: [length/2+1] complex (or [frames, length/2+1]) -> [length] (or [frames,
        length]) f32, unnormalised (0.5 * Re of the full inverse DFT)."""
        x = np.ascontiguousarray(input, np.complex64)
        one = x.ndim == 1
        x2 = x.reshape(1, -1) if one else x
        if x2.shape[1] != self.length // 2 + 1:
            raise ValueError(f"Wrong length of input, expected {self.length // 2 + 1}, got {x2.shape[1]}")
        out = np.empty((x2.shape[0], self.length), np.float32)
        check(lib.thesia_inv_real_fft(x2.view(np.float32).ctypes.data_as(_fp), x2.shape[0], self.length,
                                      out.ctypes.data_as(_fp)))
        return out[0] if one else out
