"""InvRealFFT on the device (irfftx_kernel) against the oracle restatement, bit for bit, at
every power-of-two length the engine serves, many frames per launch; the forward / inverse
round trip at full size; the reference's length errors."""
import numpy as np
import pytest

import oracle_ffi as O
import thesia
from thesia.realfft import InvRealFFT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2 ** k for k in range(1, 13)])
def test_inv_real_fft_bit_exact(n):
    rng = np.random.default_rng(3 * n)
    frames = max(1, min(64, (1 << 16) // n))
    X = (rng.normal(size=(frames, n // 2 + 1)) + 1j * rng.normal(size=(frames, n // 2 + 1))).astype(np.complex64)
    X[1 % frames] = 0
    got = InvRealFFT(n).process(X)
    for f in range(frames):
        ref = O.irfft(X[f], n)
        assert np.array_equal(got[f].view(np.uint32), ref.view(np.uint32)), (n, f)


def test_round_trip_full_size():
    n, frames = 4096, 2000
    rng = np.random.default_rng(5)
    x = rng.normal(size=(frames, n)).astype(np.float32)
    X = np.fft.rfft(x.astype(np.float64), axis=1).astype(np.complex64)
    y = InvRealFFT(n).process(X)
    assert np.abs(y / (n / 2) - x).max() < 1e-4


def test_length_errors():
    with pytest.raises(ValueError):
        InvRealFFT(7)
    with pytest.raises(thesia.ThesiaError):
        InvRealFFT(12).process(np.zeros(7, np.complex64))
    with pytest.raises(ValueError):
        InvRealFFT(8).process(np.zeros(4, np.complex64))
    with pytest.raises(thesia.ThesiaError):
        InvRealFFT(8192).process(np.zeros(4097, np.complex64))  # beyond the engine's n_fft range
