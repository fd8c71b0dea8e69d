"""The oracle's InvRealFFT restatement (realfft.rs:167-241 over rustfft 4.0 Radix4, inverse),
pinned by the reference's own complex_to_real test (realfft.rs:274-296: f64, epsilon 1e-15
against 0.5 * Re of the full inverse FFT) and by numpy at every power-of-two length."""
import numpy as np
import pytest

import oracle_ffi as O


def test_reference_complex_to_real_kat():
    ind = np.zeros(256, np.complex128)
    ind[0] = 1.0
    ind[1] = 1.0 + 0.4j
    ind[255] = 1.0 - 0.4j
    ind[3] = 0.3 + 0.2j
    ind[253] = 0.3 - 0.2j
    out_a = O.irfft(ind[:129], 256, np.float64)
    out_b = 0.5 * (np.fft.ifft(ind) * 256).real
    assert np.abs(out_a - out_b).max() <= 1e-15


@pytest.mark.parametrize("n", [2 ** k for k in range(1, 15)])
def test_irfft_matches_numpy(n):
    rng = np.random.default_rng(n)
    X = rng.normal(size=n // 2 + 1) + 1j * rng.normal(size=n // 2 + 1)
    X[0], X[-1] = X[0].real, X[-1].real  # a real signal's spectrum (numpy drops these parts)
    ref = np.fft.irfft(X, n) * (n / 2)
    got64 = O.irfft(X, n, np.float64)
    assert np.abs(got64 - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())
    got32 = O.irfft(X, n, np.float32)
    assert np.abs(got32 - ref).max() <= 2e-6 * np.abs(ref).max()


def test_irfft_length_errors():
    with pytest.raises(ValueError):
        O.irfft(np.zeros(4, np.complex64), 7)  # odd: "Length must be even"
    with pytest.raises(ValueError):
        O.irfft(np.zeros(7, np.complex64), 12)  # Radix4 needs a power of two
