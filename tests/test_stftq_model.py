"""stftq_kernel's FFT schedule on the CPU (tests/stftq_model.py: rustfft 4.0 Radix4 on L lanes x P
registers, digits moved into registers by lane / register bit swaps) against the oracle's
cfft_tab, bit for bit, for the three sizes the kernel covers (n_fft 256 / 512 / 1024)."""
import numpy as np
import pytest

import oracle_ffi as O
import stftq_model as M


def _tw(nc):
    ang = -2.0 * np.pi * np.arange(nc, dtype=np.float64) / nc
    return (np.cos(ang).astype(np.float32) + 1j * np.sin(ang).astype(np.float32)).astype(np.complex64)


def _w8():
    a = -2.0 * np.pi * np.array([1.0, 3.0]) / 8.0
    return (np.cos(a).astype(np.float32) + 1j * np.sin(a).astype(np.float32)).astype(np.complex64)


@pytest.mark.parametrize("nc", [128, 256, 512])
@pytest.mark.parametrize("seed", [0, 1])
def test_schedule_equals_oracle_cfft(nc, seed):
    rng = np.random.default_rng(seed)
    z = (rng.standard_normal(nc) + 1j * rng.standard_normal(nc)).astype(np.complex64)
    z *= np.complex64(np.float32(10.0) ** rng.uniform(-4, 1))
    want = O.cfft(z)
    got = M.fft(z, _tw(nc), _w8())
    bad = got.view(np.uint32) != want.view(np.uint32)
    assert not bad.any(), (int(bad.sum()), np.argwhere(bad.reshape(-1, 2).any(1))[:8].ravel().tolist())


def test_schedules_print():
    for nc in (128, 256, 512):
        L, P, levels, pbit = M.schedule(nc)
        assert L * P == nc
        for lev in levels:
            assert all(lev["loc"][b][0] == "r" for b in lev["digit"])
