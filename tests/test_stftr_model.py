"""stftr_kernel's index maps on the CPU (tests/stftr_model.py: the kernel's f32 operations with its
lane / register placement made explicit) against the oracle's rfft, bit for bit: the ring layout,
the level order, the permlane swaps, the LDS transpose and the untangle's partner exchange."""
import numpy as np
import pytest

import oracle_ffi as O
import stftr_model as M


def _tables():
    m = np.arange(M.NC, dtype=np.float64)
    ang = -2.0 * np.pi * m / M.NC
    tw = (np.cos(ang).astype(np.float32) + 1j * np.sin(ang).astype(np.float32)).astype(np.complex64)
    return tw, O.rfft_sin_cos(2 * M.NC)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_model_equals_oracle_rfft(seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(2 * M.NC) * np.float32(10.0) ** rng.uniform(-5, 0)).astype(np.float32)
    want = O.rfft(x)
    tw, sc = _tables()
    z = (x[0::2] + 1j * x[1::2]).astype(np.complex64)
    got = M.frame(z, tw, sc)
    bad = got.view(np.uint32) != want.view(np.uint32)
    assert not bad.any(), (int(bad.sum()), np.argwhere(bad.reshape(-1, 2).any(1))[:8].ravel().tolist())
