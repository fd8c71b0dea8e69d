"""Parity tolerances (calibrated against fp64): shared by the GPU tests."""
import numpy as np

# (i) complex STFT: per frame |dX| <= 2e-6 * max_k |X_t| vs the oracle
STFT_REL = 2e-6
# (ii)/(iii) dB after the display clamp [max_db - 120, max_db]: max 0.25 dB, p99.99 0.05 dB
DB_MAX = 0.25
DB_P9999 = 0.05


def stft_frame_err(got: np.ndarray, ref: np.ndarray) -> float:
    """max over frames of max_k |got - ref| / max_k |ref| (0 for silent frames that match)."""
    d = np.abs(got.astype(np.complex128) - ref.astype(np.complex128)).max(axis=1)
    s = np.abs(ref.astype(np.complex128)).max(axis=1)
    r = np.where(s > 0, d / np.where(s > 0, s, 1), np.where(d > 0, np.inf, 0.0))
    return float(r.max()) if r.size else 0.0


def db_clamped_err(got_db: np.ndarray, ref_db: np.ndarray, db_range: float = 120.0):
    top = float(np.max(ref_db))
    lo = top - db_range
    g = np.clip(got_db, lo, top)
    r = np.clip(ref_db, lo, top)
    d = np.abs(g.astype(np.float64) - r)
    return float(d.max()), float(np.quantile(d, 0.9999))
