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


def stft_f64(x: np.ndarray, win: int, hop: int, n_fft: int, window: np.ndarray) -> np.ndarray:
    """The spectrum the reference's f32 path approximates, in float64 (the numpy
    float64 DFT cross-check): the uniform framing rule of lib.rs:367-435 (reflect about 0 and
    N - 1, frame t starts at t * hop - win // 2, the window centred in n_fft), numpy's f64 rfft.
    window: the f32 window values (hann(win) / n_fft), widened to f64."""
    x = np.asarray(x, np.float64)
    n = len(x)
    T = (n + 2 * (win // 2) - win) // hop + 1
    pad_l = (n_fft - win) // 2
    idx = np.arange(T)[:, None] * hop - win // 2 + np.arange(win)[None, :]
    idx = np.abs(idx)
    idx = np.where(idx > n - 1, 2 * (n - 1) - idx, idx)
    fr = np.zeros((T, n_fft))
    fr[:, pad_l:pad_l + win] = x[idx] * np.asarray(window, np.float64)[None, :]
    return np.fft.rfft(fr, axis=1)


def db_err_relative_to_oracle(got_db, oracle_db, exact_db, db_range: float = 120.0):
    """(ii) at full length, where the reference's own f32 arithmetic is what limits agreement:
    the kernel's clamped dB error against the f64 spectrum may be at most max(DB_MAX, 2 x the
    oracle's own error against it) (and likewise at p99.99) -- SURVEY.md §8c contract (i),
    'never worse than 2x ref_cpu's own error vs the f64 DFT', applied to dB. Returns
    (ok, got (max, p99.99), oracle (max, p99.99))."""
    g = db_clamped_err(got_db, exact_db, db_range)
    o = db_clamped_err(oracle_db, exact_db, db_range)
    ok = g[0] <= max(DB_MAX, 2 * o[0]) and g[1] <= max(DB_P9999, 2 * o[1])
    return ok, g, o
