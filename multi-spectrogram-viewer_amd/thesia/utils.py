"""utils.rs -- calc_proper_n_fft and the AudioTrack parameter derivation."""
import ctypes as C

from ._lib import lib, check


def calc_proper_n_fft(win_length: int) -> int:
    """utils.rs:17-19: 2^ceil(log2(win_length)) in f32 arithmetic."""
    return int(lib.thesia_calc_proper_n_fft(win_length))


def track_params(sr: int, win_ms: float = 40.0, t_overlap: int = 4, f_overlap: int = 1):
    """lib.rs:43-46: (win_length, hop_length, n_fft) for a sample rate."""
    w, h, n = C.c_size_t(), C.c_size_t(), C.c_size_t()
    check(lib.thesia_track_params(sr, win_ms, t_overlap, f_overlap, C.byref(w), C.byref(h), C.byref(n)))
    return w.value, h.value, n.value


def stft_n_frames(n: int, win_length: int, hop_length: int) -> int:
    """Frame count of perform_stft's framing (lib.rs:410-435); 0 where the reference panics."""
    return int(lib.thesia_stft_n_frames(n, win_length, hop_length))
