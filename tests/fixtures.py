"""Test / baseline inputs built from the committed fixtures (tests/golden/). Test
infrastructure: no product code imports this module."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
C1_LEN = 2113529  # audio.rs:66: samples/sample.wav (= the missing sample_48k.wav) is [1, 2113529]


def c1_substitute() -> np.ndarray:
    """The 48 kHz stand-in for the missing samples/sample_48k.wav (BASELINE.json configs[0],
    SURVEY.md §8d): the committed 24 kHz sample upsampled 2x (scipy resample_poly), rounded and
    clipped to int16, cut to the 2 113 529 samples audio.rs:66 expects. Returns int16 [n]."""
    from scipy.signal import resample_poly

    x = np.load(os.path.join(GOLDEN, "samples_full.npz"))["pcm_24k"].astype(np.float64)
    y = np.clip(np.round(resample_poly(x, 2, 1)), -32768, 32767).astype(np.int16)
    assert y.shape[0] >= C1_LEN
    return y[:C1_LEN]


def s16_to_f32(x: np.ndarray) -> np.ndarray:
    """hound int -> f32 as open_audio_file does for 16-bit PCM (audio.rs:16-19): i / 2^15."""
    return (x.astype(np.float32) / np.float32(32768.0)).astype(np.float32)


SAMPLE_TAGS = ["8k", "16k", "22k05", "24k", "44k1"]


def samples_full():
    """The five committed sample WAVs whole: [(int16 pcm, sr)] in rate order."""
    z = np.load(os.path.join(GOLDEN, "samples_full.npz"))
    return [(z[f"pcm_{t}"], int(z[f"sr_{t}"])) for t in SAMPLE_TAGS]
