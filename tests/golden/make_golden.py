"""Regenerates the committed golden fixtures (run in the build container, where the
reference is mounted at /root/reference; the GPU box never reads the reference).

1. kats.json -- the expected values the reference's own unit tests assert, transcribed
   from the test bodies (values only; no reference source is copied):
     windows.rs:35-38  hann(4, false)
     utils.rs:117-123  rfft(impulse(4, 0))
     utils.rs:125-140  pad constant / reflect
     lib.rs:491-514    perform_stft(impulse(4, 2), 4, 2, 4)
     mel.rs:107-113    hz <-> mel (f64, 1e-14)
     mel.rs:115-133    first 8 weights of calc_mel_fb(24000, 2048, 80) (STALE: Slaney norm)
     realfft.rs:253-272 2-spike input, eps 1e-15 vs a complex FFT (recomputed with numpy)
     audio.rs:44-70    the missing 48 kHz sample's expected header (documentation only)
2. samples_excerpt.npz -- int16 excerpts (first 1.5 s) of the reference's sample WAVs
   (data fixtures from /root/reference/samples), keyed by sample rate, plus full lengths.
3. samples_full.npz -- the five sample WAVs whole (int16, 44.03 s each): config C2 at the size
   BASELINE.json names, and (the 24 kHz one, 1 056 765 samples) the source of the 48 kHz
   substitute for the missing samples/sample_48k.wav (config C1, SURVEY.md §8d;
   tests/fixtures.py c1_substitute).
"""
import json
import os
import wave

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def kats():
    x = np.zeros(256)
    x[0] = 1.0
    x[3] = 0.5
    return {
        "hann_4_periodic": [0.0, 0.5, 1.0, 0.5],
        "rfft_impulse_4_0": [[1.0, 0.0], [1.0, 0.0], [1.0, 0.0]],
        "pad_constant": {"input": [[1, 2, 3]], "pad": [1, 2], "axis": 0, "value": 10,
                         "expected": [[10, 10, 10], [1, 2, 3], [10, 10, 10], [10, 10, 10]]},
        "pad_reflect": {"input": [1, 2, 3], "pad": [1, 2], "expected": [2, 1, 2, 3, 2, 1]},
        "stft_impulse": {"input": [0.0, 0.0, 1.0, 0.0], "win": 4, "hop": 2, "n_fft": 4,
                         "expected": [[[0, 0], [0, 0], [0, 0]],
                                      [[0.25, 0], [-0.25, 0], [0.25, 0]],
                                      [[0.25, 0], [-0.25, 0], [0.25, 0]]]},
        "mel_hz": {"hz_to_mel": [[100.0, 1.5], [1100.0, 16.38629404765444]],
                   "mel_to_hz": [[1.0, 66.66666666666667], [16.0, 1071.1702874944676]],
                   "eps": 1e-14},
        "mel_works_stale_slaney": {
            "sr": 24000, "n_fft": 2048, "n_mel": 80,
            "first8_of_filter0": [0.0, 6.613916251808404922e-03, 1.322783250361680984e-02,
                                  1.984174735844135284e-02, 2.105801925063133240e-02,
                                  1.444410253316164017e-02, 7.830185815691947937e-03,
                                  1.216269447468221188e-03],
            "eps": 1e-8},
        "real_to_complex": {"n": 256, "spikes": [[0, 1.0], [3, 0.5]], "eps": 1e-15,
                            "expected_first4": [[float(v.real), float(v.imag)] for v in np.fft.fft(x)[:4]]},
        "open_audio_48k_missing": {"sr": 48000, "shape": [1, 2113529], "max": 0.234344482421875,
                                   "min": -0.20355224609375},
        "mel_default_property": {"srs": [400, 800, 1000, 2000, 4000, 8000, 16000, 24000, 44100,
                                         48000, 88200, 96000], "n_fft_exp": [5, 15]},
    }


def samples():
    out = {}
    for tag in ["8k", "16k", "22k05", "24k", "44k1"]:
        p = os.path.join(REF, "samples", f"sample_{tag}.wav")
        w = wave.open(p)
        sr, n = w.getframerate(), w.getnframes()
        assert w.getnchannels() == 1 and w.getsampwidth() == 2
        k = int(1.5 * sr)
        data = np.frombuffer(w.readframes(k), np.int16)
        out[f"pcm_{tag}"] = data
        out[f"sr_{tag}"] = np.array(sr)
        out[f"len_{tag}"] = np.array(n)
    return out


def samples_full():
    """The five committed sample WAVs whole (int16 mono, 44.03 s each): BASELINE.json configs[1]
    (C2) names them at full length; the 24 kHz one is also the source of the 48 kHz substitute."""
    out = {}
    for tag in ["8k", "16k", "22k05", "24k", "44k1"]:
        w = wave.open(os.path.join(REF, "samples", f"sample_{tag}.wav"))
        assert w.getnchannels() == 1 and w.getsampwidth() == 2
        out[f"pcm_{tag}"] = np.frombuffer(w.readframes(w.getnframes()), np.int16)
        out[f"sr_{tag}"] = np.array(w.getframerate())
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "samples_excerpt.npz"), **samples())
    np.savez_compressed(os.path.join(HERE, "samples_full.npz"), **samples_full())
    print("wrote kats.json, samples_excerpt.npz, samples_full.npz")
