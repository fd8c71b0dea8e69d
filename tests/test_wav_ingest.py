"""WAV parsing with hound 3.4 semantics (audio.rs:9-37) on the host: thesia.open_audio_file
against the committed synthetic fixtures (tests/golden/make_wav_fixtures.py: 8/16/24/32-bit
integer, f32, stereo / 3- / 6-channel, WAVE_FORMAT_EXTENSIBLE, an odd-length chunk before the
data) and, when the reference checkout is present, its own sample WAVs."""
import os

import numpy as np
import pytest

import thesia
from thesia._lib import ERR_IO, ERR_UNSUPPORTED

HERE = os.path.dirname(os.path.abspath(__file__))
WAV = os.path.join(HERE, "golden", "wav")


def _fixtures():
    z = np.load(os.path.join(HERE, "golden", "wav_expected.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    return [(n, z[n + "/samples"], z[n + "/meta"]) for n in names]


@pytest.mark.parametrize("name,expected,meta", _fixtures(), ids=lambda v: v if isinstance(v, str) else "")
def test_open_audio_file_matches_hound_semantics(name, expected, meta):
    wav, sr = thesia.open_audio_file(os.path.join(WAV, name + ".wav"))
    assert sr == int(meta[0]) and wav.shape[0] == int(meta[1])
    assert wav.dtype == np.float32
    got = np.ascontiguousarray(wav.T).reshape(-1)  # back to interleaved [n][ch]
    assert np.array_equal(got.view(np.uint32), expected.view(np.uint32)), name
    if meta[2] < 32 or "f32" not in name:  # integer codes: extremes map to -1 and 1 - 2^(1-bits)
        assert got.min() == -1.0


def test_open_audio_file_errors(tmp_path):
    with pytest.raises(thesia.ThesiaError) as e:
        thesia.open_audio_file(str(tmp_path / "missing.wav"))
    assert e.value.code == ERR_IO and "os error" in str(e.value)
    p = tmp_path / "x.flac"
    p.write_bytes(b"fLaC" + b"\x00" * 64)
    with pytest.raises(thesia.ThesiaError) as e:
        thesia.open_audio_file(str(p))
    assert e.value.code == ERR_UNSUPPORTED  # the rodio fallback is out of scope


REF_SAMPLES = "/root/reference/samples"


@pytest.mark.skipif(not os.path.isdir(REF_SAMPLES), reason="reference checkout not present")
@pytest.mark.parametrize("tag", ["8k", "16k", "22k05", "24k", "44k1"])
def test_reference_sample_wavs(tag):
    # the reference's own 16-bit sample files (its open_audio_works KAT names samples/sample.wav,
    # which the checkout does not hold): length, rate and the committed 1.5 s int16 excerpt
    z = np.load(os.path.join(HERE, "golden", "samples_excerpt.npz"))
    wav, sr = thesia.open_audio_file(os.path.join(REF_SAMPLES, f"sample_{tag}.wav"))
    assert sr == int(z[f"sr_{tag}"]) and wav.shape == (1, int(z[f"len_{tag}"]))
    ex = z[f"pcm_{tag}"]
    want = (ex.astype(np.float32) / np.float32(32768.0)).astype(np.float32)
    assert np.array_equal(wav[0, :ex.size], want)
