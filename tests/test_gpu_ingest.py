"""The MultiTrack ingest path (f2: audio.rs:9-37 + lib.rs:42 on the device) on the committed
WAV fixtures: samples uploaded in their file encoding, converted and downmixed by
decode_downmix_kernel, every new track of one sample rate in one batched spectrogram launch.
The device mono wav must equal the hound-semantics samples folded in lib.rs:42's order, and
the spectrogram the oracle pipeline's, bit for bit; a failing add_tracks changes nothing."""
import os

import numpy as np
import pytest

import oracle_ffi as O
import thesia

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WAV = os.path.join(HERE, "golden", "wav")


def _fixtures():
    z = np.load(os.path.join(HERE, "golden", "wav_expected.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    return [(n, z[n + "/samples"], z[n + "/meta"]) for n in names]


def _fold(inter, ch):  # lib.rs:42 sum_axis: (0 + c0) + c1 + ... (C < 8)
    x = inter.reshape(-1, ch)
    acc = np.zeros(x.shape[0], np.float32)
    for c in range(ch):
        acc = (acc + x[:, c]).astype(np.float32)
    return acc


def _oracle_spec(x, sr, freq_scale):
    win, hop, n_fft = O.track_params(sr)
    w = O.hann(win) / np.float32(n_fft)
    mag = O.norm(O.perform_stft(x, win, hop, n_fft, window=w.astype(np.float32)))
    if freq_scale == thesia.FreqScale.Mel:
        mag = O.dot(mag, O.calc_mel_fb_default(sr, n_fft))
    return O.amp_to_db_default(mag)


@pytest.mark.parametrize("scale", [thesia.FreqScale.Mel, thesia.FreqScale.Linear])
def test_wav_fixtures_ingest_bit_exact(scale):
    fx = _fixtures()
    mt = thesia.MultiTrack(freq_scale=scale)
    paths = [os.path.join(WAV, n + ".wav") for n, _, _ in fx]
    assert mt.add_tracks(list(range(len(fx))), "\n".join(paths))  # one call: batched per sr
    assert len(mt) == len(fx)
    for i, (name, inter, meta) in enumerate(fx):
        sr, ch = int(meta[0]), int(meta[1])
        assert mt.get_sr(i) == sr
        want = _fold(inter, ch)
        got = mt.get_wav(i)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), name
        spec = mt.get_spec(i)
        ref = _oracle_spec(want, sr, scale)
        assert spec.shape == ref.shape and np.array_equal(spec.view(np.uint32), ref.view(np.uint32)), name


def test_add_tracks_atomic_on_late_failure(tmp_path):
    fx = _fixtures()
    mt = thesia.MultiTrack()
    good = [os.path.join(WAV, n + ".wav") for n, _, _ in fx[:3]]
    assert mt.add_tracks([10], good[0])
    before = (len(mt), mt.get_max_db(), mt.get_min_db(), mt.get_max_sec(), mt.get_wav(10).copy())
    # the last file of the call is too short for its window (lib.rs:413 panics): validation
    # fails after every other file decoded, and nothing of the call may remain
    short = tmp_path / "short.wav"
    sr = 48000
    import struct
    data = np.zeros(16, "<i2").tobytes()
    fmt = struct.pack("<HHIIHH", 1, 1, sr, sr * 2, 2, 16)
    body = b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(data)) + data
    short.write_bytes(b"RIFF" + struct.pack("<I", 4 + len(body)) + b"WAVE" + body)
    with pytest.raises(thesia.ThesiaError) as e:
        mt.add_tracks([10, 11, 12], "\n".join([good[1], good[2], str(short)]))
    assert e.value.code == -4
    after = (len(mt), mt.get_max_db(), mt.get_min_db(), mt.get_max_sec(), mt.get_wav(10))
    assert after[:4] == before[:4] and np.array_equal(after[4], before[4])
    with pytest.raises(thesia.ThesiaError):
        mt.get_sr(11)


def test_wav_image_reports_reference_panic():
    fx = _fixtures()
    mt = thesia.MultiTrack()
    n, inter, meta = fx[0]
    assert mt.add_tracks([0], os.path.join(WAV, n + ".wav"))
    wav = mt.get_wav(0)
    # amp range [min, max] of the wav itself: the column holding the minimum reaches row nheight,
    # where the reference's slice top..bottom+1 overruns (display.rs:102-107)
    lo, hi = float(wav.min()), float(wav.max())
    ref, panicked = O.wav_to_image(wav, 50, 40, lo, hi)
    assert panicked
    with pytest.raises(thesia.ThesiaError) as e:
        mt.get_wav_image(0, 50.0 / (len(wav) / int(meta[0])), 40, lo, hi)
    assert e.value.code == thesia._lib.ERR_PANIC
    img, p = thesia.display.wav_to_image(wav, 50, 40, (lo, hi), return_panic=True)
    assert p and np.array_equal(img, ref)
