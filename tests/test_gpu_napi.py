"""The viewer's drop-in path driven from JavaScript: the Node-API addon (bindings/napi) loads
libthesia in a node process, which runs MultiTrack.add_tracks on committed WAV fixtures and
get_spec_image / get_wav_image (lib.rs:170-313) on the GPU. The RGB bytes must equal the
all-oracle pipeline from the fixtures' expected samples (decode audio.rs:9-37, channel sum
lib.rs:42, spectrogram lib.rs:112-136, global range lib.rs:193-263, grey + Lanczos3 + colormap
display.rs:44-61), and the RGBA waveform image the oracle's wav_to_image (display.rs:63-115); the reference's panic
there surfaces as a JS exception."""
import base64
import os

import numpy as np
import pytest

import fixtures
import oracle_ffi as O
from napi_util import node_bin, run_node
from thesia import shard

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(node_bin() is None, reason="node is not installed on this box: "
                                 "the N-API addon cannot be loaded (its CPU tests need node too)")]

WAVS = ["s16_stereo_16k", "s24_mono_22k", "f32_stereo_48k"]


def _fold(x, ch):  # lib.rs:42 channel sum, (0 + c0) + c1 ...
    t = x.reshape(-1, ch)
    acc = np.zeros(t.shape[0], np.float32)
    for c in range(ch):
        acc = (acc + t[:, c]).astype(np.float32)
    return acc


def test_napi_multitrack_images_equal_oracle():
    z = np.load(os.path.join(fixtures.GOLDEN, "wav_expected.npz"))
    paths = [os.path.join(fixtures.GOLDEN, "wav", w + ".wav") for w in WAVS]
    r = run_node(f"""
const b64 = a => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString('base64');
const mt = new t.MultiTrack();
const changed = mt.add_tracks(new Uint32Array([0, 1, 2]), {paths!r}.join('\\n'));
const out = {{changed, max_db: mt.get_max_db(), min_db: mt.get_min_db(), max_sec: mt.get_max_sec(),
             srs: [0, 1, 2].map(i => mt.get_sr(i)), names: [0, 1, 2].map(i => mt.get_filename(i)),
             img: {{}}, wav: {{}}}};
for (const i of [0, 1, 2]) {{
  out.img[i] = [b64(mt.get_spec_image(i, 100.0, 300)), b64(mt.get_spec_image(i, 37.5, 120))];
  out.wav[i] = b64(mt.get_wav_image(i, 100.0, 100, -2.0, 2.0));
}}
try {{ mt.get_wav_image(0, 100.0, 100, -1.0, 1.0); out.panic = null; }}  // display.rs:95-108 panics
catch (e) {{ out.panic = e.code; }}
const grab = f => {{ try {{ f(); return null; }} catch (e) {{ return [e.constructor.name, e.code]; }} }};
out.neg_spec = grab(() => mt.get_spec_image(0, 100.0, -5));  // nheight wraps to 2^32 - 5 (ToUint32)
out.neg_wav = grab(() => mt.get_wav_image(0, 100.0, -5, -2.0, 2.0));
out.removed = mt.remove_track(1);
out.after = mt.get_max_db();
mt.free();
console.log(JSON.stringify(out));
""", timeout=300)
    pcm, srs = [], []
    for w in WAVS:
        sr, ch, _ = (int(v) for v in z[w + "/meta"])
        pcm.append(_fold(z[w + "/samples"].astype(np.float32), ch))
        srs.append(sr)
    assert r["srs"] == srs and r["names"] == [w + ".wav" for w in WAVS]
    dbs = []
    for x, sr in zip(pcm, srs):
        win, hop, n_fft = O.track_params(sr)
        w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
        mag = O.norm(O.perform_stft(x, win, hop, n_fft, window=w))
        dbs.append(O.amp_to_db_default(O.dot(mag, O.calc_mel_fb_default(sr, n_fft))))  # Mel default
    gmax = float(np.float32(min(max(float(d.max()) for d in dbs), 0.0)))
    gmin = float(np.float32(max(min(float(d.min()) for d in dbs), gmax - 120.0)))
    assert r["max_db"] == np.float32(gmax) and r["min_db"] == np.float32(gmin)
    for i, (x, sr, db) in enumerate(zip(pcm, srs, dbs)):
        grey = O.spec_to_grey(db, shard.up_ratio(sr, max(srs), freq_scale_mel=True), gmax, gmin)
        for (nh, pps), got64 in zip(((300, 100.0), (120, 37.5)), r["img"][str(i)]):
            nwidth = int(np.float32(pps) * np.float32(len(x)) / np.float32(sr))
            img, _ = O.grey_to_rgb(grey, nwidth, nh)
            got = np.frombuffer(base64.b64decode(got64), np.uint8)
            assert got.size == img.size and int((got != img.reshape(-1)).sum()) == 0, (WAVS[i], nh)
        nwidth = int(np.float32(100.0) * np.float32(len(x)) / np.float32(sr))
        ref = O.wav_to_image(x, nwidth, 100, -2.0, 2.0)[0].reshape(-1)
        got = np.frombuffer(base64.b64decode(r["wav"][str(i)]), np.uint8)
        assert np.array_equal(got, ref), WAVS[i]
    assert r["panic"] == -9  # THESIA_ERR_PANIC: the folded stereo sum leaves [-1, 1]
    # a known id with a negative height (wasm-bindgen's u32 wrap): the image would need terabytes;
    # refused with a RangeError before any host buffer is sized, the process survives
    assert r["neg_spec"] == ["RangeError", "ERR_ARG"] and r["neg_wav"] == ["RangeError", "ERR_ARG"]
    assert isinstance(r["removed"], bool)
