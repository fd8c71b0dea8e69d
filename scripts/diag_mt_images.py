"""Debug aid: MultiTrack images on a 400 000-frame 48 kHz mel batch against the oracle display of
the oracle's dB rows under the MultiTrack's own range. Test infrastructure."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))

import fixtures  # noqa: E402
import oracle_ffi as O  # noqa: E402
import thesia  # noqa: E402
from thesia import engine, shard  # noqa: E402

sr = 48000
secs = int(sys.argv[1]) if len(sys.argv) > 1 else 250
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
n = secs * sr
pcm = [fixtures.s16_to_f32(engine.synth_pcm_host(1, i, n, sr, seed=5)).reshape(-1) for i in range(k)]
win, hop, n_fft = O.track_params(sr)
fb = O.calc_mel_fb_default(sr, n_fft)
x0 = pcm[0]
db = O.amp_to_db_default(O.dot(O.norm(O.perform_stft(x0, win, hop, n_fft, window=(O.hann(win) / np.float32(n_fft)).astype(np.float32))), fb))
nw = int(np.float32(100.0) * np.float32(n) / np.float32(sr))
out = {}
for fast in (True, False):
    mt = thesia.MultiTrack(freq_scale=thesia.FreqScale.Mel, fast=fast)
    mt.add_tracks_pcm(list(range(k)), pcm, [sr] * k)
    rng = (mt.get_max_db(), mt.get_min_db())
    got = np.frombuffer(mt.get_spec_image(0, 100.0, 300), np.uint8).reshape(300, nw, 3)
    spec = mt.get_spec(0)
    grey = mt.get_grey(0)
    mt.close()
    ogrey = O.spec_to_grey(spec, 1.0, rng[0], rng[1])
    img = np.asarray(O.grey_to_rgb(ogrey, nw, 300)[0], np.uint8)
    d = np.abs(got.astype(int) - img.astype(int)).max(axis=2)
    print(f"fast={fast} range={rng} grey {grey.shape} oracle grey {ogrey.shape} grey equal "
          f"{np.array_equal(grey, ogrey) if grey.shape == ogrey.shape else 'shape'}; "
          f"img diff px {(d > 0).sum()} of {d.size}, max {d.max()}", flush=True)
    bad = np.argwhere(d > 1)
    if bad.size:
        print("  first bad", bad[:8].tolist(), "cols with bad:", np.unique(bad[:, 1])[:10].tolist(),
              "rows:", np.unique(bad[:, 0])[:10].tolist(), flush=True)
        print("  got row0", got[0, :6].tolist(), "want", img[0, :6].tolist(), flush=True)
    dd = np.abs(spec - db)
    print("  spec vs oracle dB max", float(dd.max()), flush=True)
