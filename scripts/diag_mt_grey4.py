"""Debug aid (no image kernels): save MultiTrack greys + specs of a 16 x 30 s mel batch (tracks
7, 8, 9, 15) for offline analysis. Test infrastructure."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))

import fixtures  # noqa: E402
import thesia  # noqa: E402
from thesia import engine  # noqa: E402

sr, secs, k = 48000, 30, 16
n = secs * sr
pcm = [fixtures.s16_to_f32(engine.synth_pcm_host(1, i, n, sr, seed=5)).reshape(-1) for i in range(k)]
mt = thesia.MultiTrack(freq_scale=thesia.FreqScale.Mel, fast=True)
mt.add_tracks_pcm(list(range(k)), pcm, [sr] * k)
out = {"range": np.array([mt.get_max_db(), mt.get_min_db()], np.float32)}
for i in (7, 8, 9, 15):
    out[f"grey{i}"] = mt.get_grey(i)
    out[f"spec{i}"] = mt.get_spec(i)
out["spec0"] = mt.get_spec(0)
mt.close()
np.savez(os.path.join(ROOT, "gpurun_out", "r05_m", "mt.npz"), **out)
print("saved", flush=True)
