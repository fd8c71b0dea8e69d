"""Debug aid (no image kernels): MultiTrack's fast path on a 400 000-frame 48 kHz mel batch --
every track's dB rows against the batch engine's stft5 rows of the same PCM, and the grey images
against the oracle's spec_to_grey of the MultiTrack's own rows and range. Saves track 0's grey.
Test infrastructure."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))

import fixtures  # noqa: E402
import oracle_ffi as O  # noqa: E402
import thesia  # noqa: E402
from thesia import engine  # noqa: E402

sr, secs, k = 48000, 250, 16
n = secs * sr
pcm = [fixtures.s16_to_f32(engine.synth_pcm_host(1, i, n, sr, seed=5)).reshape(-1) for i in range(k)]
win, hop, n_fft = O.track_params(sr)
mt = thesia.MultiTrack(freq_scale=thesia.FreqScale.Mel, fast=True)
mt.add_tracks_pcm(list(range(k)), pcm, [sr] * k)
rng = (mt.get_max_db(), mt.get_min_db())
print("range", rng, flush=True)
flat = np.concatenate(pcm)
din = engine.DeviceBuffer.from_host(flat)
plan = engine.Plan(n_fft, win, hop, engine.OUT_MEL_AMP_DB, sr=sr)
T = engine.Batch.frames_for(plan, [n] * k)
dout = engine.DeviceBuffer(T * plan.row_bins * 4)
b = engine.Batch(plan, din, np.arange(k) * n, [n] * k, dout, kernel=5)
b.run()
engine.synchronize()
rows = dout.to_host(np.float32, (T, plan.row_bins))
for i in range(k):
    s = mt.get_spec(i)
    ref = rows[int(b.frame0[i]):int(b.frame0[i + 1])]
    g = mt.get_grey(i)
    og = O.spec_to_grey(s, 1.0, rng[0], rng[1])
    print(f"track {i}: spec {s.shape} vs batch equal {np.array_equal(s, ref)} maxdiff "
          f"{float(np.abs(s - ref).max()):.3g}; grey {g.shape} oracle {og.shape} equal "
          f"{g.shape == og.shape and np.array_equal(g, og)} finite {np.isfinite(g).all()}", flush=True)
    if i == 0:
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", "r05_f", "grey0.npz"), grey=g, spec=s[:2000])
mt.close()
