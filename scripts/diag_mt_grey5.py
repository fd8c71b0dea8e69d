"""Debug aid (no image kernels): MultiTrack mel greys of 16 x 30 s tracks against spec_to_grey of
their own rows (run with THESIA_LIB to compare library builds). Test infrastructure."""
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

sr = 48000
for secs, k in ((30, 16), (250, 4)):
    n = secs * sr
    pcm = [fixtures.s16_to_f32(engine.synth_pcm_host(1, i, n, sr, seed=5)).reshape(-1) for i in range(k)]
    mt = thesia.MultiTrack(freq_scale=thesia.FreqScale.Mel, fast=True)
    mt.add_tracks_pcm(list(range(k)), pcm, [sr] * k)
    r = (mt.get_max_db(), mt.get_min_db())
    bad = []
    for i in range(k):
        g = mt.get_grey(i)
        og = O.spec_to_grey(mt.get_spec(i), 1.0, r[0], r[1])
        nb = int((g != og).any(axis=1).sum())
        if nb:
            bad.append((i, nb))
    mt.close()
    print(f"{os.environ.get('THESIA_LIB', 'product')}: secs {secs} tracks {k}: bad greys {bad}", flush=True)
