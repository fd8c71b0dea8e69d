"""Debug aid (no image kernels): MultiTrack mel greys with pageable vs page-locked PCM.
Test infrastructure."""
import ctypes as C
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
from thesia._lib import lib, check  # noqa: E402

sr = 48000


def run(secs, k, pinned, scale=thesia.FreqScale.Mel, rep=0):
    n = secs * sr
    pcm = [fixtures.s16_to_f32(engine.synth_pcm_host(1, i, n, sr, seed=5)).reshape(-1) for i in range(k)]
    if pinned:
        for p in pcm:
            check(lib.thesia_host_register(p.ctypes.data_as(C.c_void_p), p.nbytes))
    mt = thesia.MultiTrack(freq_scale=scale, fast=True)
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
    print(f"secs {secs} tracks {k} pinned {pinned} scale {int(scale)} rep {rep}: bad greys {bad}", flush=True)


for rep in range(2):
    run(30, 16, False, rep=rep)
    run(30, 16, True, rep=rep)
run(30, 16, False, thesia.FreqScale.Linear)
