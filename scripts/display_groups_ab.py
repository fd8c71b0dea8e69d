"""Per display group A/B of the render paths on the C5 geometry: for each (rate, n_fft) pair of
the C5 generator, a pipeline of that group's tracks alone (83-84 tracks x 10 s, 100 px/s x 500
rows), its display time (HIP events, library stream) under each render path, interleaved
rounds. Usage: python scripts/display_groups_ab.py [paths=0,3] [tracks=1000]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))
from thesia import engine, pipeline  # noqa: E402

paths = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,3").split(",")]
total = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
engine.set_device(0)
res = {}
for g in range(12):
    tracks = []
    for i in range(g, total, 12):
        tracks += pipeline.c5_tracks(1, seconds=10.0, first=i)
    p = pipeline.RenderPipeline(tracks, px_per_sec=100.0, nheight=500)
    p._max_sr = 48000  # the C5 step's geometry: every group's up_ratio against the 48 kHz tracks
    p.run_spectrograms()
    times = {q: [] for q in paths}
    for _ in range(4):
        for q in paths:
            engine.set_render_path(q)
            times[q].append(p.display_timed(3)["display_ms"])
    engine.set_render_path(0)
    t = tracks[0]
    key = f"{t.sr}/{t.n_fft}"
    res[key] = {str(q): round(float(np.median(v)) * 1e3, 1) for q, v in times.items()}
    print(json.dumps({key: res[key], "tracks": len(tracks)}), flush=True)
    p.close()
print(json.dumps({"display_us_per_group": res}))
