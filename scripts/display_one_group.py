"""One C5 display group alone (for counters): the tracks of generator slot `g` (83-84 x 10 s,
100 px/s x 500 rows), `reps` display passes under render path `path`. Usage:
  python scripts/display_one_group.py g path reps"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))
from thesia import engine, pipeline  # noqa: E402

g, path, reps = (int(v) for v in sys.argv[1:4])
engine.set_device(0)
tracks = []
for i in range(g, 1000, 12):
    tracks += pipeline.c5_tracks(1, seconds=10.0, first=i)
p = pipeline.RenderPipeline(tracks, px_per_sec=100.0, nheight=500)
p._max_sr = 48000  # the C5 step's geometry: up_ratio against the 48 kHz tracks
p.run_spectrograms()
engine.set_render_path(path)
t = p.display_timed(reps)
print(tracks[0].sr, tracks[0].n_fft, len(tracks), "display_ms", t["display_ms"])
p.close()
