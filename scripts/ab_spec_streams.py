"""A/B of the C5 spectrogram phase: one launch per group in sequence (Batch.run) vs the launches
spread over the library's streams (engine.run_batches); HIP events on the library stream,
interleaved rounds. Usage: python scripts/ab_spec_streams.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))
import numpy as np  # noqa: E402
from thesia import engine, pipeline  # noqa: E402

tracks = pipeline.c5_tracks(1000, seconds=10.0)
p = pipeline.RenderPipeline(tracks, px_per_sec=100.0, nheight=500)
bs = [b for _, _, _, b in p.groups]


def seq():
    for b in bs:
        b.run()


def par():
    engine.run_batches(bs)


res = {"sequential": [], "streams": []}
for f in (seq, par):
    f()
engine.synchronize()
for _ in range(7):
    for name, f in (("sequential", seq), ("streams", par)):
        with engine.EventTimer() as tm:
            for _ in range(3):
                f()
        res[name].append(tm.ms / 3)
print(json.dumps({k: {"median_ms": float(np.median(v)), "min_ms": float(min(v))} for k, v in res.items()}))
p.close()
