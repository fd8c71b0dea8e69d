"""Per-phase cycle shares of stft5_kernel (diagnostic build: make stamps -> lib/libthesia_stamps.so).

Each wave of the stamps build reads s_memtime at the phase marks of its frame loop and sums the
cycles per phase; this script runs the bench's C4 shard once and prints, per phase, the mean
cycles per frame pair (one loop iteration) over all waves and its share. The stamps' own fences
forbid overlaps the product kernel has: read the SHARES, never the run time
(cdna_hip_programming.md §7, In-kernel stamps).

  THESIA_LIB=multi-spectrogram-viewer_amd/lib/libthesia_stamps.so python scripts/stamps.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))
from thesia import engine  # noqa: E402

PHASES = ["load+ring", "window+dft1", "twiddles", "transposes", "prefetch", "dft2",
          "untangle+|X|", "mel+stores"]


def main():
    tracks = int(os.environ.get("STAMP_TRACKS", "1000"))
    kind = {"mel": engine.OUT_MEL_AMP_DB, "complex": engine.OUT_COMPLEX,
            "power_db": engine.OUT_POWER_DB}[os.environ.get("STAMP_KIND", "mel")]
    n, sr, ch = 1_440_000, 48000, 2
    din = engine.DeviceBuffer(tracks * n * ch * 4)
    engine.synth_pcm_device(din, engine.IN_F32, ch, tracks, n, sr, seed=0)
    plan = engine.Plan(2048, 2048, 512, kind, sr=sr, n_mels=128 if kind == engine.OUT_MEL_AMP_DB else 0)
    offs = np.arange(tracks, dtype=np.uint64) * (n * ch)
    T = engine.Batch.frames_for(plan, [n] * tracks)
    dout = engine.DeviceBuffer(T * plan.row_bins * (8 if kind == engine.OUT_COMPLEX else 4))
    b = engine.Batch(plan, din, offs, [n] * tracks, dout, input_format=engine.IN_F32, channels=ch, kernel=5)
    waves = 256 * 8
    sbuf = engine.DeviceBuffer(waves * 9 * 8)
    sbuf.zero()
    b.set_option(100, sbuf.ptr.value)
    b.run()
    engine.synchronize()
    st = sbuf.to_host(np.uint64, (waves, 9)).astype(np.float64)
    used = st[:, 8] > 0
    st = st[used]
    iters = st[:, 8]
    cyc = st[:, :8].copy()
    per = cyc.sum(axis=0) / iters.sum()  # cycles per loop iteration (frame pair per wave)
    tot = per.sum()
    out = {"waves": int(used.sum()), "iters_per_wave": float(iters.mean()),
           "cycles_per_iter": float(tot),
           "phases": {PHASES[i]: {"cycles": float(per[i]), "share": float(per[i] / tot)} for i in range(8)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
