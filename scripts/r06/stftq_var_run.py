"""One kernel-7 run per n_fft at the C5 batch size (250 x 10 s mono s16 at 44.1 kHz, amp dB,
the range option on: the RG instances) for rocprofv3 --pmc passes; the experiment variant comes
from THESIA_STFT_VARIANT (THESIA_LIB=multi-spectrogram-viewer_amd/lib/libthesia_exp.so)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))
from thesia import engine  # noqa: E402

sr, ntr, n = 44100, 250, 441000
din = engine.DeviceBuffer(ntr * n * 2)
engine.synth_pcm_device(din, engine.IN_S16, 1, ntr, n, sr, seed=6)
drange = engine.DeviceBuffer(12 * ntr)
for nf in (256, 512, 1024):
    plan = engine.Plan(nf, nf, nf // 4, engine.OUT_AMP_DB, sr=sr)
    T = engine.Batch.frames_for(plan, [n] * ntr)
    dout = engine.DeviceBuffer(T * plan.row_bins * 4)
    b = engine.Batch(plan, din, [i * n for i in range(ntr)], [n] * ntr, dout, input_format=engine.IN_S16, kernel=7)
    b.set_option(engine.OPT_RANGE, drange.ptr.value)
    ms = b.run_timed(3) / 3
    print(nf, os.environ.get("THESIA_STFT_VARIANT", "0"), "ms %.4f" % ms, flush=True)
    b.close()
    dout.close()
    plan.close()
