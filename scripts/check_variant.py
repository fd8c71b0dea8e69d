"""Parity of an experiment variant of the streaming kernel (THESIA_LIB=lib/libthesia_exp.so,
THESIA_STFT_VARIANT): the C4 geometry (48 kHz stereo f32, n_fft 2048 / hop 512) for every output
kind the variant covers, against variant 0 and against the oracle on one track. Usage:
  THESIA_LIB=.../libthesia_exp.so python scripts/check_variant.py VARIANT"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-spectrogram-viewer_amd"), os.path.join(ROOT, "tests")]
from thesia import engine  # noqa: E402
import oracle_ffi as O  # noqa: E402
from tolerances import DB_MAX, DB_P9999, STFT_REL, db_clamped_err, stft_frame_err  # noqa: E402

var = sys.argv[1]
n, ntr = 48000 * 4 + 333, 6
pcm = [engine.synth_pcm_host(2, i, n, 48000) for i in range(ntr)]
x = np.stack([p.astype(np.float32) / np.float32(32768.0) for p in pcm])  # [ntr, n, 2]
ok = True
for kind, nm in ((engine.OUT_MEL_AMP_DB, 128), (engine.OUT_AMP_DB, 0), (engine.OUT_POWER_DB, 0), (engine.OUT_COMPLEX, 0)):
    plan = engine.Plan(2048, 2048, 512, kind, sr=48000, n_mels=nm)
    din = engine.DeviceBuffer.from_host(x)
    T = engine.Batch.frames_for(plan, [n] * ntr)
    isz = 8 if kind == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(T * plan.row_bins * isz)
    b = engine.Batch(plan, din, np.arange(ntr) * n * 2, [n] * ntr, dout, channels=2)
    b.set_option(engine.OPT_KERNEL, 5)
    outs = {}
    for v in ("0", var):
        os.environ["THESIA_STFT_VARIANT"] = v
        b.run()
        engine.synchronize()
        outs[v] = dout.to_host(np.complex64 if isz == 8 else np.float32, (T, plan.row_bins))
    os.environ["THESIA_STFT_VARIANT"] = "0"
    xm = (x[0, :, 0] + x[0, :, 1]).astype(np.float32)
    spec = O.perform_stft(xm, 2048, 512, 2048)
    T0 = spec.shape[0]
    if kind == engine.OUT_COMPLEX:
        e = stft_frame_err(outs[var][:T0], spec)
        e0 = stft_frame_err(outs["0"][:T0], spec)
        good = e <= STFT_REL
        print(f"kind {kind}: variant {var} stft rel err {e:.2e} (variant 0 {e0:.2e})", "ok" if good else "FAIL")
    else:
        if kind == engine.OUT_MEL_AMP_DB:
            ref = O.amp_to_db_default(O.dot(O.norm(spec), O.calc_mel_fb(48000, 2048, 128)))
        elif kind == engine.OUT_AMP_DB:
            ref = O.amp_to_db_default(O.norm(spec))
        else:
            ref = O.power_to_db_default(O.norm_sqr(spec))
        mx, p = db_clamped_err(outs[var][:T0], ref)
        mx0, _ = db_clamped_err(outs["0"][:T0], ref)
        dv = float(np.abs(outs[var] - outs["0"]).max())
        good = mx <= DB_MAX and p <= DB_P9999
        print(f"kind {kind}: variant {var} dB err {mx:.4f} p99.99 {p:.4f} (variant 0 {mx0:.4f}); max |v - v0| {dv:.3e}",
              "ok" if good else "FAIL")
    ok = ok and good and np.isfinite(outs[var].view(np.float32)).all()
    b.close(); dout.close(); din.close(); plan.close()
print("variant parity", "OK" if ok else "FAILED")
sys.exit(0 if ok else 1)
