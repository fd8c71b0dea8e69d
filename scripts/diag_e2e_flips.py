"""Which pixels of the MultiTrack e2e contract flip, and why (VERDICT r04 "Next round" item 1).

GPU leg (`--dump OUT.npz`): the six sample excerpts of test_e2e_rgb_multitrack_samples (linear
and mel scale), each track run alone through a Batch at the viewer geometry with the kernel
forced (3 = stft3, 5 = stft5 where it supports the geometry, 9 = stftx, the reference-order
kernel), rows OUT_AMP_DB and OUT_MAG (mel: OUT_MEL_AMP_DB and OUT_MEL). Saved to an npz.

CPU leg (`--analyze OUT.npz`): the oracle pipeline (dB, global range, grey, Lanczos3, colormap)
run on (a) the oracle's dB, (b) each kernel's dB rows, (c) the reference dB chain
(`amp_to_db_default`, decibel.rs:68-76) applied to each kernel's own |X| rows; pixel flips per
track against (a), and the dB error statistics behind them.
Test infrastructure (imports the oracle as the checker).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))

import fixtures  # noqa: E402

TAGS = ["8k", "16k", "22k05", "24k", "44k1"]


def excerpts():
    z = np.load(fixtures.GOLDEN + "/samples_excerpt.npz")
    pcm = [fixtures.s16_to_f32(z[f"pcm_{t}"]) for t in TAGS] + [
        fixtures.s16_to_f32(fixtures.c1_substitute()[:72000])]
    srs = [int(z[f"sr_{t}"]) for t in TAGS] + [48000]
    return pcm, srs


def dump(path):
    from thesia import engine
    import oracle_ffi as O
    pcm, srs = excerpts()
    out = {}
    for mel in (False, True):
        for i, (x, sr) in enumerate(zip(pcm, srs)):
            win, hop, n_fft = O.track_params(sr)
            x = (np.float32(0.0) + x).astype(np.float32)
            din = engine.DeviceBuffer.from_host(x)
            kinds = (engine.OUT_MEL_AMP_DB, engine.OUT_MEL) if mel else (engine.OUT_AMP_DB, engine.OUT_MAG)
            for kind in kinds:
                fb = O.calc_mel_fb_default(sr, n_fft) if mel else None
                plan = engine.Plan(n_fft, win, hop, kind, sr=sr, mel_fb=fb)
                T = engine.Batch.frames_for(plan, [x.size])
                for k in (3, 5, 9):
                    dout = engine.DeviceBuffer(T * plan.row_bins * 4)
                    try:
                        b = engine.Batch(plan, din, [0], [x.size], dout, kernel=k)
                    except Exception as e:  # noqa: BLE001 (kernel does not cover the geometry)
                        print(f"track {i} sr {sr} kernel {k}: {e}")
                        continue
                    if b.kernel != k:
                        continue
                    b.run()
                    engine.synchronize()
                    out[f"{'mel' if mel else 'lin'}_{kind}_{i}_k{k}"] = dout.to_host(np.float32, (T, plan.row_bins))
                    b.close()
                    dout.close()
                plan.close()
            din.close()
    np.savez_compressed(path, **out)
    print("saved", path, len(out))


def analyze(path):
    import oracle_ffi as O
    from thesia import shard
    z = np.load(path)
    pcm, srs = excerpts()
    for mel in (False, True):
        tag = "mel" if mel else "lin"
        kdb = 6 if mel else 3
        kmag = 5 if mel else 1
        mags, dbs = [], []
        for x, sr in zip(pcm, srs):
            win, hop, n_fft = O.track_params(sr)
            w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
            mag = O.norm(O.perform_stft((np.float32(0.0) + x).astype(np.float32), win, hop, n_fft, window=w))
            if mel:
                mag = O.dot(mag, O.calc_mel_fb_default(sr, n_fft))
            mags.append(mag)
            dbs.append(O.amp_to_db_default(mag))

        def pipeline(dbl):
            gmax = float(np.float32(min(max(float(d.max()) for d in dbl), 0.0)))
            gmin = float(np.float32(max(min(float(d.min()) for d in dbl), gmax - 120.0)))
            imgs, greys = [], []
            for x, sr, db in zip(pcm, srs, dbl):
                up = shard.up_ratio(sr, max(srs), freq_scale_mel=mel)
                grey = O.spec_to_grey(db, up, gmax, gmin)
                nwidth = int(np.float32(100.0) * np.float32(len(x)) / np.float32(sr))
                img, _ = O.grey_to_rgb(grey, nwidth, 300)
                imgs.append(np.asarray(img, np.uint8))
                greys.append(grey)
            return imgs, greys, (gmax, gmin)

        ref_imgs, ref_greys, ref_rng = pipeline(dbs)
        print(f"== {tag}: oracle range {ref_rng}")
        variants = {}
        for k in (3, 5, 9):
            have = all(f"{tag}_{kdb}_{i}_k{k}" in z for i in range(6))
            # kernels that do not cover a track fall back to stft3's rows for it
            def rows(kind, i):
                key = f"{tag}_{kind}_{i}_k{k}"
                return z[key] if key in z else z[f"{tag}_{kind}_{i}_k3"]
            variants[f"k{k} dB rows{'' if have else ' (k3 where unsupported)'}"] = [rows(kdb, i) for i in range(6)]
            variants[f"k{k} |X| -> ref dB chain"] = [O.amp_to_db_default(rows(kmag, i)) for i in range(6)]
        # the float64 spectrum (tolerances.stft_f64) through the same display: what both the
        # oracle and the kernels approximate
        from tolerances import stft_f64
        db64 = []
        for x, sr in zip(pcm, srs):
            win, hop, n_fft = O.track_params(sr)
            w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
            m64 = np.abs(stft_f64((np.float32(0.0) + x).astype(np.float32), win, hop, n_fft, w))
            if mel:
                m64 = m64 @ O.calc_mel_fb_default(sr, n_fft).astype(np.float64)
            db64.append((20.0 * np.log10(np.maximum(m64, 1e-18))).astype(np.float32))
        f64_imgs, _, _ = pipeline(db64)

        def flips(a, b):
            return [int((np.abs(a[i].reshape(-1, 3).astype(int) - b[i].reshape(-1, 3).astype(int)).max(1) > 0).sum())
                    for i in range(6)]
        per = flips(ref_imgs, f64_imgs)
        print(f"  oracle vs the f64 pipeline: flips/track {per} total {sum(per)}")
        for name, dbl in variants.items():
            imgs, greys, rng = pipeline(dbl)
            per = flips(imgs, ref_imgs)
            p64 = flips(imgs, f64_imgs)
            print(f"  {name:36s} vs f64 pipeline: flips/track {p64} total {sum(p64)}")
            derr = [float(np.abs(dbl[i] - dbs[i]).max()) for i in range(6)]
            gerr = [float(np.abs(greys[i] - ref_greys[i]).max()) for i in range(6)]
            print(f"  {name:36s} flips/track {per} total {sum(per)}; max|ddB| "
                  f"{['%.2e' % e for e in derr]}; max|dgrey| {['%.1e' % e for e in gerr]}; range {rng}")
        # where the kernel's dB differ: relative to the frame's max
        for k in (3, 5):
            i = 5
            key = f"{tag}_{kmag}_{i}_k{k}"
            if key not in z:
                continue
            m = z[key]
            ref = mags[i]
            rel = np.abs(m - ref) / np.maximum(ref.max(axis=1, keepdims=True), 1e-30)
            print(f"  k{k} 48k |X| err / frame max: max {rel.max():.2e} p99 {np.quantile(rel, 0.99):.2e}")
            dd = np.abs(z[f"{tag}_{kdb}_{i}_k{k}"] - O.amp_to_db_default(m))
            print(f"  k{k} 48k dB rows vs ref chain on own |X|: max {dd.max():.2e} mean {dd.mean():.2e}")
            dx = np.abs(O.amp_to_db_default(m) - dbs[i])
            print(f"  k{k} 48k ref chain on own |X| vs oracle dB: max {dx.max():.2e} mean {dx.mean():.2e}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump")
    ap.add_argument("--analyze")
    a = ap.parse_args()
    if a.dump:
        dump(a.dump)
    if a.analyze:
        analyze(a.analyze)
