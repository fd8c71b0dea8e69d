"""The mel kinds (lib.rs:131-132) of the streaming kernel (stft3_kernel) and the general
kernels against the oracle.

The mel projection is the k-ascending fma chain of the oracle's dot (oracle/thesia_oracle.c
or_dot_f32, lib.rs:131), so for the kernel's own |X| it must match O.dot bit for bit -- for
every filter count (several rounds, the default n_mel) and for custom filterbanks, dense ones
included (thesia_plan_desc.mel_fb)."""
import numpy as np
import pytest

import oracle_ffi as O
from thesia import engine
from thesia._lib import ThesiaError
from tolerances import DB_MAX, DB_P9999, db_clamped_err

pytestmark = pytest.mark.gpu


_LAST = {}


def _run(kind, tracks, channels, fmt, n_mels=0, sr=48000, kernel=3, gap=0, mel_fb=None,
         max_blocks=0, mel_path=0, out_shift=0):
    parts, offs, off = [], [], 0
    for t in tracks:
        offs.append(off)
        parts.append(t.reshape(-1))
        off += t.size + gap
        if gap:
            parts.append(np.zeros(gap, t.dtype))
    flat = np.concatenate(parts)
    lens = [t.shape[0] for t in tracks]
    plan = engine.Plan(2048, 2048, 512, kind, sr=sr, n_mels=n_mels, mel_fb=mel_fb)
    din = engine.DeviceBuffer.from_host(flat)
    T = engine.Batch.frames_for(plan, lens)
    esz = 8 if kind == engine.OUT_COMPLEX else 4
    dout = engine.DeviceBuffer(T * plan.row_bins * esz + out_shift)
    b = engine.Batch(plan, din, offs, lens, dout.ptr.value + out_shift, input_format=fmt, channels=channels,
                     kernel=kernel, max_blocks=max_blocks, mel_path=mel_path)
    if kernel:
        assert b.kernel == kernel
    _LAST["kernel"] = b.kernel
    b.run()
    engine.synchronize()
    dt = np.complex64 if esz == 8 else np.float32
    if out_shift:
        raw = dout.to_host(np.uint8, (T * plan.row_bins * esz + out_shift,))
        out = raw[out_shift:].view(dt).reshape(T, plan.row_bins)
    else:
        out = dout.to_host(dt, (T, plan.row_bins))
    return out, plan


def _tracks(rng, channels, fmt, lens):
    out = []
    for n in lens:
        if fmt == engine.IN_S16:
            out.append(rng.integers(-30000, 30000, size=(n, channels)).astype(np.int16))
        else:
            out.append((rng.standard_normal((n, channels)) * 0.3).astype(np.float32))
    return out


@pytest.mark.parametrize("kernel", [5, 3, 2])
@pytest.mark.parametrize("n_mels,sr", [(128, 48000), (40, 48000), (200, 44100), (0, 48000), (0, 22050)])
@pytest.mark.parametrize("channels", [1, 2])
def test_mel_is_the_dot_of_the_kernels_own_magnitude(kernel, n_mels, sr, channels):
    rng = np.random.default_rng(n_mels * 7 + channels + kernel + sr)
    tracks = _tracks(rng, channels, engine.IN_F32, [2047, 2048 * 5 + 17, 512 * 41 + 3, 30000])
    mag, _ = _run(engine.OUT_MAG, tracks, channels, engine.IN_F32, kernel=kernel, max_blocks=5)
    mel, plan = _run(engine.OUT_MEL, tracks, channels, engine.IN_F32, n_mels=n_mels, sr=sr,
                     kernel=kernel, max_blocks=5)
    fb = O.calc_mel_fb(sr, 2048, n_mels) if n_mels else O.calc_mel_fb_default(sr, 2048)
    assert plan.row_bins == fb.shape[1]
    np.testing.assert_array_equal(mel, O.dot(mag, fb))


@pytest.mark.parametrize("mel_path,out_shift", [(1, 0), (2, 0), (3, 0), (2, 4), (3, 8)])
@pytest.mark.parametrize("n_mels,sr", [(128, 48000), (40, 48000), (80, 16000), (130, 44100), (10, 48000)])
def test_stft5_mel_paths_are_the_same_chain(mel_path, out_shift, n_mels, sr):
    """stft5's mel projections (THESIA_BATCH_OPT_MEL_PATH): the rounds' chunk stream and the
    packed streams with 2 / 3 float4 steps per chunk (filters dealt to lanes by load, mels staged
    behind the |X| row; 16-byte row stores when n_mels % 4 == 0 and the rows are aligned, lane-wise
    stores otherwise -- out_shift misaligns the output) are all the k-ascending fma chain of
    O.dot over the kernel's own |X|, bit for bit; the dB rows follow from the same values."""
    rng = np.random.default_rng(n_mels + 3 * mel_path + out_shift + sr)
    tracks = _tracks(rng, 2, engine.IN_F32, [2048 * 7 + 5, 512 * 33 + 1, 30011])
    mag, _ = _run(engine.OUT_MAG, tracks, 2, engine.IN_F32, kernel=5, max_blocks=3)
    fb = O.calc_mel_fb(sr, 2048, n_mels)
    try:
        mel, plan = _run(engine.OUT_MEL, tracks, 2, engine.IN_F32, n_mels=n_mels, sr=sr, kernel=5,
                         max_blocks=3, mel_path=mel_path, out_shift=out_shift)
    except ThesiaError as e:  # the packed stream does not cover this filterbank
        assert mel_path >= 2 and ("packed" in str(e) or "fit" in str(e)), e
        pytest.skip(str(e))
    np.testing.assert_array_equal(mel, O.dot(mag, fb))
    db, _ = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=n_mels, sr=sr, kernel=5,
                 max_blocks=3, mel_path=mel_path, out_shift=out_shift)
    ref, _ = _run(engine.OUT_MEL_AMP_DB, tracks, 2, engine.IN_F32, n_mels=n_mels, sr=sr, kernel=5,
                  max_blocks=3, mel_path=1)
    np.testing.assert_array_equal(db, ref)


@pytest.mark.parametrize("which", ["dense", "two_wide_bands", "slaney_like"])
def test_custom_filterbank(which):
    """A custom mel_fb (thesia_plan_desc.mel_fb) of any sparsity: dense rows, very wide bands,
    arbitrary weights -- the dot of the kernel's own |X| (the streaming kernel where the weights
    fit its LDS, else the 4-waves/SIMD kernel, which reads them from HBM)."""
    rng = np.random.default_rng(len(which))
    F = 1025
    if which == "dense":
        fb = rng.random((F, 24)).astype(np.float32)
    elif which == "two_wide_bands":
        fb = np.zeros((F, 4), np.float32)
        fb[:700, 0] = 1.0 / 700
        fb[300:, 1] = rng.random(F - 300).astype(np.float32)
        fb[:, 2] = 1e-3
        fb[1000:, 3] = 2.0
    else:
        fb = O.calc_mel_fb(48000, 2048, 96)
        fb = (fb * rng.random(fb.shape)).astype(np.float32)
    tracks = _tracks(rng, 2, engine.IN_F32, [2048 * 9 + 5, 7000])
    mel, plan = _run(engine.OUT_MEL, tracks, 2, engine.IN_F32, mel_fb=fb, max_blocks=4, kernel=0)
    k = _LAST["kernel"]
    mag, _ = _run(engine.OUT_MAG, tracks, 2, engine.IN_F32, max_blocks=4, kernel=k)
    assert plan.row_bins == fb.shape[1]
    np.testing.assert_array_equal(mel, O.dot(mag, fb))


@pytest.mark.parametrize("channels,fmt", [(1, engine.IN_F32), (2, engine.IN_F32), (2, engine.IN_S16),
                                          (1, engine.IN_S16)])
@pytest.mark.parametrize("gap", [0, 1])
def test_mel_db_against_oracle_with_track_edges(channels, fmt, gap):
    """3 blocks at most: long streams, shift + prefetch across track ends (odd gaps break the
    16-byte alignment and force per-frame reloads)."""
    rng = np.random.default_rng(17 + channels + 5 * fmt + gap)
    lens = [2047, 2048, 2049, 6151, 512 * 37, 20483, 512 * 60 + 5]
    tracks = _tracks(rng, channels, fmt, lens)
    got, _ = _run(engine.OUT_MEL_AMP_DB, tracks, channels, fmt, n_mels=128, gap=gap, max_blocks=3)
    fb = O.calc_mel_fb(48000, 2048, 128)
    T0 = 0
    for t in tracks:
        x = t.astype(np.float32) / np.float32(32768.0) if fmt == engine.IN_S16 else t
        acc = np.zeros(x.shape[0], np.float32)
        for c in range(channels):  # lib.rs:42 channel sum
            acc = (acc + x[:, c]).astype(np.float32)
        ref = O.amp_to_db_default(O.dot(O.norm(O.perform_stft(acc, 2048, 512, 2048)), fb))
        g = got[T0:T0 + ref.shape[0]]
        T0 += ref.shape[0]
        mx, p = db_clamped_err(g, ref)
        assert mx <= DB_MAX and p <= DB_P9999, (t.shape, mx, p)


def test_kernel_choice_and_unsupported_force():
    """The streaming kernel by default for its geometry; forcing a kernel that cannot run the
    geometry is an error, not a silent fallback."""
    x = np.zeros((4096, 2), np.float32)
    _run(engine.OUT_MEL_AMP_DB, [x], 2, engine.IN_F32, n_mels=128, kernel=5)
    _run(engine.OUT_MEL_AMP_DB, [x], 2, engine.IN_F32, n_mels=128, kernel=3)
    plan = engine.Plan(2048, 1920, 480, engine.OUT_AMP_DB)  # the 48 kHz viewer geometry streams
    din = engine.DeviceBuffer.from_host(x[:, 0].copy())
    dout = engine.DeviceBuffer(engine.Batch.frames_for(plan, [4096]) * plan.row_bins * 4)
    b = engine.Batch(plan, din, [0], [4096], dout)
    assert b.kernel == 3  # a small batch: stft3 (stft5's viewer rule from 400 000 frames on)
    b.set_option(engine.OPT_KERNEL, 5)  # stft5's viewer column rule (HQ 7) runs it when forced
    import thesia
    plan = engine.Plan(2048, 1920, 480, engine.OUT_COMPLEX)  # complex rows: stft3 only
    dout = engine.DeviceBuffer(engine.Batch.frames_for(plan, [4096]) * plan.row_bins * 8)
    b = engine.Batch(plan, din, [0], [4096], dout)
    assert b.kernel == 3
    with pytest.raises(thesia.ThesiaError):
        b.set_option(engine.OPT_KERNEL, 5)
    plan = engine.Plan(2048, 1764, 441, engine.OUT_AMP_DB)  # 44.1 kHz viewer geometry: odd hop,
    x16 = np.zeros(4096, np.int16)                          # s16 mono (2-byte-aligned loads) streams
    din = engine.DeviceBuffer.from_host(x16)
    dout = engine.DeviceBuffer(engine.Batch.frames_for(plan, [4096]) * plan.row_bins * 4)
    b = engine.Batch(plan, din, [0], [4096], dout, input_format=engine.IN_S16)
    assert b.kernel == 3
    with pytest.raises(thesia.ThesiaError):
        b.set_option(engine.OPT_KERNEL, 5)
    plan = engine.Plan(2048, 1763, 441, engine.OUT_AMP_DB)  # odd win: no streaming start rule
    dout = engine.DeviceBuffer(engine.Batch.frames_for(plan, [4096]) * plan.row_bins * 4)
    b = engine.Batch(plan, din, [0], [4096], dout, input_format=engine.IN_S16)
    assert b.kernel == 2
    with pytest.raises(thesia.ThesiaError):
        b.set_option(engine.OPT_KERNEL, 3)
    with pytest.raises(thesia.ThesiaError):
        b.set_option(engine.OPT_KERNEL, 5)


_VARIANT_CHILD = r"""
import sys, hashlib
import numpy as np
sys.path.insert(0, sys.argv[1])
from thesia import engine
rng = np.random.default_rng(5)
x = (rng.standard_normal((48000, 2)) * 0.3).astype(np.float32)
plan = engine.Plan(2048, 2048, 512, engine.OUT_MEL_AMP_DB, sr=48000, n_mels=128)
din = engine.DeviceBuffer.from_host(x)
T = engine.Batch.frames_for(plan, [48000])
dout = engine.DeviceBuffer(T * 128 * 4)
b = engine.Batch(plan, din, [0], [48000], dout, channels=2, kernel=3)  # the experiments' kernel
b.run()
engine.synchronize()
print(hashlib.sha256(dout.to_host(np.uint8).tobytes()).hexdigest(), b.kernel)
"""


def test_variant_env_cannot_change_product_output():
    """THESIA_STFT_VARIANT=4 (the no-FFT ablation in the experiment build) changes nothing in
    the product library: same bytes as without it."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "multi-spectrogram-viewer_amd")
    outs = []
    for v in (None, "4", "2"):
        env = dict(os.environ)
        env.pop("THESIA_LIB", None)
        if v:
            env["THESIA_STFT_VARIANT"] = v
        r = subprocess.run([sys.executable, "-c", _VARIANT_CHILD, pkg], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.split())
    assert outs[0][1] == "3"
    assert outs[0] == outs[1] == outs[2], outs
