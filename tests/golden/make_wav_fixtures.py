"""Synthetic WAV fixtures for the ingest path (audio.rs:9-37, hound 3.4 semantics).

Writes tests/golden/wav/*.wav plus wav_expected.npz: per file the interleaved f32 samples that
open_audio_file yields -- integer x -> (x as f32) / (2^(bits-1) as f32) (8-bit WAV stores
unsigned bytes, x = byte - 128), float samples as stored -- and the sample rate / channels.
The expected values are computed here from the integers written, independently of the
library's parser. Run from the repo root: python tests/golden/make_wav_fixtures.py
"""
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "wav")

# (name, sr, channels, kind, bits, container bytes, extensible, extra chunk)
SPECS = [
    ("u8_mono_8k", 8000, 1, "int", 8, 1, False, False),
    ("s16_stereo_16k", 16000, 2, "int", 16, 2, False, True),
    ("s24_mono_22k", 22050, 1, "int", 24, 3, False, False),
    ("s24_stereo_ext_24k", 24000, 2, "int", 24, 3, True, False),
    ("s32_mono_44k", 44100, 1, "int", 32, 4, False, True),
    ("f32_stereo_48k", 48000, 2, "float", 32, 4, False, False),
    ("f32_3ch_ext_32k", 32000, 3, "float", 32, 4, True, False),
    ("s16_6ch_8k", 8000, 6, "int", 16, 2, False, False),
]
SECONDS = 0.3


def _samples(rng, n, ch, kind, bits):
    t = np.arange(n)[:, None] / n
    sig = 0.6 * np.sin(2 * np.pi * (40 + 300 * t) * t * 7 + np.arange(ch)[None, :]) + rng.normal(0, 0.05, (n, ch))
    sig = np.clip(sig, -1.0, 1.0)
    if kind == "float":
        return sig.astype(np.float32)
    full = (1 << (bits - 1)) - 1
    x = np.round(sig * full).astype(np.int64)
    x[0, 0] = -(1 << (bits - 1))  # the most negative code once
    x[1, 0] = full
    return x


def _encode(x, kind, bits, nb):
    if kind == "float":
        return x.astype("<f4").tobytes()
    flat = x.reshape(-1)
    if nb == 1:
        return (flat + 128).astype(np.uint8).tobytes()
    if nb == 2:
        return flat.astype("<i2").tobytes()
    if nb == 3:
        u = (flat & 0xFFFFFF).astype(np.uint32)
        b = np.stack([u & 0xFF, (u >> 8) & 0xFF, (u >> 16) & 0xFF], axis=1).astype(np.uint8)
        return b.tobytes()
    return flat.astype("<i4").tobytes()


def _expected(x, kind, bits):
    if kind == "float":
        return x.reshape(-1).astype(np.float32)
    return (x.reshape(-1).astype(np.float32) / np.float32(2.0 ** (bits - 1))).astype(np.float32)


def _wav_bytes(sr, ch, kind, bits, nb, ext, extra, data):
    tag = 3 if kind == "float" else 1
    block = ch * nb
    if ext:
        sub = (b"\x03\x00\x00\x00" if tag == 3 else b"\x01\x00\x00\x00") + \
            b"\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        fmt = struct.pack("<HHIIHHHHI", 0xFFFE, ch, sr, sr * block, block, nb * 8, 22, bits, 0) + sub
    else:
        fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * block, block, bits)
    chunks = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if extra:  # an odd-length LIST chunk (pad byte) before the data: the parser must skip it
        body = b"INFOISFT\x05\x00\x00\x00test\x00"
        chunks += b"LIST" + struct.pack("<I", len(body)) + body + (b"\x00" if len(body) & 1 else b"")
    chunks += b"data" + struct.pack("<I", len(data)) + data
    return b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks


def main():
    os.makedirs(OUT, exist_ok=True)
    exp = {}
    for k, (name, sr, ch, kind, bits, nb, ext, extra) in enumerate(SPECS):
        rng = np.random.default_rng(100 + k)
        n = int(SECONDS * sr) + 3 * k
        x = _samples(rng, n, ch, kind, bits)
        data = _encode(x, kind, bits, nb)
        with open(os.path.join(OUT, name + ".wav"), "wb") as f:
            f.write(_wav_bytes(sr, ch, kind, bits, nb, ext, extra, data))
        exp[name + "/samples"] = _expected(x, kind, bits)
        exp[name + "/meta"] = np.array([sr, ch, bits], np.int64)
    np.savez_compressed(os.path.join(HERE, "wav_expected.npz"), **exp)
    print("wrote", len(SPECS), "fixtures to", OUT)


if __name__ == "__main__":
    main()
