"""thesia -- MI355X-native spectrogram engine (host-side mirror of the reference API).

Mirrors the reference crate `thesia` (src_rust/lib.rs and its modules): the same names,
argument meanings and error behaviour, over the C ABI of libthesia.so (include/thesia.h).
Everything numeric runs in HIP kernels on the GPU; there is no CPU fallback.

    MultiTrack        lib.rs:72-365   (wasm-bindgen class of the viewer)
    open_audio_file   audio.rs:9-37   (WAV, hound semantics)
    perform_stft      lib.rs:388-471
    get_colormap      lib.rs:473-480
    windows.hann      windows.rs:21-30
    mel.*             mel.rs:13-99
    utils.*           utils.rs:17-19
    display.*         display.rs:10-115
    realfft.InvRealFFT realfft.rs:167-241
    engine.*          the batched device engine (plans / batches resident in HBM)
"""
from ._lib import ThesiaError, EXPORTED, LIB_PATH  # noqa: F401  (import fails loudly if .so missing)
from . import windows, mel, utils, display, engine, shard, pipeline, realfft  # noqa: F401
from .api import MultiTrack, FreqScale, perform_stft, get_colormap, open_audio_file  # noqa: F401

__all__ = ["MultiTrack", "FreqScale", "perform_stft", "get_colormap", "open_audio_file", "windows", "mel", "utils",
           "display", "engine", "realfft", "ThesiaError"]
