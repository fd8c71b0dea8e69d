"""Host-side logic of the C5 pipeline (no device): the generator's geometry cycle."""
import numpy as np

from thesia import pipeline


def test_c5_generator_cycles_rates_and_sizes():
    ts = pipeline.c5_tracks(12, seconds=0.05)
    assert [t.sr for t in ts[:6]] == [8000, 16000, 22050, 24000, 44100, 48000]
    assert [t.n_fft for t in ts[:4]] == [256, 512, 1024, 2048]
    assert len({(t.sr, t.n_fft) for t in ts}) == 12
    assert all(t.pcm.dtype == np.int16 and t.pcm.ndim == 1 and len(t.pcm) == round(0.05 * t.sr)
               for t in ts)
    # spectrogram batches are per n_fft / win / hop / layout (amp dB rows do not depend on the
    # rate): the 12 (rate, n_fft) pairs fall into 4 batches of 3 rates each
    assert pipeline._geometry(ts[0]) == (256, 256, 64, 1, 1)
    assert len({pipeline._geometry(t) for t in ts}) == 4
