"""GPU display kernels (display.rs) are bit-exact with the oracle given the same input."""
import numpy as np
import pytest

import oracle_ffi as O
import thesia
from thesia import display

pytestmark = pytest.mark.gpu


def _spec(rng, T, bins):
    s = rng.normal(-60, 25, (T, bins)).astype(np.float32)
    s[: T // 10] = np.float32(-360.0)  # silent frames
    return s


@pytest.mark.parametrize("up_ratio", [1.0, 1.3, 2.0, 1.00137])
def test_spec_to_grey_exact(up_ratio):
    rng = np.random.default_rng(1)
    spec = _spec(rng, 333, 97)
    g = display.spec_to_grey(spec, up_ratio, -3.5, -123.5)
    r = O.spec_to_grey(spec, up_ratio, -3.5, -123.5)
    assert g.shape == r.shape and np.array_equal(g, r)


@pytest.mark.parametrize("shape,new", [((97, 333), (500, 100)), ((347, 4404), (500, 4403)),
                                        ((513, 4404), (500, 4403)), ((40, 50), (50, 40)),
                                        ((64, 64), (64, 64)), ((10, 1000), (7, 3))])
def test_grey_to_rgb_exact(shape, new):
    rng = np.random.default_rng(sum(shape))
    grey = np.clip(rng.random(shape).astype(np.float32) * 1.2 - 0.1, 0, 1).astype(np.float32)
    nh, nw = new
    got = display.grey_to_rgb(grey, nw, nh)
    ref, panics = O.grey_to_rgb(grey, nw, nh)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), int((got != ref).sum())


def test_resize_then_colormap_matches_reference_formula():
    # the colormap alone: a 1-pixel-high identity resize of known greys
    g = np.linspace(0, 1, 101, dtype=np.float32)[None, :]
    got = display.grey_to_rgb(np.repeat(g, 1, 0), 101, 1)
    ref, _ = O.grey_to_rgb(g, 101, 1)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("n,nw,nh,rng_amp", [(44100, 441, 200, (-1.0, 1.0)), (1000, 3000, 50, (-1.5, 1.5)),
                                             (48000 * 3, 300, 500, (-0.5, 0.5)), (777, 100, 64, (-2, 2))])
def test_wav_to_image_exact_and_panics_reported(n, nw, nh, rng_amp):
    rng = np.random.default_rng(n)
    wav = (np.sin(np.arange(n) * 0.01) * 0.4 + rng.normal(0, 0.05, n)).astype(np.float32)
    got, got_panic = display.wav_to_image(wav, nw, nh, rng_amp, return_panic=True)
    ref, panicked = O.wav_to_image(wav, nw, nh, *rng_amp)
    assert got_panic == panicked  # THESIA_ERR_PANIC exactly where the reference panics
    assert np.array_equal(got, ref), int((got != ref).sum())
    if panicked:
        with pytest.raises(thesia.ThesiaError):
            display.wav_to_image(wav, nw, nh, rng_amp)
