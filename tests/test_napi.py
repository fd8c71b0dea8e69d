"""The Node-API addon (bindings/napi/thesia_napi.cc): the wasm-bindgen surface of lib.rs:72-365,
473-480 as a native module for the Electron main process. Host-only entries run here (no GPU):
the exports and the MultiTrack method names equal the wasm-bindgen ones, get_colormap equals
display.rs:10-21, hann / calc_mel_fb / calc_mel_fb_default equal the oracle bit for bit, and
reference errors / panics surface as JS exceptions carrying thesia_last_error() and the status.
The GPU half (add_tracks -> get_spec_image from JavaScript) is tests/test_gpu_napi.py."""
import base64

import numpy as np
import pytest

import oracle_ffi as O
from napi_util import node_bin, run_node

pytestmark = pytest.mark.skipif(node_bin() is None, reason="node is not installed")

WASM_METHODS = ["add_tracks", "remove_track", "get_spec_image", "get_wav_image", "get_frequency_hz",
                "get_max_db", "get_min_db", "get_max_sec", "get_sec", "get_sr", "get_path",
                "get_filename", "free"]


def _f32(b64):
    return np.frombuffer(base64.b64decode(b64), np.float32)


JS_F32 = "const f32 = a => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString('base64');\n"


def test_exports_and_names():
    r = run_node("console.log(JSON.stringify({keys: Object.keys(t), "
                 "methods: Object.getOwnPropertyNames(t.MultiTrack.prototype)}));")
    assert {"MultiTrack", "get_colormap", "perform_stft", "hann", "calc_mel_fb",
            "calc_mel_fb_default"} <= set(r["keys"])
    assert set(WASM_METHODS) <= set(r["methods"])


def test_colormap_is_display_rs_lut():
    r = run_node("console.log(JSON.stringify({c: Array.from(t.get_colormap())}));")
    assert bytes(r["c"]) == bytes(O.COLORMAP.ravel())  # display.rs:10-21, 30 bytes


@pytest.mark.parametrize("size,sym", [(4, False), (1920, False), (2048, False), (7, True)])
def test_hann_equals_oracle(size, sym):
    r = run_node(JS_F32 + f"console.log(JSON.stringify({{w: f32(t.hann({size}, {str(sym).lower()}))}}));")
    assert np.array_equal(_f32(r["w"]).view(np.uint32), O.hann(size, sym).view(np.uint32))


@pytest.mark.parametrize("sr,n_fft", [(8000, 512), (22050, 1024), (44100, 2048), (48000, 2048)])
def test_mel_fb_default_equals_oracle(sr, n_fft):
    r = run_node(JS_F32 + f"const m = t.calc_mel_fb_default({sr}, {n_fft});"
                 "console.log(JSON.stringify({n: m.n_mel, fb: f32(m.fb)}));")
    ref = O.calc_mel_fb_default(sr, n_fft)
    assert r["n"] == ref.shape[1]
    assert np.array_equal(_f32(r["fb"]).view(np.uint32), ref.reshape(-1).view(np.uint32))


def test_mel_fb_equals_oracle():
    r = run_node(JS_F32 + "const m = t.calc_mel_fb(48000, 2048, 128, 0, null, true);"
                 "console.log(JSON.stringify({n: m.n_mel, fb: f32(m.fb)}));")
    ref = O.calc_mel_fb(48000, 2048, 128)
    assert np.array_equal(_f32(r["fb"]).view(np.uint32), ref.reshape(-1).view(np.uint32))


def test_errors_are_js_exceptions():
    """Reference Err / panics -> thrown Error {message: thesia_last_error(), code: status}."""
    r = run_node("""
const out = {};
const grab = (k, f) => { try { f(); out[k] = null; } catch (e) { out[k] = [e.code, e.message]; } };
grab('hann1', () => t.hann(1, false));                       // windows.rs:8 assert
const mt = new t.MultiTrack();                               // lib.rs:89 (no device work yet)
grab('unknown', () => mt.get_sr(99));                        // lib.rs:341 unwrap on a missing id
grab('remove', () => mt.remove_track(7));                    // lib.rs:266
grab('io', () => mt.add_tracks([5], '/nonexistent/x.wav'));  // lib.rs:176 Err(io::Error)
grab('badids', () => mt.add_tracks('x', 'a.wav'));
out.empty = [mt.get_max_sec()];
mt.free();
grab('freed', () => mt.get_max_db());
grab('ctor', () => t.MultiTrack());
console.log(JSON.stringify(out));
""")
    assert r["hann1"][0] == -1
    assert r["unknown"][0] == -3 and r["remove"][0] == -3
    assert r["io"][0] == -2 and "No such file" in r["io"][1]
    assert r["badids"] is not None and r["freed"][0] == "ERR_FREED" and r["ctor"] is not None
    assert r["empty"] == [0]


def test_numeric_arguments_coerce_like_wasm_bindgen():
    """u32 / usize arguments (wasm32) reach the reference through wasm-bindgen's ToUint32 (`x >>> 0`):
    fractions truncate, NaN is 0, negatives wrap. The addon coerces the same way, and
    refuses with a RangeError only a length that would size an allocation beyond 2^28 elements
    after the coercion; the process survives every call."""
    r = run_node(JS_F32 + """
const out = {};
const grab = (k, f) => { try { out[k] = ['ok', f()]; } catch (e) { out[k] = [e.constructor.name, e.code]; } };
grab('hann_frac', () => f32(t.hann(4.5, false)));
grab('hann_nan', () => t.hann(NaN, false));          // size 0: windows.rs:8's assert
grab('hann_neg', () => t.hann(-4, false));           // 2^32 - 4 elements: refused
grab('stft_win', () => t.perform_stft(new Float32Array(16), -1, 4, 8));
grab('mel_frac', () => f32(t.calc_mel_fb(48000.9, 2048.2, 40.7, 0, null, true).fb));
const mt = new t.MultiTrack();
grab('nheight', () => mt.get_spec_image(0, 100, -5)); // unknown id: lib.rs:295 unwrap
out.alive = t.hann(4, false).length;
console.log(JSON.stringify(out));
""")
    assert r["hann_frac"][0] == "ok"
    assert np.array_equal(_f32(r["hann_frac"][1]).view(np.uint32), O.hann(4, False).view(np.uint32))
    assert r["hann_nan"] == ["Error", -1], r["hann_nan"]
    assert r["hann_neg"] == ["RangeError", "ERR_ARG"] and r["stft_win"] == ["RangeError", "ERR_ARG"]
    ref = O.calc_mel_fb(48000, 2048, 40)
    assert np.array_equal(_f32(r["mel_frac"][1]).view(np.uint32), ref.reshape(-1).view(np.uint32))
    assert r["nheight"][0] == "Error" and r["nheight"][1] == -3
    assert r["alive"] == 4
