// thesia_napi.cc -- Node-API addon over libthesia's C ABI (include/thesia.h): the surface the
// reference exports to JavaScript through wasm-bindgen (src_rust/lib.rs:72-365, 473-480), so the
// Electron main process (package.json:4,17-27) can load the MI355X engine in place of the wasm
// package. Names and argument meaning follow the wasm-bindgen exports one for one:
//
//   new MultiTrack()                                     lib.rs:89-110
//   mt.add_tracks(id_list, path_list) -> bool            lib.rs:170-191 (throws like Err(JsValue))
//   mt.remove_track(id) -> bool                          lib.rs:265-292
//   mt.get_spec_image(id, px_per_sec, nheight) -> Uint8Array RGB         lib.rs:294-298
//   mt.get_wav_image(id, px_per_sec, nheight, amp_min, amp_max) -> Uint8Array RGBA  lib.rs:300-313
//   mt.get_frequency_hz(id, relative_freq) -> number     lib.rs:315-322
//   mt.get_max_db() / get_min_db() / get_max_sec() / get_sec(id) / get_sr(id) /
//   get_path(id) / get_filename(id)                      lib.rs:324-364
//   mt.free()                                            wasm-bindgen's generated free()
//   get_colormap() -> Uint8Array(30)                     lib.rs:473-480
//
// plus the Rust-level pub items benches/bench.rs uses (not wasm exports): perform_stft
// (lib.rs:388-471), hann (windows.rs:21-30), calc_mel_fb / calc_mel_fb_default (mel.rs:33-99).
//
// Errors: where the reference returns Err or panics (unknown id: unwrap, lib.rs:113,266,295;
// unreadable file: io::Error, lib.rs:176) the addon throws an Error whose message is
// thesia_last_error() and whose `code` is the thesia status. Everything is synchronous, like the
// wasm calls (the engine's own work runs on the GPU; each call returns once its bytes are on the
// host).
#include <node_api.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "thesia.h"

namespace {

#define NAPI_OK(call)                                                      \
    do {                                                                   \
        if ((call) != napi_ok) {                                           \
            throw_napi(env, #call);                                        \
            return nullptr;                                                \
        }                                                                  \
    } while (0)

void throw_napi(napi_env env, const char* what) {
    bool pending = false;
    napi_is_exception_pending(env, &pending);
    if (!pending) napi_throw_error(env, "ERR_NAPI", what);
}

// throws Error(thesia_last_error()) with .code = the status; returns nullptr for the caller
napi_value throw_thesia(napi_env env, int rc) {
    napi_value msg, err, code;
    const char* m = thesia_last_error();
    std::string s = (m && *m) ? m : ("thesia error " + std::to_string(rc));
    if (napi_create_string_utf8(env, s.c_str(), s.size(), &msg) == napi_ok &&
        napi_create_error(env, nullptr, msg, &err) == napi_ok && napi_create_int32(env, rc, &code) == napi_ok) {
        napi_set_named_property(env, err, "code", code);
        napi_throw(env, err);
    } else {
        napi_throw_error(env, nullptr, s.c_str());
    }
    return nullptr;
}

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv, napi_value* self) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, self, nullptr) != napi_ok) return false;
    if (argc < want) {
        napi_throw_type_error(env, "ERR_ARGS", ("expected " + std::to_string(want) + " arguments").c_str());
        return false;
    }
    return true;
}

bool num(napi_env env, napi_value v, double* out) {
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok) return false;
    if (t == napi_number) return napi_get_value_double(env, v, out) == napi_ok;
    if (t == napi_bigint) {
        int64_t x = 0;
        bool lossless = false;
        if (napi_get_value_bigint_int64(env, v, &x, &lossless) != napi_ok) return false;
        *out = (double)x;
        return true;
    }
    napi_throw_type_error(env, "ERR_ARG", "expected a number");
    return false;
}

// wasm-bindgen hands u32 / usize (wasm32: 32-bit) parameters over with ToUint32 (`x >>> 0`):
// NaN and infinities become 0, fractions truncate toward zero, everything wraps mod 2^32
// (get_spec_image(id, 100, 250.7) renders 250 rows, as the reference does)
double to_uint32(double d) {
    if (!(d == d) || d == __builtin_inf() || d == -__builtin_inf()) return 0.0;
    double t = __builtin_trunc(d);
    double m = __builtin_fmod(t, 4294967296.0);
    if (m < 0) m += 4294967296.0;
    return m;
}

// a u32 / usize argument of the reference, coerced like wasm-bindgen (to_uint32); a value above
// `max` after that is refused with a RangeError -- only the lengths that size an allocation have
// a max below 2^32 - 1 (the one divergence from the wasm surface)
bool uint_arg(napi_env env, napi_value v, double max, const char* name, double* out) {
    double d = 0;
    if (!num(env, v, &d)) return false;
    d = to_uint32(d);
    if (!(d <= max)) {
        napi_throw_range_error(env, "ERR_ARG", (std::string(name) + ": at most " +
                                                std::to_string((uint64_t)max) + " accepted").c_str());
        return false;
    }
    *out = d;
    return true;
}
constexpr double kU32Max = 4294967295.0;
constexpr double kLenMax = 268435456.0;  // 2^28 elements: sizes beyond this are refused up front
// the largest image the addon hands to JS (a Uint8Array of at most 2^31 - 1 bytes, node 12's
// typed-array limit): a coerced nheight of ~2^32 (a negative height wraps, as wasm-bindgen's u32
// does) would otherwise size a multi-terabyte host buffer before the library is asked for it
constexpr size_t kImageMax = 2147483647u;
bool image_fits(napi_env env, size_t need) {
    if (need <= kImageMax) return true;
    napi_throw_range_error(env, "ERR_ARG", ("image of " + std::to_string(need) +
                                            " bytes: at most 2147483647 accepted").c_str());
    return false;
}

bool id_arg(napi_env env, napi_value v, uint64_t* id) {
    double d = 0;
    if (!num(env, v, &d)) return false;
    *id = (uint64_t)to_uint32(d);  // usize in the reference (wasm32): ToUint32 as wasm-bindgen
    return true;
}

bool str_arg(napi_env env, napi_value v, std::string* out) {
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, nullptr, 0, &n) != napi_ok) {
        napi_throw_type_error(env, "ERR_ARG", "expected a string");
        return false;
    }
    out->resize(n + 1);
    if (napi_get_value_string_utf8(env, v, &(*out)[0], n + 1, &n) != napi_ok) return false;
    out->resize(n);
    return true;
}

// a Float32Array's data (no copy)
bool f32_arg(napi_env env, napi_value v, const float** data, size_t* len) {
    bool is = false;
    napi_typedarray_type t;
    void* p = nullptr;
    napi_value ab;
    size_t off = 0;
    if (napi_is_typedarray(env, v, &is) != napi_ok || !is ||
        napi_get_typedarray_info(env, v, &t, len, &p, &ab, &off) != napi_ok || t != napi_float32_array) {
        napi_throw_type_error(env, "ERR_ARG", "expected a Float32Array");
        return false;
    }
    *data = static_cast<const float*>(p);
    return true;
}

// id_list: &[usize] (wasm-bindgen: a Uint32Array); also a plain Array or any integer typed array
bool ids_arg(napi_env env, napi_value v, std::vector<uint64_t>* ids) {
    bool is = false;
    if (napi_is_typedarray(env, v, &is) != napi_ok) return false;
    if (is) {
        napi_typedarray_type t;
        size_t n = 0, off = 0;
        void* p = nullptr;
        napi_value ab;
        if (napi_get_typedarray_info(env, v, &t, &n, &p, &ab, &off) != napi_ok) return false;
        ids->resize(n);
        for (size_t i = 0; i < n; ++i) {
            switch (t) {
                case napi_uint32_array: (*ids)[i] = static_cast<const uint32_t*>(p)[i]; break;
                case napi_uint16_array: (*ids)[i] = static_cast<const uint16_t*>(p)[i]; break;
                case napi_uint8_array: (*ids)[i] = static_cast<const uint8_t*>(p)[i]; break;
                case napi_biguint64_array: (*ids)[i] = static_cast<const uint64_t*>(p)[i]; break;
                case napi_int32_array: {
                    const int32_t x = static_cast<const int32_t*>(p)[i];
                    if (x < 0) { napi_throw_range_error(env, "ERR_ARG", "negative id"); return false; }
                    (*ids)[i] = (uint64_t)x;
                    break;
                }
                case napi_float64_array: {
                    const double x = static_cast<const double*>(p)[i];
                    if (!(x >= 0) || x != (double)(uint64_t)x) {
                        napi_throw_range_error(env, "ERR_ARG", "ids must be non-negative integers");
                        return false;
                    }
                    (*ids)[i] = (uint64_t)x;
                    break;
                }
                default:
                    napi_throw_type_error(env, "ERR_ARG", "id_list: an integer typed array or an Array");
                    return false;
            }
        }
        return true;
    }
    bool arr = false;
    if (napi_is_array(env, v, &arr) != napi_ok || !arr) {
        napi_throw_type_error(env, "ERR_ARG", "id_list: an integer typed array or an Array");
        return false;
    }
    uint32_t n = 0;
    if (napi_get_array_length(env, v, &n) != napi_ok) return false;
    ids->resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        napi_value e;
        if (napi_get_element(env, v, i, &e) != napi_ok || !id_arg(env, e, &(*ids)[i])) return false;
    }
    return true;
}

napi_value u8_array(napi_env env, const uint8_t* data, size_t n) {
    void* p = nullptr;
    napi_value ab, ta;
    NAPI_OK(napi_create_arraybuffer(env, n, &p, &ab));
    if (n) std::memcpy(p, data, n);
    NAPI_OK(napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta));
    return ta;
}

napi_value f32_array(napi_env env, const float* data, size_t n) {
    void* p = nullptr;
    napi_value ab, ta;
    NAPI_OK(napi_create_arraybuffer(env, n * 4, &p, &ab));
    if (n) std::memcpy(p, data, n * 4);
    NAPI_OK(napi_create_typedarray(env, napi_float32_array, n, ab, 0, &ta));
    return ta;
}

napi_value js_bool(napi_env env, bool b) {
    napi_value v;
    NAPI_OK(napi_get_boolean(env, b, &v));
    return v;
}

napi_value js_num(napi_env env, double d) {
    napi_value v;
    NAPI_OK(napi_create_double(env, d, &v));
    return v;
}

// ------------------------------------------------------------------------------- MultiTrack
struct Mt {
    thesia_mt* h = nullptr;
};

void mt_finalize(napi_env, void* data, void*) {
    Mt* m = static_cast<Mt*>(data);
    if (m->h) thesia_mt_destroy(m->h);
    delete m;
}

// the wrapped handle of `this`; throws if free() was called
thesia_mt* self_handle(napi_env env, napi_value self) {
    void* p = nullptr;
    if (napi_unwrap(env, self, &p) != napi_ok || !p) {
        napi_throw_type_error(env, "ERR_THIS", "not a MultiTrack");
        return nullptr;
    }
    Mt* m = static_cast<Mt*>(p);
    if (!m->h) napi_throw_error(env, "ERR_FREED", "MultiTrack used after free()");
    return m->h;
}

napi_value MtNew(napi_env env, napi_callback_info info) {
    napi_value self, target;
    size_t argc = 0;
    NAPI_OK(napi_get_cb_info(env, info, &argc, nullptr, &self, nullptr));
    NAPI_OK(napi_get_new_target(env, info, &target));
    if (!target) {
        napi_throw_type_error(env, "ERR_CTOR", "MultiTrack must be called with new");
        return nullptr;
    }
    Mt* m = new Mt();
    const int rc = thesia_mt_create(&m->h);
    if (rc != THESIA_OK) {
        delete m;
        return throw_thesia(env, rc);
    }
    if (napi_wrap(env, self, m, mt_finalize, nullptr, nullptr) != napi_ok) {
        thesia_mt_destroy(m->h);
        delete m;
        throw_napi(env, "napi_wrap");
        return nullptr;
    }
    return self;
}

napi_value MtFree(napi_env env, napi_callback_info info) {
    napi_value self;
    size_t argc = 0;
    NAPI_OK(napi_get_cb_info(env, info, &argc, nullptr, &self, nullptr));
    void* p = nullptr;
    if (napi_unwrap(env, self, &p) == napi_ok && p) {
        Mt* m = static_cast<Mt*>(p);
        if (m->h) thesia_mt_destroy(m->h);
        m->h = nullptr;
    }
    return nullptr;
}

napi_value MtAddTracks(napi_env env, napi_callback_info info) {
    napi_value argv[2], self;
    if (!get_args(env, info, 2, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    std::vector<uint64_t> ids;
    std::string paths;
    if (!h || !ids_arg(env, argv[0], &ids) || !str_arg(env, argv[1], &paths)) return nullptr;
    int changed = 0;
    const int rc = thesia_mt_add_tracks(h, ids.data(), ids.size(), paths.c_str(), &changed);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return js_bool(env, changed != 0);
}

napi_value MtRemoveTrack(napi_env env, napi_callback_info info) {
    napi_value argv[1], self;
    if (!get_args(env, info, 1, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    if (!h || !id_arg(env, argv[0], &id)) return nullptr;
    int changed = 0;
    const int rc = thesia_mt_remove_track(h, id, &changed);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return js_bool(env, changed != 0);
}

napi_value MtGetSpecImage(napi_env env, napi_callback_info info) {
    napi_value argv[3], self;
    if (!get_args(env, info, 3, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    double pps = 0, nh = 0;
    if (!h || !id_arg(env, argv[0], &id) || !num(env, argv[1], &pps) ||
        !uint_arg(env, argv[2], kU32Max, "nheight", &nh))
        return nullptr;
    size_t need = 0;
    int rc = thesia_mt_get_spec_image(h, id, (float)pps, (uint32_t)nh, nullptr, 0, &need);
    if (rc != THESIA_OK && rc != THESIA_ERR_BUFFER_TOO_SMALL) return throw_thesia(env, rc);
    if (!image_fits(env, need)) return nullptr;
    std::vector<uint8_t> buf(need);
    rc = thesia_mt_get_spec_image(h, id, (float)pps, (uint32_t)nh, buf.data(), buf.size(), &need);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return u8_array(env, buf.data(), need);
}

napi_value MtGetWavImage(napi_env env, napi_callback_info info) {
    napi_value argv[5], self;
    if (!get_args(env, info, 5, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    double pps = 0, nh = 0, amin = 0, amax = 0;
    if (!h || !id_arg(env, argv[0], &id) || !num(env, argv[1], &pps) ||
        !uint_arg(env, argv[2], kU32Max, "nheight", &nh) || !num(env, argv[3], &amin) || !num(env, argv[4], &amax))
        return nullptr;
    size_t need = 0;
    int rc = thesia_mt_get_wav_image(h, id, (float)pps, (uint32_t)nh, (float)amin, (float)amax, nullptr, 0, &need);
    if (rc != THESIA_OK && rc != THESIA_ERR_BUFFER_TOO_SMALL) return throw_thesia(env, rc);
    if (!image_fits(env, need)) return nullptr;
    std::vector<uint8_t> buf(need);
    rc = thesia_mt_get_wav_image(h, id, (float)pps, (uint32_t)nh, (float)amin, (float)amax, buf.data(),
                                 buf.size(), &need);
    if (rc != THESIA_OK) return throw_thesia(env, rc);  // THESIA_ERR_PANIC: the reference panics there
    return u8_array(env, buf.data(), need);
}

// set_fast(fast: boolean): not in the wasm-bindgen surface; thesia_mt_set_fast (the streaming
// kernel for the tracks added afterwards, SURVEY §8c's end-to-end contract)
napi_value MtSetFast(napi_env env, napi_callback_info info) {
    napi_value argv[1], self;
    if (!get_args(env, info, 1, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    bool fast = false;
    if (!h) return nullptr;
    if (napi_get_value_bool(env, argv[0], &fast) != napi_ok) {
        napi_throw_type_error(env, "ERR_ARG", "set_fast(fast: boolean)");
        return nullptr;
    }
    const int rc = thesia_mt_set_fast(h, fast ? 1 : 0);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return nullptr;
}

napi_value MtGetFrequencyHz(napi_env env, napi_callback_info info) {
    napi_value argv[2], self;
    if (!get_args(env, info, 2, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    double rel = 0;
    if (!h || !id_arg(env, argv[0], &id) || !num(env, argv[1], &rel)) return nullptr;
    float hz = 0;
    const int rc = thesia_mt_get_frequency_hz(h, id, (float)rel, &hz);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return js_num(env, hz);
}

template <float (*F)(const thesia_mt*)>
napi_value MtGetScalar(napi_env env, napi_callback_info info) {
    napi_value self;
    size_t argc = 0;
    NAPI_OK(napi_get_cb_info(env, info, &argc, nullptr, &self, nullptr));
    thesia_mt* h = self_handle(env, self);
    if (!h) return nullptr;
    return js_num(env, F(h));
}

napi_value MtGetSec(napi_env env, napi_callback_info info) {
    napi_value argv[1], self;
    if (!get_args(env, info, 1, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    if (!h || !id_arg(env, argv[0], &id)) return nullptr;
    float s = 0;
    const int rc = thesia_mt_get_sec(h, id, &s);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return js_num(env, s);
}

napi_value MtGetSr(napi_env env, napi_callback_info info) {
    napi_value argv[1], self;
    if (!get_args(env, info, 1, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    if (!h || !id_arg(env, argv[0], &id)) return nullptr;
    uint32_t sr = 0;
    const int rc = thesia_mt_get_sr(h, id, &sr);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return js_num(env, sr);
}

template <int (*F)(const thesia_mt*, uint64_t, char*, size_t, size_t*)>
napi_value MtGetString(napi_env env, napi_callback_info info) {
    napi_value argv[1], self;
    if (!get_args(env, info, 1, argv, &self)) return nullptr;
    thesia_mt* h = self_handle(env, self);
    uint64_t id = 0;
    if (!h || !id_arg(env, argv[0], &id)) return nullptr;
    size_t need = 0;
    int rc = F(h, id, nullptr, 0, &need);
    if (rc != THESIA_OK && rc != THESIA_ERR_BUFFER_TOO_SMALL) return throw_thesia(env, rc);
    std::vector<char> buf(need + 1, 0);
    rc = F(h, id, buf.data(), buf.size(), &need);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    napi_value s;
    NAPI_OK(napi_create_string_utf8(env, buf.data(), NAPI_AUTO_LENGTH, &s));
    return s;
}

// ------------------------------------------------------------------------------- free functions
napi_value GetColormap(napi_env env, napi_callback_info) {
    uint8_t lut[30];
    thesia_get_colormap(lut);
    return u8_array(env, lut, 30);
}

napi_value Hann(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv, nullptr)) return nullptr;
    double size = 0;
    bool sym = false;
    if (!uint_arg(env, argv[0], kLenMax, "size", &size)) return nullptr;
    if (napi_get_value_bool(env, argv[1], &sym) != napi_ok) {
        throw_napi(env, "hann(size: number, symmetric: boolean)");
        return nullptr;
    }
    std::vector<float> w((size_t)size);
    const int rc = thesia_hann(w.size(), sym ? 1 : 0, w.data());
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return f32_array(env, w.data(), w.size());
}

napi_value mel_result(napi_env env, size_t n_mel, const std::vector<float>& fb) {
    napi_value o, nm, arr;
    NAPI_OK(napi_create_object(env, &o));
    NAPI_OK(napi_create_uint32(env, (uint32_t)n_mel, &nm));
    arr = f32_array(env, fb.data(), fb.size());
    if (!arr) return nullptr;
    NAPI_OK(napi_set_named_property(env, o, "n_mel", nm));
    NAPI_OK(napi_set_named_property(env, o, "fb", arr));  // [n_fft/2+1, n_mel] row-major
    return o;
}

napi_value CalcMelFbDefault(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv, nullptr)) return nullptr;
    double sr = 0, n_fft = 0;
    if (!uint_arg(env, argv[0], kU32Max, "sr", &sr) || !uint_arg(env, argv[1], kLenMax, "n_fft", &n_fft))
        return nullptr;
    size_t n_mel = 0;
    int rc = thesia_calc_mel_fb_default((uint32_t)sr, (size_t)n_fft, &n_mel, nullptr, 0);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    std::vector<float> fb(((size_t)n_fft / 2 + 1) * n_mel);
    rc = thesia_calc_mel_fb_default((uint32_t)sr, (size_t)n_fft, &n_mel, fb.data(), fb.size());
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return mel_result(env, n_mel, fb);
}

// calc_mel_fb(sr, n_fft, n_mel, fmin, fmax (null = None), do_norm)
napi_value CalcMelFb(napi_env env, napi_callback_info info) {
    napi_value argv[6];
    if (!get_args(env, info, 6, argv, nullptr)) return nullptr;
    double sr = 0, n_fft = 0, n_mel = 0, fmin = 0, fmax = -1;
    bool norm = true;
    napi_valuetype t;
    if (!uint_arg(env, argv[0], kU32Max, "sr", &sr) || !uint_arg(env, argv[1], kLenMax, "n_fft", &n_fft) ||
        !uint_arg(env, argv[2], 65536.0, "n_mel", &n_mel) || !num(env, argv[3], &fmin) ||
        napi_typeof(env, argv[4], &t) != napi_ok)
        return nullptr;
    if (t != napi_null && t != napi_undefined && !num(env, argv[4], &fmax)) return nullptr;
    if (napi_get_value_bool(env, argv[5], &norm) != napi_ok) {
        throw_napi(env, "do_norm: boolean");
        return nullptr;
    }
    std::vector<float> fb(((size_t)n_fft / 2 + 1) * (size_t)n_mel);
    const int rc = thesia_calc_mel_fb((uint32_t)sr, (size_t)n_fft, (size_t)n_mel, (float)fmin, (float)fmax,
                                      norm ? 1 : 0, fb.data());
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    return mel_result(env, (size_t)n_mel, fb);
}

// perform_stft(input: Float32Array, win_length, hop_length, n_fft, window?: Float32Array)
//   -> { n_frames, n_bins, data: Float32Array [n_frames][n_bins][re, im] }
napi_value PerformStft(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    size_t argc = 5;
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 4) {
        napi_throw_type_error(env, "ERR_ARGS", "perform_stft(input, win_length, hop_length, n_fft, window?)");
        return nullptr;
    }
    const float* x = nullptr;
    size_t n = 0;
    double win = 0, hop = 0, n_fft = 0;
    if (!f32_arg(env, argv[0], &x, &n) || !uint_arg(env, argv[1], kLenMax, "win_length", &win) ||
        !uint_arg(env, argv[2], kLenMax, "hop_length", &hop) || !uint_arg(env, argv[3], kLenMax, "n_fft", &n_fft))
        return nullptr;
    const float* w = nullptr;
    if (argc > 4) {
        napi_valuetype t;
        NAPI_OK(napi_typeof(env, argv[4], &t));
        if (t != napi_null && t != napi_undefined) {
            size_t wn = 0;
            if (!f32_arg(env, argv[4], &w, &wn)) return nullptr;
            if (wn != (size_t)win) {  // lib.rs:404 assert_eq!
                napi_throw_range_error(env, "ERR_ARG", "window length must equal win_length (lib.rs:404)");
                return nullptr;
            }
        }
    }
    const size_t T = thesia_stft_n_frames(n, (size_t)win, (size_t)hop);
    const size_t F = (size_t)n_fft / 2 + 1;
    std::vector<float> out(T * F * 2 + 2);
    size_t nf = 0;
    const int rc = thesia_perform_stft(x, n, (size_t)win, (size_t)hop, (size_t)n_fft, w, out.data(), T, &nf);
    if (rc != THESIA_OK) return throw_thesia(env, rc);
    napi_value o, vt, vf;
    NAPI_OK(napi_create_object(env, &o));
    NAPI_OK(napi_create_uint32(env, (uint32_t)nf, &vt));
    NAPI_OK(napi_create_uint32(env, (uint32_t)F, &vf));
    napi_value data = f32_array(env, out.data(), nf * F * 2);
    if (!data) return nullptr;
    NAPI_OK(napi_set_named_property(env, o, "n_frames", vt));
    NAPI_OK(napi_set_named_property(env, o, "n_bins", vf));
    NAPI_OK(napi_set_named_property(env, o, "data", data));
    return o;
}

napi_value Version(napi_env env, napi_callback_info) {
    napi_value s;
    NAPI_OK(napi_create_string_utf8(env, thesia_version(), NAPI_AUTO_LENGTH, &s));
    return s;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
    int n = 0;
    if (thesia_device_count(&n) != THESIA_OK) n = 0;  // no GPU: 0, not an exception
    return js_num(env, n);
}

// every callback behind a C++ exception barrier: an exception escaping into node (std::bad_alloc
// from a result vector) would call std::terminate and end the Electron main process
template <napi_value (*F)(napi_env, napi_callback_info)>
napi_value Guarded(napi_env env, napi_callback_info info) {
    try {
        return F(env, info);
    } catch (const std::bad_alloc&) {
        napi_throw_range_error(env, "ERR_NOMEM", "out of host memory");
    } catch (const std::exception& e) {
        napi_throw_error(env, "ERR_NATIVE", e.what());
    } catch (...) {
        napi_throw_error(env, "ERR_NATIVE", "native exception");
    }
    return nullptr;
}

napi_value Init(napi_env env, napi_value exports) {
    napi_property_descriptor mt_methods[] = {
        {"add_tracks", nullptr, Guarded<MtAddTracks>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"remove_track", nullptr, Guarded<MtRemoveTrack>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_spec_image", nullptr, Guarded<MtGetSpecImage>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_wav_image", nullptr, Guarded<MtGetWavImage>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_frequency_hz", nullptr, Guarded<MtGetFrequencyHz>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_max_db", nullptr, Guarded<MtGetScalar<thesia_mt_get_max_db>>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_min_db", nullptr, Guarded<MtGetScalar<thesia_mt_get_min_db>>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_max_sec", nullptr, Guarded<MtGetScalar<thesia_mt_get_max_sec>>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_sec", nullptr, Guarded<MtGetSec>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_sr", nullptr, Guarded<MtGetSr>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_path", nullptr, Guarded<MtGetString<thesia_mt_get_path>>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"get_filename", nullptr, Guarded<MtGetString<thesia_mt_get_filename>>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"set_fast", nullptr, Guarded<MtSetFast>, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"free", nullptr, Guarded<MtFree>, nullptr, nullptr, nullptr, napi_default, nullptr},
    };
    napi_value cls;
    NAPI_OK(napi_define_class(env, "MultiTrack", NAPI_AUTO_LENGTH, Guarded<MtNew>, nullptr,
                              sizeof(mt_methods) / sizeof(mt_methods[0]), mt_methods, &cls));
    // module exports are plain enumerable properties (as a wasm-bindgen package's exports)
    constexpr napi_property_attributes kExport =
        static_cast<napi_property_attributes>(napi_writable | napi_enumerable | napi_configurable);
    napi_property_descriptor fns[] = {
        {"MultiTrack", nullptr, nullptr, nullptr, nullptr, cls, kExport, nullptr},
        {"get_colormap", nullptr, Guarded<GetColormap>, nullptr, nullptr, nullptr, kExport, nullptr},
        {"hann", nullptr, Guarded<Hann>, nullptr, nullptr, nullptr, kExport, nullptr},
        {"calc_mel_fb", nullptr, Guarded<CalcMelFb>, nullptr, nullptr, nullptr, kExport, nullptr},
        {"calc_mel_fb_default", nullptr, Guarded<CalcMelFbDefault>, nullptr, nullptr, nullptr, kExport, nullptr},
        {"perform_stft", nullptr, Guarded<PerformStft>, nullptr, nullptr, nullptr, kExport, nullptr},
        {"version", nullptr, Guarded<Version>, nullptr, nullptr, nullptr, kExport, nullptr},
        {"device_count", nullptr, Guarded<DeviceCount>, nullptr, nullptr, nullptr, kExport, nullptr},
    };
    NAPI_OK(napi_define_properties(env, exports, sizeof(fns) / sizeof(fns[0]), fns));
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
