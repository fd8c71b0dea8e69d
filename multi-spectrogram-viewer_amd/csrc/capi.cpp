// capi.cpp -- extern "C" entry points of libthesia (include/thesia.h). Every function
// catches C++ exceptions and maps failures to status codes; nothing aborts across FFI.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/thesia.h"
#include "engine.hpp"
#include "host_tables.hpp"
#include "multitrack.hpp"
#include "wav.hpp"

using namespace thesia;

// The opaque handle types of thesia.h are never defined: handles are the C++ objects
// themselves, reinterpret_cast at the boundary.

#define GUARD_BEGIN try {
#define GUARD_END                                                                       \
    }                                                                                   \
    catch (const std::bad_alloc&) {                                                     \
        return set_error(THESIA_ERR_DEVICE, "host out of memory");                      \
    }                                                                                   \
    catch (const std::exception& e) {                                                   \
        return set_error(THESIA_ERR_INVALID_ARG, e.what());                             \
    }                                                                                   \
    catch (...) {                                                                       \
        return set_error(THESIA_ERR_INVALID_ARG, "unknown error");                      \
    }

static int copy_out(const void* src, size_t bytes, void* out, size_t cap, size_t* needed) {
    if (needed) *needed = bytes;
    if (!out || cap < bytes)
        return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "output buffer too small");
    if (bytes) std::memcpy(out, src, bytes);
    return THESIA_OK;
}

extern "C" {

const char* thesia_last_error(void) { return last_error(); }
const char* thesia_version(void) { return "thesia-hip 0.1.0 (gfx950)"; }

// ---------------------------------------------------------------- runtime
int thesia_device_count(int* n) {
    THESIA_HIP(hipGetDeviceCount(n));
    return THESIA_OK;
}
int thesia_set_device(int device) {
    THESIA_HIP(hipSetDevice(device));
    return THESIA_OK;
}
int thesia_get_device(int* device) {
    THESIA_HIP(hipGetDevice(device));
    return THESIA_OK;
}
int thesia_device_malloc(void** ptr, size_t bytes) {
    if (!ptr) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    hipError_t e = hipMalloc(ptr, bytes ? bytes : 16);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
        // the library pool's idle reserve is not visible to hipMalloc: hand it back, retry once
        (void)hipGetLastError();
        if (trim_pool() == THESIA_OK) e = hipMalloc(ptr, bytes ? bytes : 16);
    }
    THESIA_HIP(e);
    return THESIA_OK;
}
int thesia_pool_trim(void) {
    GUARD_BEGIN
    return trim_pool();
    GUARD_END
}
int thesia_pool_bytes(uint64_t* reserved, uint64_t* used) {
    GUARD_BEGIN
    return pool_bytes(reserved, used);
    GUARD_END
}
int thesia_device_free(void* ptr) {
    THESIA_HIP(hipFree(ptr));
    return THESIA_OK;
}
int thesia_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    THESIA_HIP(copy_ordered(dst, src, bytes, hipMemcpyHostToDevice));
    return THESIA_OK;
}
int thesia_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    THESIA_HIP(copy_ordered(dst, src, bytes, hipMemcpyDeviceToHost));
    return THESIA_OK;
}
int thesia_host_register(void* host, size_t bytes) {
    if (!host || !bytes) return set_error(THESIA_ERR_INVALID_ARG, "null / empty host range");
    THESIA_HIP(hipHostRegister(host, bytes, hipHostRegisterDefault));
    return THESIA_OK;
}
int thesia_host_unregister(void* host) {
    THESIA_HIP(hipHostUnregister(host));
    return THESIA_OK;
}
int thesia_memset_device(void* dst, int value, size_t bytes) {
    THESIA_HIP(hipMemset(dst, value, bytes));
    return THESIA_OK;
}
int thesia_device_synchronize(void) {
    THESIA_HIP(hipDeviceSynchronize());
    return THESIA_OK;
}
int thesia_device_info(char* name, size_t cap, int* n_cu) {
    int dev = 0;
    THESIA_HIP(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    THESIA_HIP(hipGetDeviceProperties(&prop, dev));
    if (name && cap) {
        std::strncpy(name, prop.gcnArchName, cap - 1);
        name[cap - 1] = 0;
    }
    if (n_cu) *n_cu = prop.multiProcessorCount;
    return THESIA_OK;
}

int thesia_event_create(void** event) {
    if (!event) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    hipEvent_t e = nullptr;
    THESIA_HIP(hipEventCreate(&e));
    *event = e;
    return THESIA_OK;
}
int thesia_event_destroy(void* event) {
    if (event) THESIA_HIP(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return THESIA_OK;
}
int thesia_event_record(void* event, void* stream) {
    if (!event) return set_error(THESIA_ERR_INVALID_ARG, "null event");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : default_stream();
    THESIA_HIP(hipEventRecord(static_cast<hipEvent_t>(event), s));
    return THESIA_OK;
}
int thesia_event_elapsed_ms(void* start, void* stop, float* ms) {
    if (!start || !stop || !ms) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    THESIA_HIP(hipEventSynchronize(static_cast<hipEvent_t>(stop)));
    THESIA_HIP(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)));
    return THESIA_OK;
}

int thesia_hbm_ceiling(const void* d_src, size_t src_bytes, void* d_dst, size_t dst_bytes, int reps,
                       float* ms, float* gbps) {
    if (!d_src || !d_dst || !ms || src_bytes < 16 || dst_bytes < 16 || reps < 1 ||
        (reinterpret_cast<uintptr_t>(d_src) | reinterpret_cast<uintptr_t>(d_dst)) % 16)
        return set_error(THESIA_ERR_INVALID_ARG, "hbm_ceiling: 16-byte aligned non-empty buffers and reps >= 1");
    hipStream_t s = default_stream();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    THESIA_HIP(hipEventCreate(&e0));
    THESIA_HIP(hipEventCreate(&e1));
    float best = 0.0f;
    int rc = THESIA_OK;
    for (int grid : {2048, 8192}) {  // 8 / 32 blocks of 256 per CU (scripts/microbench/hbm_mix.hip)
        for (int r = 0; r <= reps && rc == THESIA_OK; ++r) {  // r = 0: warm-up
            float t = 0.0f;
            if (hipEventRecord(e0, s) != hipSuccess || hbm_mix(d_src, src_bytes, d_dst, dst_bytes, grid, s) ||
                hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&t, e0, e1) != hipSuccess)
                rc = set_error(THESIA_ERR_DEVICE, "hbm_ceiling launch failed");
            else if (r > 0 && (best == 0.0f || t < best))
                best = t;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    *ms = best;
    if (gbps) *gbps = (float)((double)(src_bytes / 16 + dst_bytes / 16) * 16.0 / (best * 1e-3) / 1e9);
    return THESIA_OK;
}

// ---------------------------------------------------------------- tables
int thesia_hann(size_t size, int symmetric, float* out) {
    GUARD_BEGIN
    if (size < 2) return set_error(THESIA_ERR_INVALID_ARG, "windows.rs:8 asserts size > 1");
    std::vector<float> w = hann(size, symmetric != 0);
    std::memcpy(out, w.data(), size * sizeof(float));
    return THESIA_OK;
    GUARD_END
}
size_t thesia_calc_proper_n_fft(size_t win_length) { return calc_proper_n_fft(win_length); }
float thesia_hz_to_mel(float hz) { return hz_to_mel(hz); }
float thesia_mel_to_hz(float mel) { return mel_to_hz(mel); }

int thesia_calc_mel_fb(uint32_t sr, size_t n_fft, size_t n_mel, float fmin, float fmax,
                       int do_norm, float* out) {
    GUARD_BEGIN
    if (n_fft % 2 || n_mel == 0) return set_error(THESIA_ERR_INVALID_ARG, "mel.rs:52-53 asserts");
    std::vector<float> fb = calc_mel_fb(sr, n_fft, n_mel, fmin, fmax, do_norm != 0);
    std::memcpy(out, fb.data(), fb.size() * sizeof(float));
    return THESIA_OK;
    GUARD_END
}

int thesia_calc_mel_fb_default(uint32_t sr, size_t n_fft, size_t* n_mel, float* out, size_t cap) {
    GUARD_BEGIN
    size_t nm = 0;
    std::vector<float> fb = calc_mel_fb_default(sr, n_fft, &nm);
    *n_mel = nm;
    if (!out) return THESIA_OK;
    if (cap < fb.size()) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "mel_fb buffer too small");
    std::memcpy(out, fb.data(), fb.size() * sizeof(float));
    return THESIA_OK;
    GUARD_END
}

void thesia_get_colormap(uint8_t out[30]) {
    for (int i = 0; i < 10; ++i)
        for (int k = 0; k < 3; ++k) out[i * 3 + k] = kColormap[i][k];
}

int thesia_track_params(uint32_t sr, float win_ms, size_t t_overlap, size_t f_overlap,
                        size_t* win, size_t* hop, size_t* n_fft) {
    if (t_overlap == 0) return set_error(THESIA_ERR_INVALID_ARG, "t_overlap must be > 0");
    track_params(sr, win_ms, t_overlap, f_overlap, win, hop, n_fft);
    return THESIA_OK;
}

// ---------------------------------------------------------------- perform_stft
size_t thesia_stft_n_frames(size_t n, size_t win, size_t hop) { return stft_n_frames(n, win, hop); }

int thesia_perform_stft(const float* input, size_t n, size_t win, size_t hop, size_t n_fft,
                        const float* window, float* out, size_t out_cap_frames, size_t* n_frames) {
    GUARD_BEGIN
    const uint64_t T = stft_n_frames(n, win, hop);
    if (T == 0) return set_error(THESIA_ERR_TOO_SHORT, "input shorter than win_length - 1 (lib.rs:413)");
    if (n_frames) *n_frames = T;
    if (!out || out_cap_frames < T) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "output too small");
    thesia_plan_desc d{};
    d.win_length = win;
    d.hop_length = hop;
    d.n_fft = n_fft;
    d.window = window;
    d.output = THESIA_OUT_COMPLEX;
    Plan* plan = nullptr;
    int rc = plan_create(d, &plan);
    if (rc) return rc;
    DevBuf din, dout;
    rc = din.upload(input, n * sizeof(float));
    const size_t F = n_fft / 2 + 1;
    if (!rc) rc = dout.alloc((size_t)T * F * 8);
    Batch* b = nullptr;
    if (!rc) {
        const uint64_t off = 0, len = n;
        thesia_batch_desc bd{};
        bd.input_format = THESIA_IN_F32;
        bd.channels = 1;
        bd.fold_mono = 0;
        bd.d_input = din.p;
        bd.track_offset = &off;
        bd.track_len = &len;
        bd.n_tracks = 1;
        bd.d_output = dout.p;
        rc = batch_create(plan, bd, &b);
    }
    if (!rc) rc = batch_run(b, default_stream());
    if (!rc) {
        hipError_t e = hipStreamSynchronize(default_stream());
        if (e == hipSuccess) e = copy_ordered(out, dout.p, (size_t)T * F * 8, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = set_error(THESIA_ERR_DEVICE, hipGetErrorString(e));
    }
    delete b;
    delete plan;
    return rc;
    GUARD_END
}

// ---------------------------------------------------------------- batch engine
int thesia_plan_create(const thesia_plan_desc* desc, thesia_plan** plan) {
    GUARD_BEGIN
    if (!desc || !plan) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    Plan* p = nullptr;
    int rc = plan_create(*desc, &p);
    if (rc) return rc;
    *plan = reinterpret_cast<thesia_plan*>(p);
    return THESIA_OK;
    GUARD_END
}
int thesia_plan_destroy(thesia_plan* plan) {
    // a plan's tables may still be read by work the caller enqueued on its own streams; its
    // buffers return to the stream-ordered pool (DevBuf), so wait for the device first, as the
    // hipFree this replaced did
    if (plan) (void)hipDeviceSynchronize();
    delete reinterpret_cast<Plan*>(plan);
    return THESIA_OK;
}
int thesia_plan_row_bins(const thesia_plan* plan, size_t* bins) {
    if (!plan || !bins) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    *bins = reinterpret_cast<const Plan*>(plan)->row_bins();
    return THESIA_OK;
}

int thesia_batch_create(thesia_plan* plan, const thesia_batch_desc* desc, thesia_batch** batch) {
    GUARD_BEGIN
    if (!plan || !desc || !batch) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    Batch* b = nullptr;
    int rc = batch_create(reinterpret_cast<Plan*>(plan), *desc, &b);
    if (rc) return rc;
    *batch = reinterpret_cast<thesia_batch*>(b);
    return THESIA_OK;
    GUARD_END
}
int thesia_batch_destroy(thesia_batch* batch) {
    // no device synchronisation: the batch's only device block (its track tables) was last used
    // on the stream of its last run, where its release is ordered (engine.hpp, the block cache's
    // invariant); the caller's input / output buffers stay the caller's
    delete reinterpret_cast<Batch*>(batch);
    return THESIA_OK;
}
int thesia_batch_frames(const thesia_batch* batch, uint64_t* total, uint64_t* frame0) {
    if (!batch) return set_error(THESIA_ERR_INVALID_ARG, "null batch");
    const Batch* b = reinterpret_cast<const Batch*>(batch);
    if (total) *total = b->total_frames;
    if (frame0) std::memcpy(frame0, b->frame0.data(), b->frame0.size() * 8);
    return THESIA_OK;
}
int thesia_batch_output_bytes(const thesia_batch* batch, uint64_t* bytes) {
    if (!batch || !bytes) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    const Batch* b = reinterpret_cast<const Batch*>(batch);
    *bytes = b->total_frames * b->plan->row_bins() * b->plan->out_elem_bytes();
    return THESIA_OK;
}
int thesia_batch_run(thesia_batch* batch, void* stream) {
    GUARD_BEGIN
    if (!batch) return set_error(THESIA_ERR_INVALID_ARG, "null batch");
    return batch_run(reinterpret_cast<Batch*>(batch), static_cast<hipStream_t>(stream));
    GUARD_END
}
int thesia_batches_run(thesia_batch* const* batches, size_t n, void* stream) {
    GUARD_BEGIN
    if (n && !batches) return set_error(THESIA_ERR_INVALID_ARG, "null batches");
    for (size_t i = 0; i < n; ++i)
        if (!batches[i]) return set_error(THESIA_ERR_INVALID_ARG, "null batch");
    return batches_run(reinterpret_cast<Batch* const*>(batches), n, static_cast<hipStream_t>(stream));
    GUARD_END
}
int thesia_batch_run_timed(thesia_batch* batch, void* stream, int iters, float* ms) {
    GUARD_BEGIN
    if (!batch || iters < 1) return set_error(THESIA_ERR_INVALID_ARG, "bad argument");
    Batch* b = reinterpret_cast<Batch*>(batch);
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : default_stream();
    THESIA_HIP(hipEventRecord(b->ev0, s));
    for (int i = 0; i < iters; ++i) {
        int rc = batch_run(b, s);
        if (rc) return rc;
    }
    THESIA_HIP(hipEventRecord(b->ev1, s));
    THESIA_HIP(hipEventSynchronize(b->ev1));
    float t = 0.f;
    THESIA_HIP(hipEventElapsedTime(&t, b->ev0, b->ev1));
    if (ms) *ms = t;
    return THESIA_OK;
    GUARD_END
}
int thesia_batch_kernel_info(const thesia_batch* batch, int* lds_bytes, int* tile_frames, int* grid) {
    if (!batch) return set_error(THESIA_ERR_INVALID_ARG, "null batch");
    const Batch* b = reinterpret_cast<const Batch*>(batch);
    if (lds_bytes) *lds_bytes = b->plan->lds_bytes;
    if (tile_frames) *tile_frames = b->plan->tile_frames;
    if (grid) *grid = b->launch.grid;
    return THESIA_OK;
}

int thesia_batch_kernel(const thesia_batch* batch, int* kernel) {
    if (!batch || !kernel) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    *kernel = reinterpret_cast<const Batch*>(batch)->kernel;
    return THESIA_OK;
}

int thesia_batch_set_option(thesia_batch* batch, int option, int64_t value) {
    GUARD_BEGIN
    if (!batch) return set_error(THESIA_ERR_INVALID_ARG, "null batch");
    return batch_set_option(reinterpret_cast<Batch*>(batch), option, value);
    GUARD_END
}

int thesia_set_render_path(int path) { return set_render_path(path); }
int thesia_get_render_path(void) { return render_path(); }
int thesia_set_batches_policy(int policy) { return set_batches_policy(policy); }


int thesia_synth_pcm_device(void* d_out, int format, uint32_t channels, uint64_t n_tracks,
                            uint64_t n_samples, uint32_t sr, uint64_t seed) {
    GUARD_BEGIN
    static DevBuf lut;  // per process (single device use in benches / tests)
    static int lut_dev = -1;
    int dev = 0;
    THESIA_HIP(hipGetDevice(&dev));
    if (lut_dev != dev) {
        int rc = lut.upload(synth_lut_host(), 4096 * sizeof(int16_t));
        if (rc) return rc;
        lut_dev = dev;
    }
    if (launch_synth_pcm(d_out, format, channels, n_tracks, n_samples, sr, seed, lut.as<int16_t>(),
                         default_stream()))
        return set_error(THESIA_ERR_DEVICE, "synth launch failed");
    THESIA_HIP(hipStreamSynchronize(default_stream()));
    return THESIA_OK;
    GUARD_END
}
int thesia_synth_pcm_host(int16_t* out, uint32_t channels, uint64_t track, uint64_t n_samples,
                          uint32_t sr, uint64_t seed) {
    GUARD_BEGIN
    synth_host(out, channels, track, n_samples, sr, seed, synth_lut_host());
    return THESIA_OK;
    GUARD_END
}

// ---------------------------------------------------------------- display primitives
int thesia_spec_grey_height(size_t bins, float up_ratio, uint32_t* height) {
    const float h = roundf((float)bins * up_ratio);
    *height = h > 0.f ? (h >= 4294967295.0f ? 4294967295u : (uint32_t)h) : 0u;
    return THESIA_OK;
}

int thesia_spec_to_grey(const float* spec, size_t T, size_t bins, float up_ratio, float max,
                        float min, float* grey, size_t cap) {
    GUARD_BEGIN
    uint32_t H = 0;
    thesia_spec_grey_height(bins, up_ratio, &H);
    if (H < bins) return set_error(THESIA_ERR_INVALID_ARG, "up_ratio < 1 (display.rs:47 underflows)");
    if (cap < (size_t)H * T) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "grey buffer too small");
    DevBuf ds, dg;
    int rc = ds.upload(spec, T * bins * sizeof(float));
    if (!rc) rc = dg.alloc((size_t)H * T * sizeof(float));
    if (rc) return rc;
    if (launch_spec_to_grey(ds.as<float>(), (uint32_t)T, (uint32_t)bins, H, max, min, dg.as<float>(), default_stream()))
        return set_error(THESIA_ERR_DEVICE, "spec_to_grey launch failed");
    THESIA_HIP(hipStreamSynchronize(default_stream()));
    THESIA_HIP(copy_ordered(grey, dg.p, (size_t)H * T * sizeof(float), hipMemcpyDeviceToHost));
    return THESIA_OK;
    GUARD_END
}

int thesia_grey_to_rgb(const float* grey, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                       uint8_t* out, size_t cap) {
    GUARD_BEGIN
    const size_t bytes = (size_t)nw * nh * 3;
    if (cap < bytes) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "rgb buffer too small");
    if (bytes == 0) return THESIA_OK;
    DevBuf dg, drgb;
    int rc = dg.upload(grey, (size_t)w * h * sizeof(float));
    if (!rc) rc = drgb.alloc(bytes);
    if (!rc) rc = grey_to_rgb_device(dg.as<float>(), w, h, nw, nh, drgb.as<uint8_t>(), default_stream());
    if (rc) return rc;
    THESIA_HIP(copy_ordered(out, drgb.p, bytes, hipMemcpyDeviceToHost));
    return THESIA_OK;
    GUARD_END
}

int thesia_minmax_device(const float* d_x, uint64_t n, float* max, float* min, int* has_nan) {
    GUARD_BEGIN
    if (!max || !min || (n && !d_x)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    bool nan = false;
    int rc = minmax_device(d_x, n, max, min, &nan, default_stream());
    if (has_nan) *has_nan = nan ? 1 : 0;
    return rc;
    GUARD_END
}

int thesia_spec_to_grey_device(const float* d_spec, size_t T, size_t bins, float up_ratio,
                               float max, float min, float* d_grey) {
    GUARD_BEGIN
    uint32_t H = 0;
    thesia_spec_grey_height(bins, up_ratio, &H);
    if (H < bins) return set_error(THESIA_ERR_INVALID_ARG, "up_ratio < 1 (display.rs:47 underflows)");
    if (T == 0 || H == 0) return THESIA_OK;
    if (!d_spec || !d_grey) return set_error(THESIA_ERR_INVALID_ARG, "null device pointer");
    if (launch_spec_to_grey(d_spec, (uint32_t)T, (uint32_t)bins, H, max, min, d_grey, default_stream()))
        return set_error(THESIA_ERR_DEVICE, "spec_to_grey launch failed");
    THESIA_HIP(hipStreamSynchronize(default_stream()));
    return THESIA_OK;
    GUARD_END
}

int thesia_grey_to_rgb_device(const float* d_grey, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                              uint8_t* d_rgb) {
    GUARD_BEGIN
    if ((size_t)nw * nh == 0) return THESIA_OK;
    if (!d_grey || !d_rgb) return set_error(THESIA_ERR_INVALID_ARG, "null device pointer");
    return grey_to_rgb_device(d_grey, w, h, nw, nh, d_rgb, default_stream());
    GUARD_END
}

int thesia_minmax_segments_device(const float* d_spec, const uint64_t* row0, size_t bins,
                                  size_t n, float* max, float* min, int* has_nan) {
    GUARD_BEGIN
    if (n && (!d_spec || !row0 || !max || !min || !has_nan))
        return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    return minmax_segments_device(d_spec, row0, bins, n, max, min, has_nan, default_stream());
    GUARD_END
}

int thesia_render_rgb_batch_device(const float* d_spec, const uint64_t* row0, size_t bins,
                                   size_t n, const float* up_ratio, const uint32_t* nwidth,
                                   uint32_t nheight, float max, float min, uint8_t* d_rgb,
                                   const uint64_t* rgb_off) {
    GUARD_BEGIN
    if (n && (!d_spec || !row0 || !up_ratio || !nwidth || !d_rgb || !rgb_off))
        return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    return render_rgb_batch_device(d_spec, row0, bins, n, up_ratio, nwidth, nheight, max, min,
                                   d_rgb, rgb_off, default_stream());
    GUARD_END
}

int thesia_batch_ranges_read(const void* d_range, size_t n, float* max, float* min, int* has_nan) {
    GUARD_BEGIN
    if (n && (!d_range || !max || !min || !has_nan)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    return ranges_read(static_cast<const int*>(d_range), n, max, min, has_nan, default_stream());
    GUARD_END
}

int thesia_minmax_segments_multi(size_t n_groups, const float* const* d_specs,
                                 const uint64_t* const* row0s, const size_t* bins, const size_t* ns,
                                 float* max, float* min, int* has_nan) {
    GUARD_BEGIN
    if (n_groups && (!d_specs || !row0s || !bins || !ns || !max || !min || !has_nan))
        return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    for (size_t k = 0; k < n_groups; ++k)
        if (ns[k] && (!d_specs[k] || !row0s[k])) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    return minmax_segments_multi(n_groups, d_specs, row0s, bins, ns, max, min, has_nan, default_stream());
    GUARD_END
}

int thesia_render_rgb_multi(size_t n_groups, const float* const* d_specs, const uint64_t* const* row0s,
                            const size_t* bins, const size_t* ns, const float* up_ratio,
                            const uint32_t* nwidth, uint32_t nheight, float max, float min,
                            uint8_t* d_rgb, const uint64_t* rgb_off) {
    GUARD_BEGIN
    size_t tot = 0;
    if (n_groups && (!d_specs || !row0s || !bins || !ns)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    for (size_t k = 0; k < n_groups; ++k) {
        if (ns[k] && (!d_specs[k] || !row0s[k])) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
        tot += ns[k];
    }
    if (tot && (!up_ratio || !nwidth || !d_rgb || !rgb_off)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    if (render_path() == 0 || render_path() >= 3)
        return render_rgb_fused(n_groups, d_specs, row0s, bins, ns, up_ratio, nwidth, nheight, max, min,
                                d_rgb, rgb_off, default_stream());
    size_t t0 = 0;
    for (size_t k = 0; k < n_groups; ++k) {
        const int rc = render_rgb_batch_device(d_specs[k], row0s[k], bins[k], ns[k], up_ratio + t0,
                                               nwidth + t0, nheight, max, min, d_rgb, rgb_off + t0,
                                               default_stream());
        if (rc) return rc;
        t0 += ns[k];
    }
    return THESIA_OK;
    GUARD_END
}

int thesia_ranges_global(const int* d_trk_range, size_t n, float db_range, float* d_out) {
    GUARD_BEGIN
    if (!d_out || (n && !d_trk_range)) return set_error(THESIA_ERR_INVALID_ARG, "null device pointer");
    if (n > 0xFFFFFFFFull) return set_error(THESIA_ERR_INVALID_ARG, "too many tracks");
    if (launch_range_global(d_trk_range, (uint32_t)n, (double)db_range, d_out, default_stream()))
        return set_error(THESIA_ERR_DEVICE, "range_global launch failed");
    return THESIA_OK;
    GUARD_END
}

int thesia_render_rgb_multi_dev(size_t n_groups, const float* const* d_specs, const uint64_t* const* row0s,
                                const size_t* bins, const size_t* ns, const float* up_ratio,
                                const uint32_t* nwidth, uint32_t nheight, const float* d_range,
                                uint8_t* d_rgb, const uint64_t* rgb_off) {
    GUARD_BEGIN
    size_t tot = 0;
    if (!d_range) return set_error(THESIA_ERR_INVALID_ARG, "null device range");
    if (n_groups && (!d_specs || !row0s || !bins || !ns)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    for (size_t k = 0; k < n_groups; ++k) {
        if (ns[k] && (!d_specs[k] || !row0s[k])) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
        tot += ns[k];
    }
    if (tot && (!up_ratio || !nwidth || !d_rgb || !rgb_off)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    if (!(render_path() == 0 || render_path() >= 3))
        return set_error(THESIA_ERR_UNSUPPORTED, "render_rgb_multi_dev: the fused render paths (0, 3, 4) only");
    return render_rgb_fused(n_groups, d_specs, row0s, bins, ns, up_ratio, nwidth, nheight, 0.0f, 0.0f,
                            d_rgb, rgb_off, default_stream(), d_range);
    GUARD_END
}

int thesia_inv_real_fft_device(const float* d_in, size_t n_frames, size_t length, float* d_out) {
    GUARD_BEGIN
    if (n_frames && (!d_in || !d_out)) return set_error(THESIA_ERR_INVALID_ARG, "null device pointer");
    return inv_real_fft_device(d_in, n_frames, length, d_out, default_stream());
    GUARD_END
}

int thesia_inv_real_fft(const float* in, size_t n_frames, size_t length, float* out) {
    GUARD_BEGIN
    if (n_frames && (!in || !out)) return set_error(THESIA_ERR_INVALID_ARG, "null pointer");
    if (length % 2) return set_error(THESIA_ERR_INVALID_ARG, "Length must be even (realfft.rs:171)");
    if (n_frames == 0) return inv_real_fft_device(nullptr, 0, length, nullptr, default_stream());
    DevBuf din, dout;
    int rc = din.upload(in, n_frames * (length / 2 + 1) * 2 * sizeof(float));
    if (!rc) rc = dout.alloc(n_frames * length * sizeof(float));
    if (!rc) rc = inv_real_fft_device(din.as<float>(), n_frames, length, dout.as<float>(), default_stream());
    if (rc) return rc;
    THESIA_HIP(hipStreamSynchronize(default_stream()));
    THESIA_HIP(copy_ordered(out, dout.p, n_frames * length * sizeof(float), hipMemcpyDeviceToHost));
    return THESIA_OK;
    GUARD_END
}

int thesia_wav_to_image(const float* wav, size_t n, uint32_t nwidth, uint32_t nheight,
                        float amp_min, float amp_max, uint8_t* out, size_t cap) {
    GUARD_BEGIN
    const size_t bytes = (size_t)nwidth * nheight * 4;
    if (cap < bytes) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "rgba buffer too small");
    if (bytes == 0) return THESIA_OK;
    DevBuf dw, dimg;
    int rc = dw.upload(wav, n * sizeof(float));
    if (!rc) rc = dimg.alloc(bytes);
    int panicked = 0;
    if (!rc) rc = wav_to_image_device(dw.as<float>(), n, nwidth, nheight, amp_min, amp_max,
                                      dimg.as<uint8_t>(), &panicked, default_stream());
    if (rc) return rc;
    THESIA_HIP(copy_ordered(out, dimg.p, bytes, hipMemcpyDeviceToHost));
    if (panicked)
        return set_error(THESIA_ERR_PANIC, "the reference panics for these arguments (display.rs:95-108); "
                                           "the image is written with the column clamped");
    return THESIA_OK;
    GUARD_END
}

// ---------------------------------------------------------------- MultiTrack
int thesia_mt_create(thesia_mt** mt) {
    GUARD_BEGIN
    *mt = reinterpret_cast<thesia_mt*>(new MultiTrack());
    return THESIA_OK;
    GUARD_END
}
void thesia_mt_destroy(thesia_mt* mt) {
    if (!mt) return;
    delete reinterpret_cast<MultiTrack*>(mt);
    (void)trim_pool();  // the handle's buffers leave the library pool's reserve too
}

static MultiTrack* M(thesia_mt* mt) { return reinterpret_cast<MultiTrack*>(mt); }
static const MultiTrack* M(const thesia_mt* mt) { return reinterpret_cast<const MultiTrack*>(mt); }

int thesia_mt_set_setting(thesia_mt* mt, float win_ms, size_t t_overlap, size_t f_overlap,
                          int freq_scale, float db_range) {
    GUARD_BEGIN
    return M(mt)->set_setting(win_ms, t_overlap, f_overlap, freq_scale, db_range);
    GUARD_END
}

int thesia_mt_set_fast(thesia_mt* mt, int fast) {
    if (!mt) return set_error(THESIA_ERR_INVALID_ARG, "null handle");
    if (fast != 0 && fast != 1) return set_error(THESIA_ERR_INVALID_ARG, "fast must be 0 or 1");
    M(mt)->set_fast(fast == 1);
    return THESIA_OK;
}

static std::vector<std::string> split_paths(const char* paths) {
    std::vector<std::string> out;
    std::string s(paths ? paths : "");
    size_t start = 0;
    while (true) {  // path_list.split("\n"), lib.rs:173
        const size_t e = s.find('\n', start);
        out.push_back(s.substr(start, e == std::string::npos ? std::string::npos : e - start));
        if (e == std::string::npos) break;
        start = e + 1;
    }
    return out;
}

int thesia_mt_add_tracks(thesia_mt* mt, const uint64_t* ids, size_t n_ids, const char* paths,
                         int* changed) {
    GUARD_BEGIN
    std::vector<std::string> pl = split_paths(paths);
    const size_t n = std::min(n_ids, pl.size());  // zip stops at the shorter list
    std::vector<WavData> wavs(n);
    std::vector<uint64_t> idv(ids, ids + n);
    std::vector<PcmIn> pcm(n);
    // the files are read straight into the handle's page-locked staging (one read per file, no
    // copy of the samples on the host; the uploads then run as DMA), sized from the files
    std::vector<size_t> fsz(n, 0), foff(n + 1, 0);
    for (size_t i = 0; i < n; ++i) {
        std::string err;
        int rc = wav_file_size(pl[i], &fsz[i], &err);
        if (rc) return set_error(rc, err);
        foff[i + 1] = foff[i] + ((fsz[i] + 63) & ~size_t(63));
    }
    PinnedTmp big;  // a call larger than the handle's kept staging (freed when the call returns)
    uint8_t* stage = M(mt)->staging(foff[n], &big);
    // the files read concurrently (the reference's per-track rayon loop, lib.rs:161-166, reads
    // and transforms each track on its own worker); errors reported in list order
    std::vector<int> rcs(n, 0);
    std::vector<std::string> errs(n);
    auto read_one = [&](size_t i) {
        rcs[i] = stage && fsz[i] ? read_wav_into(pl[i], stage + foff[i], fsz[i], &wavs[i], &errs[i])
                                 : read_wav(pl[i], &wavs[i], &errs[i]);
    };
    const size_t nthr = std::min<size_t>(n, std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
    if (nthr <= 1) {
        for (size_t i = 0; i < n; ++i) read_one(i);
    } else {
        std::atomic<size_t> next{0};
        std::vector<std::thread> pool;
        for (size_t t = 0; t < nthr; ++t)
            pool.emplace_back([&] {
                for (size_t i; (i = next.fetch_add(1)) < n;) read_one(i);
            });
        for (auto& th : pool) th.join();
    }
    for (size_t i = 0; i < n; ++i) {
        if (rcs[i]) return set_error(rcs[i], errs[i]);
        pcm[i].data = wavs[i].samples();
        pcm[i].kind = wavs[i].kind;
        pcm[i].scale = pcm_scale(wavs[i].kind, wavs[i].bits);
        pcm[i].channels = wavs[i].channels;
        pcm[i].n_samples = wavs[i].n_frames;
        pcm[i].sr = wavs[i].sr;
        pcm[i].path = pl[i];
    }
    return M(mt)->add_tracks(idv, pcm, changed);
    GUARD_END
}

int thesia_mt_add_tracks_pcm(thesia_mt* mt, const uint64_t* ids, size_t n_ids,
                             const float* const* pcm_in, const uint64_t* n_samples,
                             const uint32_t* channels, const uint32_t* sr, const char* paths,
                             int* changed) {
    GUARD_BEGIN
    std::vector<std::string> pl = split_paths(paths);
    std::vector<uint64_t> idv(ids, ids + n_ids);
    std::vector<PcmIn> pcm(n_ids);
    for (size_t i = 0; i < n_ids; ++i) {
        pcm[i].data = pcm_in[i];
        pcm[i].kind = PCM_F32;
        pcm[i].n_samples = n_samples[i];
        pcm[i].channels = channels[i];
        pcm[i].sr = sr[i];
        pcm[i].path = i < pl.size() ? pl[i] : std::string();
    }
    return M(mt)->add_tracks(idv, pcm, changed);
    GUARD_END
}

int thesia_mt_remove_track(thesia_mt* mt, uint64_t id, int* changed) {
    GUARD_BEGIN
    return M(mt)->remove_track(id, changed);
    GUARD_END
}

int thesia_mt_get_spec_image(thesia_mt* mt, uint64_t id, float px_per_sec, uint32_t nheight,
                             uint8_t* out, size_t cap, size_t* needed) {
    GUARD_BEGIN
    return M(mt)->spec_image(id, px_per_sec, nheight, out, cap, needed);
    GUARD_END
}

int thesia_mt_get_wav_image(thesia_mt* mt, uint64_t id, float px_per_sec, uint32_t nheight,
                            float amp_min, float amp_max, uint8_t* out, size_t cap, size_t* needed) {
    GUARD_BEGIN
    return M(mt)->wav_image(id, px_per_sec, nheight, amp_min, amp_max, out, cap, needed);
    GUARD_END
}

int thesia_mt_get_frequency_hz(thesia_mt* mt, uint64_t id, float rel, float* hz) {
    return M(mt)->frequency_hz(id, rel, hz);
}
float thesia_mt_get_max_db(const thesia_mt* mt) { return M(mt)->max_db(); }
float thesia_mt_get_min_db(const thesia_mt* mt) { return M(mt)->min_db(); }
float thesia_mt_get_max_sec(const thesia_mt* mt) { return M(mt)->max_sec(); }

int thesia_mt_get_sec(const thesia_mt* mt, uint64_t id, float* sec) {
    const Track* t = M(mt)->find(id);
    if (!t) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    *sec = (float)t->n / (float)t->sr;  // lib.rs:336-339
    return THESIA_OK;
}
int thesia_mt_get_sr(const thesia_mt* mt, uint64_t id, uint32_t* sr) {
    const Track* t = M(mt)->find(id);
    if (!t) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    *sr = t->sr;
    return THESIA_OK;
}
int thesia_mt_get_path(const thesia_mt* mt, uint64_t id, char* out, size_t cap, size_t* needed) {
    const Track* t = M(mt)->find(id);
    if (!t) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    std::string s = t->path;
    s.push_back('\0');
    return copy_out(s.data(), s.size(), out, cap, needed);
}
int thesia_mt_get_filename(const thesia_mt* mt, uint64_t id, char* out, size_t cap, size_t* needed) {
    const Track* t = M(mt)->find(id);
    if (!t) return set_error(THESIA_ERR_UNKNOWN_ID, "unknown track id");
    std::string s = MultiTrack::filename_of(*t);
    s.push_back('\0');
    return copy_out(s.data(), s.size(), out, cap, needed);
}
int thesia_mt_get_spec(const thesia_mt* mt, uint64_t id, float* out, size_t cap, size_t* T,
                       size_t* bins) {
    GUARD_BEGIN
    std::vector<float> v;
    int rc = M(mt)->spec_host(id, &v, T, bins);
    if (rc) return rc;
    if (!out) return THESIA_OK;
    if (cap < v.size()) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "spec buffer too small");
    std::memcpy(out, v.data(), v.size() * 4);
    return THESIA_OK;
    GUARD_END
}
int thesia_mt_get_wav(const thesia_mt* mt, uint64_t id, float* out, size_t cap, size_t* n) {
    GUARD_BEGIN
    std::vector<float> v;
    int rc = M(mt)->wav_host(id, &v);
    if (rc) return rc;
    if (n) *n = v.size();
    if (!out) return THESIA_OK;
    if (cap < v.size()) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "wav buffer too small");
    std::memcpy(out, v.data(), v.size() * 4);
    return THESIA_OK;
    GUARD_END
}

int thesia_open_audio_file(const char* path, float* out, size_t cap, size_t* n_floats, uint32_t* sr,
                           uint32_t* channels) {
    GUARD_BEGIN
    if (!path) return set_error(THESIA_ERR_INVALID_ARG, "null path");
    WavData w;
    std::string err;
    int rc = read_wav(path, &w, &err);
    if (rc) return set_error(rc, err);
    const size_t n = (size_t)w.n_frames * w.channels;
    if (n_floats) *n_floats = n;
    if (sr) *sr = w.sr;
    if (channels) *channels = w.channels;
    if (!out) return THESIA_OK;
    if (cap < n) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "sample buffer too small");
    decode_pcm_f32(w.samples(), w.kind, pcm_scale(w.kind, w.bits), n, out);
    return THESIA_OK;
    GUARD_END
}

int thesia_mt_get_grey(const thesia_mt* mt, uint64_t id, float* out, size_t cap, uint32_t* w,
                       uint32_t* h) {
    GUARD_BEGIN
    std::vector<float> v;
    int rc = M(mt)->grey_host(id, &v, w, h);
    if (rc) return rc;
    if (!out) return THESIA_OK;
    if (cap < v.size()) return set_error(THESIA_ERR_BUFFER_TOO_SMALL, "grey buffer too small");
    std::memcpy(out, v.data(), v.size() * 4);
    return THESIA_OK;
    GUARD_END
}
int thesia_mt_track_count(const thesia_mt* mt, size_t* n) {
    *n = M(mt)->size();
    return THESIA_OK;
}

int thesia_mt_device_bytes(const thesia_mt* mt, size_t* bytes) {
    if (!mt || !bytes) return set_error(THESIA_ERR_INVALID_ARG, "null argument");
    *bytes = M(mt)->device_bytes();
    return THESIA_OK;
}

}  // extern "C"
