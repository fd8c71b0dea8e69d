// engine.hpp -- internal C++ runtime of libthesia: errors, device buffers, streams, plans
// (per-(sr, win, hop, n_fft, output) tables resident in HBM) and batches (track
// descriptors resident in HBM, one launch per pass).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/thesia.h"
#include "kernels.hpp"

namespace thesia {

// ---- errors: thread-local message + status code (never abort across the C ABI) ----
int set_error(int code, const std::string& msg);
void clear_error();
const char* last_error();

#define THESIA_HIP(expr)                                                                 \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return ::thesia::set_error(THESIA_ERR_DEVICE,                                \
                                       std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// ---- device buffer (move-only RAII) ----
// hipMalloc'd blocks kept by the library's block cache (engine.cpp) once released: a release
// costs no device synchronisation (a hipFree costs ~160 us, profiles/r03_viewer).
//
// The cache's invariant (round 6): a block may be handed out again only after every use of it
// has been ordered before the next user's work. A block last used on its allocation stream (the
// library stream) is released with an event recorded there and goes back out at once to the next
// allocation on that stream (in order behind the uses), to other streams once the event has
// completed. A block whose work ran on another stream -- a caller's, for a batch run there --
// is marked by used_on(s) right after that work is enqueued: an event recorded on s then (the
// stream may be gone by the release: only the event is kept), and the released block goes back
// out only once that event has completed, on any stream. Work on the library's pool streams is
// joined into the caller's stream before used_on (batches_run). tests/test_gpu_multitrack.py
// test_block_cache_cross_stream_reuse checks a block released while a kernel on a busy caller
// stream still reads it.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t st = nullptr;      // the stream it was allocated on
    hipEvent_t use_ev = nullptr;   // recorded after its last use on another stream (used_on)
    bool foreign = false;          // last used on another stream: released behind use_ev only
    bool pooled = false;           // a block of the cache (else a plain hipFree on release)
    int dev = 0;                   // the device it was allocated on
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept
        : p(o.p), bytes(o.bytes), st(o.st), use_ev(o.use_ev), foreign(o.foreign), pooled(o.pooled), dev(o.dev) {
        o.p = nullptr;
        o.bytes = 0;
        o.use_ev = nullptr;
        o.foreign = false;
    }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            if (use_ev) (void)hipEventDestroy(use_ev);
            p = o.p; bytes = o.bytes; st = o.st; use_ev = o.use_ev; foreign = o.foreign; pooled = o.pooled; dev = o.dev;
            o.p = nullptr; o.bytes = 0; o.use_ev = nullptr; o.foreign = false;
        }
        return *this;
    }
    ~DevBuf() {
        release();
        if (use_ev) (void)hipEventDestroy(use_ev);
    }
    void release();
    int alloc(size_t n);
    int upload(const void* host, size_t n);  // alloc + copy (synchronous)
    // the block's work has just been enqueued on (or joined into) stream s: its release is
    // ordered behind that work (an event recorded on s now, unless s is the allocation stream)
    void used_on(hipStream_t s);
    template <class T> T* as() const { return static_cast<T*>(p); }
};

hipStream_t default_stream();  // library stream of the current device
// the block cache: hand every idle block back to the device (after the work ordered before
// their release completes); the current device's cached + handed-out / handed-out bytes
int trim_pool();
int pool_bytes(uint64_t* reserved, uint64_t* used);
hipError_t copy_ordered(void* dst, const void* src, size_t bytes, hipMemcpyKind kind);
bool host_pinned(const void* p);  // page-locked (hipHostMalloc / hipHostRegister) host memory
// a copy on stream s: async where the host side is page-locked (or device to device); with a
// pageable host side the copy is enqueued on s and s is synchronised before the call returns
// (the host range may be reused at once; nothing else in the process waits)
hipError_t copy_on(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s);

// ---- plan ----
struct Plan {
    thesia_plan_desc desc{};
    int out_kind = 0;
    size_t n_fft = 0, NC = 0, win = 0, hop = 0, pad_left = 0;
    size_t n_mels = 0;
    std::vector<float> window;  // [win]
    std::vector<float> mel_fb;  // [F, n_mels]
    float log_amin = 0.f;
    int tile_frames = 0, lds_bytes = 0;
    DevBuf wpad, tw, tw2, tw3, sincos, mel_round, mel_k0, mel_wt;
    int mel_rounds = 0;
    size_t mel_wt_rows = 0;  // padded band lengths summed over the rounds
    DevBuf mel4_round, mel4_k0, mel4_wt;  // stft2_kernel layout (float4 steps)
    int mel4_rounds = 0;
    DevBuf mel_xo;      // the rounds as a chunk stream (kernels.hpp mel_xo)
    DevBuf xpos, xmel_band, xmel_w;  // the reference-order kernel's tables (stftx)
    float xw8[4] = {0.f, 0.f, 0.f, 0.f};
    int mel_chunks = 0;
    size_t mel4_wt_rows = 0;
    // stft5's packed mel stream, built for 2 and 3 float4 steps per chunk (build_melp)
    struct Melp {
        DevBuf meta, wt;
        int chunks = 0;  // 0: not available for this filterbank
        int steps = 0;
    } melp[2];
    int melp_best = -1;  // index into melp of the default (fewest estimated instructions), -1 none
    Melp melr[2];        // the same stream for 64 lanes per frame (stftr_kernel)
    int melr_best = -1;
    bool use_v2 = false;  // stft2_kernel runs this plan (n_fft 256..2048)
    size_t row_bins() const;
    size_t out_elem_bytes() const { return out_kind == OUT_COMPLEX ? 8 : 4; }
};
int plan_create(const thesia_plan_desc& d, Plan** out);

// ---- batch ----
struct Batch {
    Plan* plan = nullptr;
    thesia_batch_desc desc{};
    std::vector<uint64_t> in_off, len, frame0;
    DevBuf d_tabs;  // [in_off | len | frame0] on the device (launch.trk_* point into it)
    uint64_t total_frames = 0;
    StftLaunch launch{};
    // 1 stft_kernel, 2 stft2_kernel, 3 stft3_kernel, 5 stft5_kernel (streaming), 7 stftr_kernel
    // (streaming, reference operation order), 9 stftx_kernel (reference operation order)
    int kernel = 1;
    bool k3_ok = false;  // the streaming kernel supports this batch's geometry
    bool k5_ok = false;  // ... and so does its n_fft 2048 variant (stft5_kernel)
    bool kr_ok = false;  // the reference-order streaming kernel (stftr_kernel) runs this batch
    // automatic choice: stft5 for the mel kinds at n_fft 2048 and for linear rows without the
    // range option (measured faster there: stereo power dB 5.64 vs 6.22 ms in round 3; slower for
    // complex rows, 9.0 vs 6.98 ms, and stft3 folds the per-track range into its row epilogue;
    // DESIGN.md §6), stft3 for the other streaming geometries, then the 4-waves/SIMD kernel for
    // its sizes, else the general one
    // at the viewer geometry (k5_view) stft5 pays only on large batches: its per-block setup
    // (the packed mel stream, the rotation tables) against stft3's, measured at 48 kHz mel-128
    // (profiles/r04_viewer/batch_size_ab.txt): 3.0e6 frames 4.48 vs 4.76 ms, 3.0e5 0.576 vs
    // 0.570, 2.6e4 0.102 vs 0.077
    static constexpr uint64_t kView5MinFrames = 400000;
    bool k5_view = false;
    int auto_kernel() const {
        const bool mel = launch.out_kind == OUT_MEL || launch.out_kind == OUT_MEL_AMP_DB;
        const bool lin = !mel && launch.out_kind != OUT_COMPLEX && !range;
        const bool k5 = k5_ok && (mel || lin) && (!k5_view || total_frames >= kView5MinFrames);
        return k5 ? 5 : k3_ok ? 3 : plan->use_v2 ? 2 : 1;
    }
    bool kernel_forced = false;  // THESIA_BATCH_OPT_KERNEL set a kernel (else auto_kernel follows)
    // mel projection of stft5 (THESIA_BATCH_OPT_MEL_PATH): 0 automatic, 1 the rounds' chunk
    // stream (mel4p), 2 / 3 the packed stream with 2 / 3 float4 steps per chunk
    int mel_path = 0;
    void apply_mel_path();
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int* range = nullptr;  // THESIA_BATCH_OPT_RANGE: per-track {ord max, ord min, NaN} on the device
    ~Batch();
};
int batch_create(Plan* plan, const thesia_batch_desc& d, Batch** out);
int batch_run(Batch* b, hipStream_t s);
int batches_run(Batch* const* b, size_t n, hipStream_t s);  // thesia_batches_run
int batches_policy();  // thesia_set_batches_policy
int set_batches_policy(int policy);
int batch_set_option(Batch* b, int option, int64_t value);  // thesia_batch_set_option
int ranges_read(const int* d_range, size_t n, float* mx, float* mn, int* nan, hipStream_t s);

// display path selection (thesia_set_render_path): 0 fused batched launches (the single-pass
// stripe kernel for the groups that downsample along time at least 3:1, else grey + vertical in
// one pass, then horizontal + colormap), 1 per-track launches, 2 three-stage batched launches
// (grey, vertical, horizontal + colormap), 3 path 0 without the stripe kernel, 4 path 0 with the
// stripe kernel wherever its instances cover the geometry
int render_path();
int set_render_path(int path);

// ---- display helpers on device buffers (used by MultiTrack and the C ABI) ----
int grey_to_rgb_device(const float* d_grey, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                       uint8_t* d_rgb, hipStream_t s);
int wav_to_image_device(const float* d_wav, uint64_t n, uint32_t nwidth, uint32_t nheight,
                        float amp_min, float amp_max, uint8_t* d_out, int* panicked,
                        hipStream_t s);
int minmax_device(const float* d_x, uint64_t n, float* mx, float* mn, bool* nan, hipStream_t s);
// K3 for n tracks packed in one buffer: rows [row0[i], row0[i+1]) of `bins` floats each.
int minmax_segments_device(const float* d_x, const uint64_t* row0, size_t bins, size_t n,
                           float* mx, float* mn, int* nan, hipStream_t s);
// K4-K6 for n tracks packed in one buffer, one stream, one sync: track i's [T_i, bins] dB rows
// -> grey [H_i, T_i] (H_i = round(bins * up_ratio[i])) -> Lanczos3 -> RGB at rgb_off[i].
// Several groups (each: one spectrogram buffer, its bin count, ns[k] tracks) in one call: the
// per-track arrays (up_ratio, nwidth, rgb_off; outputs mx/mn/nan) are concatenated in group
// order. One host->device table upload and one stream synchronisation per call.
int minmax_segments_multi(size_t n_groups, const float* const* d_x, const uint64_t* const* row0,
                          const size_t* bins, const size_t* ns, float* mx, float* mn, int* nan,
                          hipStream_t s);
int render_rgb_fused(size_t n_groups, const float* const* d_specs, const uint64_t* const* row0s,
                     const size_t* bins, const size_t* ns, const float* up_ratio,
                     const uint32_t* nwidth, uint32_t nheight, float max, float min, uint8_t* d_rgb,
                     const uint64_t* rgb_off, hipStream_t s, const float* d_grange = nullptr);
int inv_real_fft_device(const float* d_in, size_t n_frames, size_t length, float* d_out, hipStream_t s);
int render_rgb_batch_device(const float* d_spec, const uint64_t* row0, size_t bins, size_t n,
                            const float* up_ratio, const uint32_t* nwidth, uint32_t nheight,
                            float max, float min, uint8_t* d_rgb, const uint64_t* rgb_off,
                            hipStream_t s);

// sine LUT for the synthetic generator (host copy + lazily uploaded device copy)
const int16_t* synth_lut_host();

}  // namespace thesia
