/*
 * thesia.h -- C ABI of libthesia, the MI355X-native spectrogram engine.
 *
 * Drop-in boundary for the reference's wasm-bindgen surface (src_rust/lib.rs:72-365,
 * 473-480) and its Rust-level pub API used by benches/bench.rs (perform_stft, decibel,
 * mel, windows, display). Every entry point cites the reference item it replaces.
 *
 * Conventions:
 *   - every function returns int status (THESIA_OK = 0) unless it cannot fail;
 *   - the reference panics (unwrap / assert) where this ABI returns an error code and sets
 *     a thread-local message readable with thesia_last_error(); nothing aborts across FFI;
 *   - outputs are caller-allocated; variable-size outputs take (out, cap, needed) and
 *     return THESIA_ERR_BUFFER_TOO_SMALL with *needed set when cap is short (out may be
 *     NULL for a size query);
 *   - a handle is not thread-safe (mirrors &mut self); distinct handles are independent;
 *   - "device" pointers are HBM pointers on the calling thread's current device
 *     (thesia_set_device); host pointers are plain process memory.
 */
#ifndef THESIA_H
#define THESIA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define THESIA_OK 0
#define THESIA_ERR_INVALID_ARG -1
#define THESIA_ERR_IO -2           /* add_tracks Err(io::Error) -> JsValue string, lib.rs:176 */
#define THESIA_ERR_UNKNOWN_ID -3   /* reference: unwrap() panic on a missing id, lib.rs:113,266,295 */
#define THESIA_ERR_TOO_SHORT -4    /* reference: slice panic for n < win-1, lib.rs:413 */
#define THESIA_ERR_UNSUPPORTED -5
#define THESIA_ERR_DEVICE -6
#define THESIA_ERR_BUFFER_TOO_SMALL -7
#define THESIA_ERR_NEGATIVE -8     /* reference: assert!(x >= 0) in log_for_db, decibel.rs:34 */
#define THESIA_ERR_PANIC -9        /* the reference panics for these arguments; the output is
                                      * still written (documented per function) */

const char* thesia_last_error(void);
const char* thesia_version(void);

/* ---------------------------------------------------------------------------------- */
/* runtime / device memory (plumbing for callers that keep data resident in HBM)       */
/* ---------------------------------------------------------------------------------- */
int thesia_device_count(int* n);
int thesia_set_device(int device);
int thesia_get_device(int* device);
int thesia_device_malloc(void** ptr, size_t bytes);
int thesia_device_free(void* ptr);
int thesia_memcpy_h2d(void* dst_device, const void* src_host, size_t bytes);
int thesia_memcpy_d2h(void* dst_host, const void* src_device, size_t bytes);
/* Page-lock (pin) a caller-owned host range so device-to-host copies into it run at DMA rate;
 * for the RGB image readback that get_spec_image implies (lib.rs:294-298 hands the bytes to JS).
 * The range stays the caller's; unregister it before freeing it. */
int thesia_host_register(void* host, size_t bytes);
int thesia_host_unregister(void* host);
int thesia_memset_device(void* dst_device, int value, size_t bytes);
int thesia_device_synchronize(void);
/* The library's block cache on the current device (round 5; the runtime's stream-ordered pool is
 * not used: on ROCm 7.2 it lost kernel writes into reused memory, profiles/r06_pool): device
 * buffers are hipMalloc blocks that, once released, stay with the library for its next
 * allocations of their size class, ordered behind their last use by an event (no device
 * synchronisation). thesia_pool_trim hands the idle blocks back to the device (it also runs in
 * thesia_mt_destroy, after MultiTrack compaction and before an allocation that ran out of memory
 * is retried); thesia_pool_bytes reports cached + in-use and in-use bytes (either may be NULL).
 * Plumbing, not part of the reference surface. */
int thesia_pool_trim(void);
int thesia_pool_bytes(uint64_t* reserved, uint64_t* used);
/* Device name / CU count of the current device (for reports). */
int thesia_device_info(char* name, size_t cap, int* n_cu);
/* HIP events for timing work on a stream (NULL stream => the library's stream of the current
 * device, where every thesia_* call without a stream argument runs). elapsed synchronises on
 * the second event. */
int thesia_event_create(void** event);
int thesia_event_destroy(void* event);
int thesia_event_record(void* event, void* stream);
int thesia_event_elapsed_ms(void* start, void* stop, float* ms);
/* The box's practical HBM ceiling for a read : write mix, on the caller's device buffers: every
 * 16 B of d_src read once and every 16 B of d_dst written once (coalesced float4, grid-stride;
 * d_dst's old contents are overwritten). Best of `reps` timed launches at two grid sizes on the
 * library stream (synchronous): *ms and the bytes moved per second in *gbps (may be NULL). A
 * measurement aid beside a kernel's roofline (bench.py); not part of the reference surface. */
int thesia_hbm_ceiling(const void* d_src, size_t src_bytes, void* d_dst, size_t dst_bytes, int reps,
                       float* ms, float* gbps);

/* ---------------------------------------------------------------------------------- */
/* host tables (bit-exact f32 restatements; computed with the same libm the reference  */
/* calls on Linux)                                                                     */
/* ---------------------------------------------------------------------------------- */
/* windows::hann(size, symmetric) -- windows.rs:21-30 */
int thesia_hann(size_t size, int symmetric, float* out);
/* utils::calc_proper_n_fft -- utils.rs:17-19 */
size_t thesia_calc_proper_n_fft(size_t win_length);
/* mel::hz_to_mel / mel_to_hz (f32) -- mel.rs:13-31 */
float thesia_hz_to_mel(float hz);
float thesia_mel_to_hz(float mel);
/* mel::calc_mel_fb(sr, n_fft, n_mel, fmin, fmax, do_norm) -- mel.rs:33-85.
 * fmax < 0 means None (Nyquist). out: [n_fft/2+1, n_mel] row-major f32. */
int thesia_calc_mel_fb(uint32_t sr, size_t n_fft, size_t n_mel, float fmin, float fmax,
                       int do_norm, float* out);
/* mel::calc_mel_fb_default(sr, n_fft) -- mel.rs:87-99. Writes n_mel; out may be NULL
 * (query) else needs (n_fft/2+1) * n_mel floats. */
int thesia_calc_mel_fb_default(uint32_t sr, size_t n_fft, size_t* n_mel, float* out,
                               size_t cap_floats);
/* get_colormap() -- lib.rs:473-480: the 10 inferno stops as 30 RGB bytes. */
void thesia_get_colormap(uint8_t out[30]);
/* AudioTrack::new parameter derivation -- lib.rs:43-46 */
int thesia_track_params(uint32_t sr, float win_ms, size_t t_overlap, size_t f_overlap,
                        size_t* win_length, size_t* hop_length, size_t* n_fft);

/* ---------------------------------------------------------------------------------- */
/* perform_stft -- lib.rs:388-471 (host buffers in / out; runs on the device)          */
/* ---------------------------------------------------------------------------------- */
/* Frame count the reference yields for (n, win, hop); 0 where it panics. */
size_t thesia_stft_n_frames(size_t n, size_t win_length, size_t hop_length);
/* X[T, n_fft/2+1] complex64 interleaved (re, im). window may be NULL (hann/n_fft,
 * lib.rs:407) else has win_length values (lib.rs:404 asserts the length). The `parallel`
 * flag of the reference changes nothing numerically and is not needed. */
int thesia_perform_stft(const float* input, size_t n, size_t win_length, size_t hop_length,
                        size_t n_fft, const float* window, float* out, size_t out_cap_frames,
                        size_t* n_frames);

/* ---------------------------------------------------------------------------------- */
/* batch engine: many tracks, one plan, one launch (the MI355X-native hot path)         */
/* ---------------------------------------------------------------------------------- */
typedef enum {
    THESIA_OUT_COMPLEX = 0,    /* perform_stft output, lib.rs:436 */
    THESIA_OUT_MAG = 1,        /* stft.mapv(|x| x.norm()), lib.rs:124 */
    THESIA_OUT_POWER = 2,      /* x.norm_sqr() */
    THESIA_OUT_AMP_DB = 3,     /* FreqScale::Linear: amp_to_db_default, lib.rs:126-129 */
    THESIA_OUT_POWER_DB = 4,   /* power_to_db_default(|X|^2), decibel.rs:91-100 */
    THESIA_OUT_MEL = 5,        /* linspec.dot(mel_fb), lib.rs:131 */
    THESIA_OUT_MEL_AMP_DB = 6  /* FreqScale::Mel: dot then amp_to_db_default, lib.rs:130-134 */
} thesia_output;

typedef enum {
    THESIA_IN_F32 = 0,  /* f32, channel-interleaved (audio.rs:33-35 [ch, n] view) */
    THESIA_IN_S16 = 1   /* s16 PCM, channel-interleaved, value / 32768 (audio.rs:16-19) */
} thesia_input_format;

typedef struct thesia_plan_desc {
    uint32_t sr;            /* sample rate (mel filterbank) */
    size_t win_length;
    size_t hop_length;
    size_t n_fft;           /* power of two, 2..4096 */
    const float* window;    /* NULL => hann(win, false) / n_fft (lib.rs:138-140) */
    int output;             /* thesia_output */
    size_t n_mels;          /* mel outputs: 0 => calc_mel_fb_default (mel.rs:87-99) */
    float fmin;             /* mel fmin (0) */
    float fmax;             /* mel fmax; < 0 => Nyquist */
    const float* mel_fb;    /* optional custom [n_fft/2+1, n_mels] filterbank (host) */
} thesia_plan_desc;

typedef struct thesia_plan thesia_plan;
int thesia_plan_create(const thesia_plan_desc* desc, thesia_plan** plan);
int thesia_plan_destroy(thesia_plan* plan);
/* Bins per output row: n_fft/2+1 (linear kinds) or n_mels (mel kinds). */
int thesia_plan_row_bins(const thesia_plan* plan, size_t* bins);

typedef struct thesia_batch_desc {
    int input_format;             /* thesia_input_format */
    uint32_t channels;            /* interleaved channels; summed (lib.rs:42) if > 1 */
    int fold_mono;                /* 1: apply the channel-sum fold for mono too (0.0 + x) */
    const void* d_input;          /* device base pointer */
    const uint64_t* track_offset; /* host [n_tracks]: element offset of each track */
    const uint64_t* track_len;    /* host [n_tracks]: samples per channel */
    size_t n_tracks;
    void* d_output;               /* device: rows packed track after track */
} thesia_batch_desc;

typedef struct thesia_batch thesia_batch;
/* Validates tracks (THESIA_ERR_TOO_SHORT for n < win-1) and uploads descriptors. */
int thesia_batch_create(thesia_plan* plan, const thesia_batch_desc* desc, thesia_batch** batch);
int thesia_batch_destroy(thesia_batch* batch);
/* Frame counts: total and per track (frame0 prefix, host array of n_tracks+1, may be NULL). */
int thesia_batch_frames(const thesia_batch* batch, uint64_t* total_frames, uint64_t* frame0);
/* Output bytes the batch writes (total_frames * row_bins * elem size). */
int thesia_batch_output_bytes(const thesia_batch* batch, uint64_t* bytes);
/* One pass of the hot path over the whole batch on `stream` (a hipStream_t; NULL => the
 * library's stream of the current device). Asynchronous. */
int thesia_batch_run(thesia_batch* batch, void* stream);
/* One pass of each of n batches (e.g. one per geometry group of a multi-rate track set), spread
 * over the library's internal streams of the current device and joined back to `stream` (NULL
 * => the library stream): the same results as n thesia_batch_run calls, with the launches
 * overlapping -- so the batches must share nothing they write: distinct handles
 * (THESIA_ERR_INVALID_ARG for a repeated one), output rows and range buffers that do not
 * overlap. Not part of the reference surface (its per-track loop is lib.rs:161-166).
 * Asynchronous. */
int thesia_batches_run(thesia_batch* const* batches, size_t n, void* stream);
/* Process-wide block-count policy of thesia_batches_run for batches whose block count is
 * automatic (THESIA_BATCH_OPT_MAX_BLOCKS 0): 0 (default) = each batch sized for the whole
 * device, as thesia_batch_run; 1 = the batches share one occupancy wave of the device in
 * proportion to their work (frames x n_fft log2 n_fft), so each frame stream walks more frames;
 * 2 = one after another on `stream`, each sized for the whole device (no fork). Same results
 * every way; 1 measured 1.6x slower on the C5 batches. */
int thesia_set_batches_policy(int policy);
/* Runs `iters` passes bracketed by HIP events on the launch stream; returns the elapsed
 * milliseconds of all passes (synchronous). */
int thesia_batch_run_timed(thesia_batch* batch, void* stream, int iters, float* ms);
/* Kernel geometry report for roofline accounting. */
int thesia_batch_kernel_info(const thesia_batch* batch, int* lds_bytes, int* tile_frames,
                             int* grid);

/* Which fused kernel runs the batch: 1 stft_kernel (general), 2 stft2_kernel (4 waves/SIMD),
 * 3 stft3_kernel (streaming; win = n_fft, hop = n_fft/4), 5 stft5_kernel (streaming, n_fft 2048:
 * untangle pairs co-resident in a lane), 7 the streaming reference-order kernels (stftr_kernel at
 * n_fft 2048, stftq_kernel at 256 / 512 / 1024; win = n_fft, hop = n_fft/4 with f32 / s16 input,
 * or any even win <= n_fft and any hop with f32 input -- the viewer's geometries, lib.rs:43-46:
 * rows equal the reference's bit for bit), 9 stftx_kernel (the reference's operation order, any
 * geometry). At win < n_fft, 7 and 9 read no sample in a frame's centring pads (lib.rs:377-385),
 * so a non-finite sample there leaves the frame finite, as in the reference; the tolerance
 * kernels (1-5) multiply the pads by the zero-padded window, and such a frame comes out
 * non-finite. */
int thesia_batch_kernel(const thesia_batch* batch, int* kernel);

/* Named alternatives of a batch (none changes what is computed, only how; all results stay
 * within the parity contract). Not part of the reference surface. */
typedef enum {
    /* 0 = automatic (streaming kernel where its geometry allows), 1 / 2 / 3 / 5 / 7 / 9 = force
     * that kernel (THESIA_ERR_UNSUPPORTED if it cannot run the geometry); 7 and 9 compute in
     * the reference's operation order (bit-exact rows) */
    THESIA_BATCH_OPT_KERNEL = 1,
    /* at most this many workgroups per launch (0 = one full occupancy wave of the device);
     * small values make every frame stream walk many frames */
    THESIA_BATCH_OPT_MAX_BLOCKS = 2,
    /* output-row store method of the streaming kernel stft3 (identical bytes):
     * 0 = default (complex rows as whole 128-byte lines, the line two rows share carried from
     * frame to frame; linear rows LDS-staged 16-byte stores), 1 = the other method (LDS-staged
     * 16-byte for complex / lane-wise for linear rows), 2 = complex whole lines, 3 = complex
     * lane-wise 8-byte stores (2 and 3: complex rows only, THESIA_ERR_INVALID_ARG otherwise);
     * 1 and 3 at n_fft 2048 stereo f32 only */
    THESIA_BATCH_OPT_ROW_STORE = 3,
    /* a device buffer of 3 int32 per track (value = its address, 0 = off): every run also
     * leaves each track's max / min over its output rows and a NaN flag there (the per-track
     * reduction of update_spec_greys, lib.rs:194-207), folded into the streaming kernel's row
     * epilogue (stft3: the linear kinds; kernel 7: amp dB), else one pass over the rows; read with
     * thesia_batch_ranges_read. Real output kinds only. */
    THESIA_BATCH_OPT_RANGE = 4,
    /* mel projection of stft5_kernel (the mel kinds at n_fft 2048): 0 = automatic, 1 = the
     * filter rounds as one chunk stream, 2 / 3 = the packed stream (filters dealt to lanes by
     * load) with 2 / 3 float4 steps per chunk. Every path is the same k-ascending fma chain
     * per mel (identical bits). */
    THESIA_BATCH_OPT_MEL_PATH = 5
} thesia_batch_option;
int thesia_batch_set_option(thesia_batch* batch, int option, int64_t value);
/* Decode n tracks' range slots (THESIA_BATCH_OPT_RANGE buffer, device) after the runs that
 * wrote them: max / min per track (ndarray-stats: -inf / +inf for an empty track), has_nan. */
int thesia_batch_ranges_read(const void* d_range, size_t n, float* max, float* min, int* has_nan);

/* Deterministic synthetic PCM (int16-quantised chirp + noise) written on the device, and
 * its bit-identical host twin. format: thesia_input_format. Layout [track][sample][ch]. */
int thesia_synth_pcm_device(void* d_out, int format, uint32_t channels, uint64_t n_tracks,
                            uint64_t n_samples, uint32_t sr, uint64_t seed);
int thesia_synth_pcm_host(int16_t* out, uint32_t channels, uint64_t track, uint64_t n_samples,
                          uint32_t sr, uint64_t seed);

/* ---------------------------------------------------------------------------------- */
/* display primitives on the device (host buffers in / out) -- display.rs               */
/* ---------------------------------------------------------------------------------- */
/* spec_to_grey -- display.rs:44-54. spec [T, bins]; grey [H, T], H = round(bins*up_ratio). */
int thesia_spec_grey_height(size_t bins, float up_ratio, uint32_t* height);
int thesia_spec_to_grey(const float* spec, size_t T, size_t bins, float up_ratio, float max,
                        float min, float* grey, size_t cap_floats);
/* grey_to_rgb -- display.rs:56-61 (Lanczos3 resize + colormap). out [nh, nw, 3]. */
int thesia_grey_to_rgb(const float* grey, uint32_t width, uint32_t height, uint32_t nwidth,
                       uint32_t nheight, uint8_t* out, size_t cap);
/* InvRealFFT -- realfft.rs:167-241 (InvRealFFT::new(length) + process per frame): n_frames
 * spectra of length/2+1 complex values (re, im interleaved f32) -> n_frames rows of `length`
 * reals, unnormalised (0.5 * Re of the full inverse DFT, the reference's complex_to_real test),
 * in the reference's operation order (rustfft 4.0 Radix4, inverse). length even
 * (THESIA_ERR_INVALID_ARG otherwise, "Length must be even") and a power of two <= 4096
 * (THESIA_ERR_UNSUPPORTED: Radix4 panics on other sizes). _device: HBM buffers, stream-ordered. */
int thesia_inv_real_fft_device(const float* d_in, size_t n_frames, size_t length, float* d_out);
int thesia_inv_real_fft(const float* in, size_t n_frames, size_t length, float* out);
/* wav_to_image -- display.rs:63-115. out [nheight, nwidth, 4] RGBA. THESIA_ERR_PANIC where
 * the reference panics (a pixel's sample slice empty or holding NaN, or a column reaching row
 * nheight, display.rs:95-108); the image is written anyway, such columns clamped / left blank. */
int thesia_wav_to_image(const float* wav, size_t n, uint32_t nwidth, uint32_t nheight,
                        float amp_min, float amp_max, uint8_t* out, size_t cap);

/* Device-resident display (HBM pointers on the current device; synchronous). Used by the
 * batched render pipeline (thesia/pipeline.py) where spectrograms never leave HBM. */
/* max / min of n f32 values (lib.rs:194-207 per track; NaN -> *has_nan, like the
 * ndarray-stats error the reference maps to -inf / +inf). n == 0 gives -inf / +inf. */
int thesia_minmax_device(const float* d_x, uint64_t n, float* max, float* min, int* has_nan);
/* spec_to_grey on HBM buffers -- display.rs:44-54. d_grey holds H * T floats
 * (thesia_spec_grey_height). */
int thesia_spec_to_grey_device(const float* d_spec, size_t T, size_t bins, float up_ratio,
                               float max, float min, float* d_grey);
/* grey_to_rgb on HBM buffers -- display.rs:56-61. d_rgb holds nh * nw * 3 bytes. */
int thesia_grey_to_rgb_device(const float* d_grey, uint32_t width, uint32_t height,
                              uint32_t nwidth, uint32_t nheight, uint8_t* d_rgb);

/* Batched display for n tracks whose dB spectrograms are packed in one HBM buffer (rows
 * [row0[i], row0[i+1]) of `bins` floats; row0 is a host array of n+1 entries) -- the
 * per-track max/min of update_spec_greys (lib.rs:194-207) in one launch, and grey + Lanczos3
 * + colormap for every track in one stream pass (lib.rs:249-260, 294-298): track i's RGB image
 * [nheight, nwidth[i], 3] lands at d_rgb + rgb_off[i] (host arrays of n entries). */
int thesia_minmax_segments_device(const float* d_spec, const uint64_t* row0, size_t bins,
                                  size_t n, float* max, float* min, int* has_nan);
/* Process-wide choice of the batched display path's launch structure (all byte-identical):
 * 0 = the fused path (default): per geometry group, where the group downsamples along time at
 * least 3:1 (frames >= 3 x image columns) and its geometry allows (at most 16 vertical taps and
 * 16 output columns meeting one 8-frame step), ONE kernel for grey + vertical Lanczos3 +
 * horizontal Lanczos3 + colormap whose f32 intermediate never leaves registers
 * (render_stripe_kernel); for the other groups one kernel for grey + vertical Lanczos3 in one
 * pass over the spectrogram, then one for horizontal Lanczos3 + colormap (row spans staged by
 * LDS-DMA); every track of a call in each launch; 1 = per-track launches (the reference's one
 * image at a time structure); 2 = every track in one launch per stage: grey, vertical,
 * horizontal + colormap; 3 = path 0 with the two-kernel structure for every group (round 3's
 * default); 4 = path 0 with the single-pass kernel wherever its geometry allows. */
int thesia_set_render_path(int path);
/* The render path in effect (the value thesia_set_render_path last stored, 0 by default). */
int thesia_get_render_path(void);
int thesia_render_rgb_batch_device(const float* d_spec, const uint64_t* row0, size_t bins,
                                   size_t n, const float* up_ratio, const uint32_t* nwidth,
                                   uint32_t nheight, float max, float min, uint8_t* d_rgb,
                                   const uint64_t* rgb_off);

/* The _device display entries are stream-ordered on the library stream: they return once
 * their launches are enqueued, and every later library call (thesia_memcpy_d2h included) sees
 * their results. thesia_memcpy_h2d / _d2h are blocking and ordered after all enqueued work. */
/* Several geometry groups in one call (group k: spectrogram buffer d_specs[k] of bins[k]
 * floats per row, ns[k] tracks with row table row0s[k] of ns[k]+1 entries); the per-track
 * arrays (max/min/has_nan out; up_ratio, nwidth, rgb_off in) are concatenated in group order.
 * Same results as one single-group call per group, with one table upload and one stream
 * synchronisation for the whole call instead of one per group. */
int thesia_minmax_segments_multi(size_t n_groups, const float* const* d_specs,
                                 const uint64_t* const* row0s, const size_t* bins, const size_t* ns,
                                 float* max, float* min, int* has_nan);
/* render_rgb_multi runs its groups concurrently on the library's stream pool (largest first;
 * THESIA_RENDER_STREAMS=1 in the environment keeps them serial), still stream-ordered on the
 * library stream as a whole: the tracks' RGB ranges (rgb_off, nwidth x nheight x 3 bytes) must
 * not overlap, as two tracks writing the same bytes would race. */
int thesia_render_rgb_multi(size_t n_groups, const float* const* d_specs, const uint64_t* const* row0s,
                            const size_t* bins, const size_t* ns, const float* up_ratio,
                            const uint32_t* nwidth, uint32_t nheight, float max, float min,
                            uint8_t* d_rgb, const uint64_t* rgb_off);
/* The display's global range without a host round trip (single-device callers): the global
 * (max, min) dB over n tracks' THESIA_BATCH_OPT_RANGE slots d_trk_range (3 ints per track, as
 * the batches leave them), as lib.rs:194-209 computes it -- NaN-holding tracks skipped, max =
 * min(max, 0), min = max(min, max - db_range) -- written to d_out[0], d_out[1] (device floats)
 * by one kernel on the library stream. Asynchronous. Multi-device callers exchange the per-rank
 * ranges on the host instead (thesia.shard.global_db_range). */
int thesia_ranges_global(const int* d_trk_range, size_t n, float db_range, float* d_out);
/* thesia_render_rgb_multi with the (max, min) read from the device (d_range[0], d_range[1], e.g.
 * thesia_ranges_global's output) when the kernels run: the whole step -- batches, range, display
 * -- enqueues without a host synchronisation. Render paths 0, 3, 4 (THESIA_ERR_UNSUPPORTED
 * otherwise). Same bytes as thesia_render_rgb_multi with those values. */
int thesia_render_rgb_multi_dev(size_t n_groups, const float* const* d_specs, const uint64_t* const* row0s,
                                const size_t* bins, const size_t* ns, const float* up_ratio,
                                const uint32_t* nwidth, uint32_t nheight, const float* d_range,
                                uint8_t* d_rgb, const uint64_t* rgb_off);

/* ---------------------------------------------------------------------------------- */
/* MultiTrack -- lib.rs:72-365 (the viewer's stateful surface)                          */
/* ---------------------------------------------------------------------------------- */
typedef struct thesia_mt thesia_mt;
/* MultiTrack::new -- lib.rs:89-110 (win_ms 40, t_overlap 4, f_overlap 1, Mel, 120 dB) */
int thesia_mt_create(thesia_mt** mt);
void thesia_mt_destroy(thesia_mt* mt);
/* SpecSetting (lib.rs:64-70) has no setter in the reference; exposed for Linear-scale use.
 * freq_scale: 0 = Linear, 1 = Mel. Must be called before any track is added. */
int thesia_mt_set_setting(thesia_mt* mt, float win_ms, size_t t_overlap, size_t f_overlap,
                          int freq_scale, float db_range);
/* Spectrogram kernel of the tracks added from now on (not part of the reference surface):
 * 0 (default) = the reference-order kernel, whose images equal the oracle pipeline's bytes;
 * 1 = the batch engine's streaming kernel for the viewer's geometry (3.3x faster behind
 * add_tracks), held to SURVEY.md §8c's end-to-end contract: at most 1 LSB on at
 * most 1e-4 of the pixels. */
int thesia_mt_set_fast(thesia_mt* mt, int fast);
/* add_tracks(id_list, path_list) -> Result<bool, JsValue> -- lib.rs:170-191.
 * paths are '\n'-separated; *changed = "global dB range / max sr changed: refetch all
 * images". On error nothing is added (the reference would leave a half-added state).
 * The files are read concurrently into a page-locked host buffer the handle keeps between calls
 * (about 1.25x the call's total file size, at most 256 MiB; a call whose files exceed that reads
 * into a page-locked buffer of its own, freed when the call returns; thesia_mt_destroy frees it). */
int thesia_mt_add_tracks(thesia_mt* mt, const uint64_t* ids, size_t n_ids, const char* paths,
                         int* changed);
/* WAV files keep their sample encoding up to the device: 8/16/24/32-bit integer or f32 samples
 * are uploaded as stored (1-4 B per sample) and converted ((x as f32) / 2^(bits-1), 8-bit
 * unsigned; audio.rs:15-19) and downmixed (lib.rs:42) there. All new tracks of one sample rate
 * run as one batched spectrogram launch; the call synchronises once. */
/* Same, from in-memory interleaved f32 PCM (what open_audio_file returns, audio.rs:9-37). */
int thesia_mt_add_tracks_pcm(thesia_mt* mt, const uint64_t* ids, size_t n_ids,
                             const float* const* pcm, const uint64_t* n_samples,
                             const uint32_t* channels, const uint32_t* sr, const char* paths,
                             int* changed);
/* remove_track(id) -> bool -- lib.rs:265-292 */
int thesia_mt_remove_track(thesia_mt* mt, uint64_t id, int* changed);
/* get_spec_image(id, px_per_sec, nheight) -> Vec<u8> RGB -- lib.rs:294-298 */
int thesia_mt_get_spec_image(thesia_mt* mt, uint64_t id, float px_per_sec, uint32_t nheight,
                             uint8_t* out, size_t cap, size_t* needed);
/* get_wav_image(id, px_per_sec, nheight, amp_min, amp_max) -> Vec<u8> RGBA -- lib.rs:300-313
 * (THESIA_ERR_PANIC as thesia_wav_to_image, image written) */
int thesia_mt_get_wav_image(thesia_mt* mt, uint64_t id, float px_per_sec, uint32_t nheight,
                            float amp_min, float amp_max, uint8_t* out, size_t cap,
                            size_t* needed);
/* get_frequency_hz(id, relative_freq) -- lib.rs:315-322 */
int thesia_mt_get_frequency_hz(thesia_mt* mt, uint64_t id, float relative_freq, float* hz);
/* getters -- lib.rs:324-364 */
float thesia_mt_get_max_db(const thesia_mt* mt);
float thesia_mt_get_min_db(const thesia_mt* mt);
float thesia_mt_get_max_sec(const thesia_mt* mt);
int thesia_mt_get_sec(const thesia_mt* mt, uint64_t id, float* sec);
int thesia_mt_get_sr(const thesia_mt* mt, uint64_t id, uint32_t* sr);
int thesia_mt_get_path(const thesia_mt* mt, uint64_t id, char* out, size_t cap, size_t* needed);
int thesia_mt_get_filename(const thesia_mt* mt, uint64_t id, char* out, size_t cap,
                           size_t* needed);
/* Introspection for parity tests (not in the reference surface): the dB spectrogram
 * [T, bins] (lib.rs:112-136 calc_spec_of) and the grey image [H, T] (lib.rs:249-260). */
int thesia_mt_get_spec(const thesia_mt* mt, uint64_t id, float* out, size_t cap_floats,
                       size_t* n_frames, size_t* n_bins);
int thesia_mt_get_grey(const thesia_mt* mt, uint64_t id, float* out, size_t cap_floats,
                       uint32_t* width, uint32_t* height);
int thesia_mt_track_count(const thesia_mt* mt, size_t* n);
/* Device bytes the tracks hold (wav + spectrogram buffers, each shared buffer once, + greys).
 * Tracks added by one call share buffers; removals that leave a buffer at most half used move its
 * survivors into their own buffers and free it (the reference frees per track, lib.rs:265-292). */
int thesia_mt_device_bytes(const thesia_mt* mt, size_t* bytes);
/* the track's mono wav (audio.rs:9-37 decode + lib.rs:42 channel sum) as held on the device */
int thesia_mt_get_wav(const thesia_mt* mt, uint64_t id, float* out, size_t cap_floats,
                      size_t* n_samples);

/* open_audio_file (audio.rs:9-37) on the host, WAV only (hound semantics; the rodio fallback
 * for FLAC / Vorbis returns THESIA_ERR_UNSUPPORTED): interleaved f32 samples [n][channels].
 * out may be NULL to query *n_floats. */
int thesia_open_audio_file(const char* path, float* out, size_t cap_floats, size_t* n_floats,
                           uint32_t* sr, uint32_t* channels);

#ifdef __cplusplus
}
#endif
#endif /* THESIA_H */
