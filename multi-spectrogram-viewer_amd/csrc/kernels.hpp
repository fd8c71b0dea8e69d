// kernels.hpp -- host-visible launch descriptors for the HIP kernels (no HIP types leak
// out of libthesia's C ABI; these structs are internal to the library).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace thesia {

enum OutKind : int {
    OUT_COMPLEX = 0,   // X[t, k] complex (perform_stft, lib.rs:388-471)
    OUT_MAG = 1,       // |X| (lib.rs:124)
    OUT_POWER = 2,     // |X|^2 (num-complex norm_sqr)
    OUT_AMP_DB = 3,    // amp_to_db_default(|X|) (lib.rs:127, decibel.rs:79-88)
    OUT_POWER_DB = 4,  // power_to_db_default(|X|^2) (decibel.rs:91-100)
    OUT_MEL = 5,       // |X| . mel_fb (lib.rs:131)
    OUT_MEL_AMP_DB = 6 // amp_to_db_default(|X| . mel_fb) (lib.rs:131-132)
};

enum InFormat : int {
    IN_F32 = 0,  // f32 samples, channel-interleaved (audio.rs:33-35 layout)
    IN_S16 = 1   // s16 PCM, channel-interleaved; value / 2^15 (audio.rs:16-19)
};

struct StftLaunch {
    // geometry
    int n_fft = 0, win = 0, hop = 0, pad_left = 0;
    int out_kind = OUT_AMP_DB;
    int in_format = IN_F32;
    int channels = 1;
    int fold = 0;  // apply the reference's channel-sum fold even for mono (AudioTrack::new)
    // input / tracks (device pointers)
    const void* in = nullptr;
    const uint64_t* trk_in_off = nullptr;  // element offset of each track's first sample
    const uint64_t* trk_len = nullptr;     // samples per channel
    const uint64_t* trk_frame0 = nullptr;  // [n_tracks + 1] prefix sum of frame counts
    int n_tracks = 0;
    uint64_t total_frames = 0;
    // tables (device pointers)
    const float* wpad = nullptr;     // [n_fft] window zero-padded to n_fft
    const float2* tw1 = nullptr;     // [NC] W_NC^m, m < NC (stage-1 twiddle bases)
    const float2* sincos = nullptr;  // [NC] realfft untangle table (sin, cos)
    const float2* tw2 = nullptr;     // stft2: [TB + TA][L] W_NC^{j*b}, W_NC^{j*TB*a} (lane-major)
    const float2* tw3 = nullptr;     // stft3: [P][L] W_NC^{j*k1} (lane-major)
    float log_amin = 0.f;            // log10f(amin), host-computed
    // mel (lib.rs:131): round r gives lane j of a frame mel r*L + j (L = lanes per frame);
    // the lane runs bins mel_k0[r*L + j] + it, it < mel_round[r].y, with weights
    // mel_wt[(mel_round[r].x + it) * L + j] (zero outside the filter's band)
    int n_mels = 0;
    int mel_rounds = 0;
    const int2* mel_round = nullptr;  // [rounds] {first weight row, band length}
    const int* mel_k0 = nullptr;      // [rounds][L]
    const float* mel_wt = nullptr;    // [sum of band lengths][L]
    // the same projection for stft2/stft3 (4 bins per step): lane j runs float4 steps
    // it < mel4_round[r].y from bin k0 = mel4_k0[r*L + j] & 0xFFFF (a multiple of 4) for mel
    // mel4_k0[r*L + j] >> 16 (0xFFFF: idle lane), weights mel4_wt[(mel4_round[r].x + it) * L + j]
    // (float4, zero outside the band); engine.cpp build_mel4 places filters on lanes bank-aware
    int mel4_rounds = 0;
    int mel4_rows = 0;  // float4 rows of mel4_wt (x L lanes)
    const int2* mel4_round = nullptr;
    const int* mel4_k0 = nullptr;
    const float4* mel4_wt = nullptr;
    // the same rounds as one stream of 4-step chunks (stft5's pipelined mel, mel4p): chunk c
    // reads weight rows 4c .. 4c+3 (the rounds' rows are contiguous) and, in lane j, the |X|
    // floats from mel_xo[c*L + j] & 0xFFFF; bits 16..30 hold the lane's mel, bit 31 marks the
    // last chunk of its round. 0 chunks when the plan does not fit (<= 8 chunks).
    int mel_chunks = 0;
    const int* mel_xo = nullptr;
    // stft5's packed mel stream (engine.cpp build_melp): every lane runs its own sequence of
    // whole filters, each padded to chunks of melp_steps float4 steps (lanes load-balanced, so
    // a frame runs melp_chunks chunks instead of the rounds' widest bands). Chunk c of lane j:
    // weights melp_wt[(c * melp_steps + u) * L + j], u < melp_steps; its |X| floats start at
    // byte xoff(c) of the stream's LDS region; after its fma chain the running sum is stored
    // at byte woff(c) of the region (the mel's slot behind the |X| row, kMelpOut, or a dummy
    // slot) and ANDed with keep(c) (0: the chunk ends a filter, the next starts from +0).
    // melp_meta[(c + 1) * L + j] = {woff(c), keep(c), xoff(c + 1), 0}, c = -1 .. melp_chunks - 1
    // (one zero chunk of padding at the end: the pipeline reads one chunk ahead).
    int melp_chunks = 0;
    int melp_steps = 0;
    int melp_v4 = 0;  // n_mels % 4 == 0 and 16-byte aligned rows: float4 row stores
    const int4* melp_meta = nullptr;
    const float4* melp_wt = nullptr;
    // the same packed stream built for 64 lanes per frame (stftr_kernel's one frame per wave)
    int melr_chunks = 0;
    int melr_steps = 0;
    const int4* melr_meta = nullptr;
    const float4* melr_wt = nullptr;
    // output
    void* out = nullptr;  // packed rows: frame g at out + g * row_elems
    // scheduling / named alternatives (thesia_batch_set_option)
    int grid = 0;     // 0 => computed from occupancy, else at most this many blocks
    float grid_share = 0.f;  // grid 0: this share of the occupancy wave (0 = all of it)
    // row-store method (stft3): 0 default (complex: whole 128-B lines; linear: LDS-
    // staged 16-byte), 1 the other one (complex: LDS-staged 16-byte; linear: lane-wise), 2 complex
    // whole lines, 3 complex lane-wise 8-byte; 1 and 3 at n_fft 2048 stereo f32 only
    int row_alt = 0;
    // the reference-order kernel (stftx_kernels.hip): input point m sits at xpos[m] of the
    // rustfft prepare_radix4 order; xw8 = {twiddle(1, 8), twiddle(3, 8)}; per mel m its nonzero
    // band {first bin, bins, offset into xmel_w}
    const int* xpos = nullptr;
    float xw8[4] = {0.f, 0.f, 0.f, 0.f};
    const int4* xmel_band = nullptr;
    const float* xmel_w = nullptr;
    // diagnostic builds only (-DTHESIA_STAMPS, scripts/stamps.py): per-wave phase cycle sums
    unsigned long long* stamps = nullptr;
    // per-track range of the output rows (update_spec_greys' max / min, lib.rs:194-207),
    // accumulated in the epilogue of the kernels that support it: 3 ints per track
    // {ordered max, ordered min, NaN seen} (range_ord below); null = off
    int* trk_range = nullptr;
};

// stft5 stream region (floats) and where the packed mel stream stages a frame's mels in it:
// behind the |X| row of F4 = 1028 floats; dummy slots follow the n_mels slots
constexpr int kStft5Region = 1184, kMelpOut = 1028, kMelpDummies = 16;

// f32 <-> int32 with the order of the floats (max / min by integer atomics); NaN excluded
__host__ __device__ inline int range_ord(float x) {
    const int b = __builtin_bit_cast(int, x);
    return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
__host__ __device__ inline float range_unord(int o) {
    return __builtin_bit_cast(float, o >= 0 ? o : o ^ 0x7FFFFFFF);
}
// trk_range slots set to {ord(-inf), ord(+inf), 0}
int launch_range_init(int* range, uint64_t n_tracks, hipStream_t s);
// the range of each track's rows [frame0[t] * row_floats, frame0[t+1] * row_floats) of `out`
// (for the kernels without the in-epilogue accumulation)
int launch_range_rows(const float* out, const uint64_t* d_frame0, uint64_t n_tracks, uint32_t row_floats,
                      int* range, hipStream_t s);

// Returns 0 on success, -2 for an unsupported n_fft.
int launch_stft(const StftLaunch& a, hipStream_t stream);
// stft2_kernel (n_fft 256..2048): 0 on success, -2 when n_fft is not one of its sizes.
int launch_stft2(const StftLaunch& a, hipStream_t stream);
bool stft2_supports(int n_fft);
int stft2_kernel_info(int n_fft, int* lds_bytes, int* tile_frames, int* lanes_per_frame);
// stft3_kernel (streaming; win = n_fft, hop = n_fft/4, f32 mono/stereo): 0 on success, -2 when
// the geometry is not its own (or the mel rows do not fit LDS).
int launch_stft3(const StftLaunch& a, hipStream_t stream);
bool stft3_supports(int n_fft, int win, int hop, int in_format, int channels);
int stft3_lds_bytes(const StftLaunch& a);  // dynamic LDS of the launch (> 163840: cannot run)
// the streaming kernel at the viewer geometries (stft3v_kernels.hip: win = 4 hop < n_fft, even
// hop; launch_stft3 / stft3_supports / stft3_lds_bytes dispatch to these)
int launch_stft3v(const StftLaunch& a, hipStream_t stream);
bool stft3v_supports(int n_fft, int win, int hop, int in_format, int channels);
int stft3v_lds_bytes(const StftLaunch& a);
// stftx_kernel (every n_fft: the reference's operation order, bit-exact with the oracle)
int launch_stftx(const StftLaunch& a, hipStream_t stream);
int stftx_lds_bytes(int n_fft, bool mel);
// InvRealFFT (realfft.rs:167-241) in the reference's operation order: n_frames spectra of
// length/2+1 complex (re, im interleaved) -> n_frames rows of `length` reals; tables of the
// length's Plan (xpos, forward twiddles, sin_cos, base butterfly_8 twiddles)
int launch_irfftx(const float* in, uint64_t n_frames, int length, const int* xpos, const float* tw1,
                  const float* sincos, const float* xw8, float* out, hipStream_t s);
// stft5_kernel (streaming, n_fft 2048 only, co-resident untangle pairs; stft5_kernels.hip)
int launch_stft5(const StftLaunch& a, hipStream_t stream);
bool stft5_supports(int n_fft, int win, int hop, int in_format, int channels);
int stft5_lds_bytes(const StftLaunch& a);
// stftr_kernel (streaming, reference operation order: rows equal the oracle's bit for bit;
// n_fft 2048, win = n_fft, hop = n_fft / 4; stftr_kernels.hip)
int launch_stftr(const StftLaunch& a, hipStream_t stream);
bool stftr_supports(int n_fft, int win, int hop, int in_format, int channels);
int stftr_lds_bytes(const StftLaunch& a);
constexpr int stftr_region_floats() { return 16 * 130; }  // GeoR::REGION
// stftq_kernel (the same contract for n_fft 256 / 512 / 1024, win = n_fft, hop = n_fft / 4;
// stftq_kernels.hip): batch kernel 7 at those sizes
int launch_stftq(const StftLaunch& a, hipStream_t stream);
bool stftq_supports(int n_fft, int win, int hop, int in_format, int channels);
int stftq_lds_bytes(const StftLaunch& a);
// LDS bytes / frames per block pass / lanes per frame of the kernel for n_fft.
int stft_kernel_info(int n_fft, int* lds_bytes, int* tile_frames, int* lanes_per_frame);

// ---- display / misc kernels (display_kernels.hip) ----
// WAV sample bytes (kind: wav.hpp PcmKind) -> f32 (hound, audio.rs:15-19) + channel sum (lib.rs:42)
int launch_decode_downmix(const void* raw, int kind, float scale, int channels, uint64_t n, float* out,
                          hipStream_t s);
int launch_downmix(const void* in, int in_format, int channels, uint64_t n, float* out,
                   hipStream_t s);
int launch_minmax(const float* x, uint64_t n, float* partial /*[2*nblk]*/, int* nan_flag,
                  int nblk, hipStream_t s);
int launch_minmax_seg(const float* x, const uint64_t* seg0, int n_seg, int nper, float* partial,
                      int* nan_flag, hipStream_t s);
// One track of a batched render (launch_render_batch): offsets in elements of the batch's
// spectrogram / grey / tmp buffers and bytes of the RGB buffer; the vertical (H -> nheight) and
// horizontal (T -> nw) Lanczos3 tap tables (device pointers, cached per geometry).
struct RenderDesc {
    uint64_t spec_off, grey_off, tmp_off, rgb_off;
    uint32_t T, H, nw;
    // oz: leading output rows whose vertical taps reach only the zero fill above the track's
    // band (display.rs:44-54). Their sums are +0 exactly (t = +0; t += 0 * w stays +0), so the
    // fused path neither forms nor reads them: colormap(+0) rows. 0 = no shortcut.
    uint32_t oz;
    uint32_t ts, pad_;  // row stride of the f32 intermediate (>= T; the fused path pads to 16)

    const int32_t *vl, *vc, *vo;
    const float* vw;
    const int32_t *hl, *hc, *ho;
    const float* hw;
    // the horizontal taps regrouped by 8-frame step (render_stripe_kernel, A slots): per step s
    // of the track its first column hst[s] (the columns whose supports meet frames [8s, 8s + 8)
    // are hst[s] ..), and hsw[(s * 8 + u) * A + a] = the weight of column hst[s] + a at frame
    // 8s + u (+0 outside its support)
    const int32_t* hst;
    const float* hsw;
    // the display's (max, min) dB on the device (thesia_ranges_global: the global range reduced
    // there, no host round trip), read by the grey stages in place of their max / min
    // arguments; null = the arguments
    const float* grange;
};
// the global (max, min) dB of n tracks' THESIA_BATCH_OPT_RANGE slots (lib.rs:194-209: NaN tracks
// skipped, max = min(max, 0), min = max(min, max - db_range), as thesia.shard.global_db_range) ->
// out[0], out[1] on the device; one block
int launch_range_global(const int* trk_range, uint32_t n, double db_range, float* out, hipStream_t s);
int launch_render_batch(const float* spec, uint32_t bins, float max, float min,
                        const RenderDesc* d_desc, uint32_t n, uint32_t T_max, uint32_t H_max,
                        uint32_t nw_max, uint32_t nh, int h_taps, int h_span, float* grey,
                        float* tmp, const uint8_t* cmap, uint8_t* rgb, hipStream_t s);
// The fused display path: grey + vertical Lanczos3 in one pass over the dB spectrogram (the
// grey image is never materialised), then the batched horizontal Lanczos3 + colormap. Same
// per-pixel arithmetic and summation order as launch_render_batch (bit-identical bytes).
// v_band: output rows per vertical block; v_rows: the largest grey-row span of such a band
// including the kv padding (its LDS tile); v_kv: taps per row padded to a multiple of 4.
int launch_render_batch2(const float* spec, uint32_t bins, float max, float min,
                         const RenderDesc* d_desc, uint32_t n, uint32_t T_max, uint32_t H_max,
                         uint32_t nw_max, uint32_t nh, int h_taps, int h_span, uint32_t v_band,
                         int v_rows, int v_kv, float* tmp, const uint8_t* cmap, uint8_t* rgb,
                         hipStream_t s, bool h_dma = true,  // h_dma: the LDS-DMA horizontal pass
                         int v_fpl = 1);  // frames per lane of the vertical pass (1, or 4: wide)
// The single-pass display (render_stripe_kernel, render_stripe.hip): grey + vertical Lanczos3 +
// horizontal Lanczos3 + colormap in one kernel, the f32 intermediate never leaving registers.
// A block owns `strip` output columns (a multiple of 16) x 64 `waves` output rows of one track,
// each wave 64 of the rows; its geometry bounds (host, plan_stripe): kv vertical taps (8, 12 or 16,
// zero-padded), at most `acc` columns meeting one 8-frame step (the accumulators: 8 .. 12 or 16),
// the step table's row stride `slots` (8, 12 or 16 >= acc), fc frames per staged chunk (8 or 16),
// npf staged values per lane and chunk (8 or 16), at most tile_cap grey rows per wave, hdr_cap
// steps and wts_cap step weights per strip. -2 when no instance fits.
struct StripeLaunch {
    const float* spec;
    uint32_t bins;
    float max, min;
    uint32_t nh;
    const RenderDesc* desc;
    uint32_t n;          // tracks (grid.z)
    uint32_t nw_max;
    uint32_t strip;      // output columns per block (multiple of 16)
    int kv, slots, acc, fc, npf;
    int waves;           // per block (4 or 8: 256 or 512 output rows)
    int tile_cap, hdr_cap, wts_cap;
    bool dword_rgb;      // every track's nw and rgb_off are multiples of 4 (dword RGB stores)
    const uint8_t* cmap;
    uint8_t* rgb;
    int abl;             // experiment build only (THESIA_STRIPE_ABL, timing ablations): 0
    // ring mode (hg > 0, render path 5): the lane's vertical sums of the strip's last `ring`
    // frames (a power of 2) in a per-lane LDS ring, each column summed over exactly its taps (hg
    // float4 groups, zero-padded) when its support has been formed; 0: the slot mode above
    int ring, hg;
};
int launch_render_stripe(const StripeLaunch& L, hipStream_t s);
// ring_slots: the ring mode's LDS frames per wave (ring + 4 hg + 1), 0 in slot mode
int render_stripe_lds_bytes(int fc, int tile_cap, int hdr_cap, int wts_cap, int waves, int ring_slots = 0);

// LDS bytes of the wide vertical pass (grey_vert_wide_kernel<fpl>) for a band / tile / kv
int grey_vert_wide_lds_bytes(int fpl, uint32_t band, int tile_cap, int kv);
int launch_spec_to_grey(const float* spec, uint32_t T, uint32_t bins, uint32_t H, float max,
                        float min, float* grey, hipStream_t s);
int launch_resize_v(const float* in, uint32_t w, uint32_t h, uint32_t nh, const int32_t* left,
                    const int32_t* cnt, const int32_t* woff, const float* wts, int max_taps,
                    float* out, hipStream_t s);
int launch_resize_h_rgb(const float* in, uint32_t w, uint32_t nh, uint32_t nw,
                        const int32_t* left, const int32_t* cnt, const int32_t* woff,
                        const float* wts, int max_taps, const uint8_t* cmap, uint8_t* out,
                        hipStream_t s);
int launch_wav_image(const float* wav, uint64_t n, const float* wav_up, uint64_t n_up,
                     uint32_t nwidth, uint32_t nheight, float spp, float amp_min, float amp_max,
                     uint8_t* out, int* panicked, hipStream_t s);
int launch_wav_upsample(const float* wav, uint64_t n, uint32_t factor, float* out,
                        hipStream_t s);
int launch_synth_pcm(void* out, int out_format, uint32_t channels, uint64_t n_tracks,
                     uint64_t n_samples, uint32_t sr, uint64_t seed, const int16_t* sine_lut,
                     hipStream_t s);
void synth_phase_coeffs(uint64_t n, uint32_t sr, uint64_t* ph_a, uint64_t* ph_b);
void synth_host(int16_t* out, uint32_t C, uint64_t track, uint64_t n, uint32_t sr, uint64_t seed,
                const int16_t* lut);

// probe_kernels.hip: read src once, write dst once (16-byte accesses, grid-stride)
int hbm_mix(const void* src, size_t src_bytes, void* dst, size_t dst_bytes, int grid, hipStream_t s);

}  // namespace thesia
