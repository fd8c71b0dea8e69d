// display_kernels.hip -- the display half of the path (display.rs) and small helpers.
//
//   K3 minmax        : per-track max/min of a dB spectrogram (lib.rs:194-207; ndarray-stats
//                      max/min error -> (-inf, +inf) on NaN)
//   K4 spec_to_grey  : transpose + vertical flip + normalise + zero top fill (display.rs:44-54)
//   K5 resize        : separable Lanczos3 (image 0.23.12 resize: vertical pass into an f32
//                      image, then horizontal), weights from the host (same f32 formulas)
//   K6 colormap      : fused into the horizontal pass epilogue (display.rs:24-42, 56-61)
//   wav image        : min/max envelope raster in WAVECOLOR (display.rs:63-115)
//   downmix          : channel sum in ndarray's unrolled_fold order (lib.rs:42)
//   synth            : deterministic integer PCM generator for benches / tests
// All accumulations run in the reference's order with -ffp-contract=off, so given the
// same f32 input these kernels reproduce the oracle bit for bit.
#include "kernels.hpp"
#include "display_common.hpp"

#include <cmath>
#include <cstdlib>
#include <cstdint>

// compile-time choices A/B'd with scripts/build_variant.sh (defaults = the product)
#ifndef THESIA_V_ABL
#define THESIA_V_ABL 0
#endif
#ifndef THESIA_VDEPTH
#define THESIA_VDEPTH 8  // grey_vert: tile loads in flight per thread
#endif
#ifndef THESIA_RYH
#define THESIA_RYH 16  // horizontal pass: row blocks per image
#endif
#ifndef THESIA_HKT_MAX
#define THESIA_HKT_MAX 48  // horizontal pass: most taps held in registers
#endif
#ifndef THESIA_H_ABL
#define THESIA_H_ABL 0
#endif
#ifndef THESIA_H_DIRECT
#define THESIA_H_DIRECT 1  // horizontal pass: RGB bytes stored lane by lane (no LDS assembly)
#endif
#ifndef THESIA_H_2ROW
#define THESIA_H_2ROW 1  // horizontal pass: two rows per block step
#endif

namespace thesia {

// ------------------------------------------------------------------------------------
// downmix (lib.rs:42 sum_axis over channels -> unrolled_fold)
// ------------------------------------------------------------------------------------
template <int INF>
__device__ __forceinline__ float chan_at(const void* in, uint64_t idx) {
    if constexpr (INF == IN_S16) return (float)static_cast<const int16_t*>(in)[idx] / 32768.0f;
    else return static_cast<const float*>(in)[idx];
}

template <int INF>
__global__ void downmix_kernel(const void* in, int C, uint64_t n, float* out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = i * (uint64_t)C;
        float acc = 0.0f;
        if (C < 8) {
            for (int c = 0; c < C; ++c) acc = acc + chan_at<INF>(in, p + c);
        } else {
            float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            int c = 0;
            for (; C - c >= 8; c += 8)
                for (int u = 0; u < 8; ++u) q[u] = q[u] + chan_at<INF>(in, p + c + u);
            acc = acc + (q[0] + q[4]);
            acc = acc + (q[1] + q[5]);
            acc = acc + (q[2] + q[6]);
            acc = acc + (q[3] + q[7]);
            for (; c < C; ++c) acc = acc + chan_at<INF>(in, p + c);
        }
        out[i] = acc;
    }
}

int launch_downmix(const void* in, int in_format, int channels, uint64_t n, float* out,
                   hipStream_t s) {
    if (n == 0) return 0;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (in_format == IN_S16)
        hipLaunchKernelGGL(downmix_kernel<IN_S16>, dim3((unsigned)blocks), dim3(256), 0, s, in, channels, n, out);
    else
        hipLaunchKernelGGL(downmix_kernel<IN_F32>, dim3((unsigned)blocks), dim3(256), 0, s, in, channels, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// WAV ingest (audio.rs:9-37 + lib.rs:42): the file's sample bytes -> f32 by hound's rule
// ((x as f32) / 2^(bits-1), 8-bit unsigned x - 128, float as is), then the channel sum in the
// order of downmix_kernel. kind: PCM_F32 0, PCM_U8 1, PCM_S16 2, PCM_S24 3, PCM_S32 4 (wav.hpp).
template <int KIND>
__device__ __forceinline__ float pcm_at(const uint8_t* raw, float scale, uint64_t i) {
    if constexpr (KIND == 0) {
        return reinterpret_cast<const float*>(raw)[i];
    } else if constexpr (KIND == 1) {
        return (float)((int32_t)raw[i] - 128) / scale;
    } else if constexpr (KIND == 2) {
        return (float)reinterpret_cast<const int16_t*>(raw)[i] / scale;
    } else if constexpr (KIND == 3) {
        const uint8_t* p = raw + 3 * i;
        const int32_t v = (int32_t)((uint32_t)p[0] << 8 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 24) >> 8;
        return (float)v / scale;
    } else {
        return (float)reinterpret_cast<const int32_t*>(raw)[i] / scale;
    }
}

template <int KIND>
__global__ void decode_downmix_kernel(const uint8_t* raw, float scale, int C, uint64_t n, float* out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = i * (uint64_t)C;
        float acc = 0.0f;
        if (C < 8) {
            for (int c = 0; c < C; ++c) acc = acc + pcm_at<KIND>(raw, scale, p + c);
        } else {
            float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            int c = 0;
            for (; C - c >= 8; c += 8)
                for (int u = 0; u < 8; ++u) q[u] = q[u] + pcm_at<KIND>(raw, scale, p + c + u);
            acc = acc + (q[0] + q[4]);
            acc = acc + (q[1] + q[5]);
            acc = acc + (q[2] + q[6]);
            acc = acc + (q[3] + q[7]);
            for (; c < C; ++c) acc = acc + pcm_at<KIND>(raw, scale, p + c);
        }
        out[i] = acc;
    }
}

int launch_decode_downmix(const void* raw, int kind, float scale, int channels, uint64_t n, float* out,
                          hipStream_t s) {
    if (n == 0) return 0;
    if (kind < 0 || kind > 4 || channels <= 0) return -2;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    const uint8_t* r = static_cast<const uint8_t*>(raw);
    const dim3 g((unsigned)blocks), b(256);
    switch (kind) {
        case 0: hipLaunchKernelGGL(decode_downmix_kernel<0>, g, b, 0, s, r, scale, channels, n, out); break;
        case 1: hipLaunchKernelGGL(decode_downmix_kernel<1>, g, b, 0, s, r, scale, channels, n, out); break;
        case 2: hipLaunchKernelGGL(decode_downmix_kernel<2>, g, b, 0, s, r, scale, channels, n, out); break;
        case 3: hipLaunchKernelGGL(decode_downmix_kernel<3>, g, b, 0, s, r, scale, channels, n, out); break;
        default: hipLaunchKernelGGL(decode_downmix_kernel<4>, g, b, 0, s, r, scale, channels, n, out); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// per-track output ranges for Batch::range (the kernels without the in-epilogue accumulation)
__global__ void range_init_kernel(int* r, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) {
        r[3 * i] = range_ord(-INFINITY);
        r[3 * i + 1] = range_ord(INFINITY);
        r[3 * i + 2] = 0;
    }
}

int launch_range_init(int* range, uint64_t n_tracks, hipStream_t s) {
    if (n_tracks == 0) return 0;
    hipLaunchKernelGGL(range_init_kernel, dim3((unsigned)((n_tracks + 255) / 256)), dim3(256), 0, s, range,
                       n_tracks);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void __launch_bounds__(256) range_rows_kernel(const float* out, const uint64_t* frame0,
                                                         uint32_t row_floats, int* range) {
    const uint64_t t = blockIdx.y;
    const uint64_t beg = frame0[t] * row_floats, end = frame0[t + 1] * row_floats;
    float mx = -INFINITY, mn = INFINITY;
    int nan = 0;
    for (uint64_t i = beg + blockIdx.x * 256ull + threadIdx.x; i < end; i += gridDim.x * 256ull) {
        const float v = out[i];
        mx = fmaxf(mx, v);
        mn = fminf(mn, v);
        nan |= v != v;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, m));
        mn = fminf(mn, __shfl_xor(mn, m));
        nan |= __shfl_xor(nan, m);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(range + 3 * t, range_ord(mx));
        atomicMin(range + 3 * t + 1, range_ord(mn));
        if (nan) atomicOr(range + 3 * t + 2, 1);
    }
}

int launch_range_rows(const float* out, const uint64_t* d_frame0, uint64_t n_tracks, uint32_t row_floats,
                      int* range, hipStream_t s) {
    if (n_tracks == 0) return 0;
    if (n_tracks > 65535) return -2;
    hipLaunchKernelGGL(range_rows_kernel, dim3(32, (unsigned)n_tracks), dim3(256), 0, s, out, d_frame0,
                       row_floats, range);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// K3 per-track max/min (NaN -> flag)
// ------------------------------------------------------------------------------------
__global__ void minmax_kernel(const float* x, uint64_t n, float* partial, int* nan_flag) {
    float mx = -INFINITY, mn = INFINITY;
    int nan = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const float v = x[i];
        if (v != v) nan = 1;
        mx = fmaxf(mx, v);
        mn = fminf(mn, v);
    }
    __shared__ float smx[256], smn[256];
    __shared__ int snan;
    if (threadIdx.x == 0) snan = 0;
    __syncthreads();
    smx[threadIdx.x] = mx;
    smn[threadIdx.x] = mn;
    if (nan) snan = 1;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) {
            smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + st]);
            smn[threadIdx.x] = fminf(smn[threadIdx.x], smn[threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = smx[0];
        partial[2 * blockIdx.x + 1] = smn[0];
        if (snan) atomicOr(nan_flag, 1);
    }
}

int launch_minmax(const float* x, uint64_t n, float* partial, int* nan_flag, int nblk,
                  hipStream_t s) {
    hipLaunchKernelGGL(minmax_kernel, dim3(nblk), dim3(256), 0, s, x, n, partial, nan_flag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// K3 over many tracks at once: segment s = elements [seg0[s], seg0[s+1]) of x; blockIdx.y is
// the segment, blockIdx.x one of nper blocks striding through it. 16-byte loads in the body
// (the scalar head up to 16-byte alignment and the tail are read lane-wise), four independent
// running max/min pairs per lane, a wave-level shuffle reduction.
__device__ __forceinline__ void mm_acc(float v, float& mx, float& mn, int& nan) {
    if (v != v) nan = 1;
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
}
__global__ void __launch_bounds__(256) minmax_seg_kernel(const float* x, const uint64_t* seg0, int nper,
                                                         float* partial, int* nan_flag) {
    // segment i: elements [seg0[2i], seg0[2i+1]) of x
    const int seg = blockIdx.y;
    const uint64_t beg = seg0[2 * seg], end = seg0[2 * seg + 1];
    float mx0 = -INFINITY, mn0 = INFINITY, mx1 = -INFINITY, mn1 = INFINITY;
    int nan = 0;
    const uint64_t n = end - beg;
    const float* p = x + beg;
    uint64_t head = (uint64_t)((4 - ((reinterpret_cast<uintptr_t>(p) >> 2) & 3)) & 3);
    head = head < n ? head : n;
    const uint64_t n4 = (n - head) / 4;
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, stride = (uint64_t)nper * blockDim.x;
    if (tid < head) mm_acc(p[tid], mx0, mn0, nan);
    const float4* p4 = reinterpret_cast<const float4*>(p + head);
    for (uint64_t i = tid; i < n4; i += stride) {
        const float4 v = p4[i];
        mm_acc(v.x, mx0, mn0, nan);
        mm_acc(v.y, mx1, mn1, nan);
        mm_acc(v.z, mx0, mn0, nan);
        mm_acc(v.w, mx1, mn1, nan);
    }
    for (uint64_t i = head + 4 * n4 + tid; i < n; i += stride) mm_acc(p[i], mx0, mn0, nan);
    float mx = fmaxf(mx0, mx1), mn = fminf(mn0, mn1);
    for (int o = 32; o > 0; o >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        mn = fminf(mn, __shfl_xor(mn, o, 64));
    }
    nan = __any(nan) ? 1 : 0;
    __shared__ float smx[4], smn[4];
    __shared__ int snan[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { smx[wave] = mx; smn[wave] = mn; snan[wave] = nan; }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t o = ((uint64_t)seg * nper + blockIdx.x) * 2;
        partial[o] = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
        partial[o + 1] = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
        if (snan[0] | snan[1] | snan[2] | snan[3]) atomicOr(nan_flag + seg, 1);
    }
}

int launch_minmax_seg(const float* x, const uint64_t* seg0, int n_seg, int nper, float* partial,
                      int* nan_flag, hipStream_t s) {
    if (n_seg == 0) return 0;
    hipLaunchKernelGGL(minmax_seg_kernel, dim3(nper, n_seg), dim3(256), 0, s, x, seg0, nper,
                       partial, nan_flag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// K4 spec_to_grey (display.rs:44-54): grey[y][x], y < H, x < T
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void grey_px(const float* spec, uint32_t T, uint32_t bins, uint32_t H,
                                        float max, float min, float* grey, uint32_t x, uint32_t y) {
    float v = 0.0f;
    if (y >= H - bins) {
        const float db = spec[(uint64_t)x * bins + (H - 1 - y)];
        v = (db - min) / (max - min);
        v = fmaxf(v, 0.0f);  // Rust f32::max / min: NaN-ignoring, like fmaxf/fminf
        v = fminf(v, 1.0f);
    }
    grey[(uint64_t)y * T + x] = v;
}

__global__ void spec_to_grey_kernel(const float* spec, uint32_t T, uint32_t bins, uint32_t H,
                                    float max, float min, float* grey) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t y = blockIdx.y;
    if (x >= T || y >= H) return;
    grey_px(spec, T, bins, H, max, min, grey, x, y);
}

int launch_spec_to_grey(const float* spec, uint32_t T, uint32_t bins, uint32_t H, float max,
                        float min, float* grey, hipStream_t s) {
    if (T == 0 || H == 0) return 0;
    dim3 grid((T + 255) / 256, H);
    hipLaunchKernelGGL(spec_to_grey_kernel, grid, dim3(256), 0, s, spec, T, bins, H, max, min, grey);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// K5 vertical Lanczos3 pass: out[oy][x] = sum_i in[left+i][x] * w[i] (sequential order)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void resize_v_px(const float* in, uint32_t w, const int32_t* left,
                                            const int32_t* cnt, const int32_t* woff,
                                            const float* wts, float* out, uint32_t x, uint32_t oy) {
    const int32_t l = left[oy], n = cnt[oy];
    const float* wr = wts + woff[oy];
    float t = 0.0f;
    for (int32_t i = 0; i < n; ++i) t += in[(uint64_t)(l + i) * w + x] * wr[i];
    out[(uint64_t)oy * w + x] = t;
}

__global__ void resize_v_kernel(const float* in, uint32_t w, uint32_t nh, const int32_t* left,
                                const int32_t* cnt, const int32_t* woff, const float* wts,
                                float* out) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t oy = blockIdx.y;
    if (x >= w || oy >= nh) return;
    resize_v_px(in, w, left, cnt, woff, wts, out, x, oy);
}

int launch_resize_v(const float* in, uint32_t w, uint32_t h, uint32_t nh, const int32_t* left,
                    const int32_t* cnt, const int32_t* woff, const float* wts, int max_taps,
                    float* out, hipStream_t s) {
    (void)h;
    (void)max_taps;
    if (w == 0 || nh == 0) return 0;
    dim3 grid((w + 255) / 256, nh);
    hipLaunchKernelGGL(resize_v_kernel, grid, dim3(256), 0, s, in, w, nh, left, cnt, woff, wts, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// K5 horizontal pass + K6 colormap (display.rs:24-42): RGB u8 [nh][nw][3]
// ------------------------------------------------------------------------------------

__device__ __forceinline__ void resize_h_rgb_px(const float* in, uint32_t w, uint32_t nw,
                                                const int32_t* left, const int32_t* cnt,
                                                const int32_t* woff, const float* wts,
                                                const uint8_t* cmap, uint8_t* out, uint32_t ox,
                                                uint32_t y) {
    const int32_t l = left[ox], n = cnt[ox];
    const float* wr = wts + woff[ox];
    const float* row = in + (uint64_t)y * w;
    float t = 0.0f;
    for (int32_t i = 0; i < n; ++i) t += row[l + i] * wr[i];
    // convert_grey_to_color; the reference asserts x >= 0 (a panic on Lanczos undershoot):
    // product policy treats x < 0 (and NaN) as 0 -- bit-identical wherever it does not panic.
    float x = t;
    if (!(x >= 0.0f)) x = 0.0f;
    const float position = 10.0f * x;
    const float fl = floorf(position);
    uint8_t* o = out + ((uint64_t)y * nw + ox) * 3;
    if (fl >= 9.0f) {
        o[0] = cmap[27];
        o[1] = cmap[28];
        o[2] = cmap[29];
        return;
    }
    const int index = (int)fl;
    const float ratio = position - (float)index;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float av = (float)cmap[index * 3 + c], bv = (float)cmap[(index + 1) * 3 + c];
        o[c] = sat_u8(roundf(ratio * bv + (1.0f - ratio) * av));
    }
}

__global__ void resize_h_rgb_kernel(const float* in, uint32_t w, uint32_t nh, uint32_t nw,
                                    const int32_t* left, const int32_t* cnt, const int32_t* woff,
                                    const float* wts, const uint8_t* cmap, uint8_t* out) {
    const uint32_t ox = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t y = blockIdx.y;
    if (ox >= nw || y >= nh) return;
    resize_h_rgb_px(in, w, nw, left, cnt, woff, wts, cmap, out, ox, y);
}

// ------------------------------------------------------------------------------------
// Batched render (render_rgb_batch_device): every track of a geometry group in ONE launch per
// stage, blockIdx.z = track, per-track geometry, workspace offsets and Lanczos tap tables from a
// descriptor array (RenderDesc). Same per-pixel bodies as the per-track kernels (bit-identical
// bytes); replaces 3 launches per track (9-17 us each for one image, launch- and tail-bound).
// ------------------------------------------------------------------------------------
// 64 x 64 tiles through LDS: the spectrogram is read along bins (coalesced) and the grey image
// written along frames (coalesced); the per-pixel arithmetic is grey_px's.
__global__ void __launch_bounds__(256) spec_to_grey_batch_kernel(const float* spec, uint32_t bins,
                                                                 float max, float min,
                                                                 const RenderDesc* d, float* grey) {
    __shared__ float tile[64][65];
    const RenderDesc r = d[blockIdx.z];
    const uint32_t x0 = blockIdx.x * 64, y0 = blockIdx.y * 64;
    if (x0 >= r.T || y0 >= r.H) return;  // block-uniform
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const float* sp = spec + r.spec_off;
    const uint32_t y = y0 + tx;
#pragma unroll 4
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t xi = ty + 4 * k, x = x0 + xi;
        float v = 0.0f;
        if (x < r.T && y < r.H && y >= r.H - bins) {
            const float db = sp[(uint64_t)x * bins + (r.H - 1 - y)];
            v = (db - min) / (max - min);
            v = fmaxf(v, 0.0f);
            v = fminf(v, 1.0f);
        }
        tile[tx][xi] = v;
    }
    __syncthreads();
    float* g = grey + r.grey_off;
#pragma unroll 4
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t yi = ty + 4 * k, yy = y0 + yi, x = x0 + tx;
        if (yy < r.H && x < r.T) g[(uint64_t)yy * r.T + x] = tile[yi][tx];
    }
}

__global__ void resize_v_batch_kernel(uint32_t nh, const RenderDesc* d, const float* grey,
                                      float* tmp) {
    const RenderDesc r = d[blockIdx.z];
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= r.T) return;
    const float* in = grey + r.grey_off + x;
    // a block walks a contiguous run of output rows: consecutive rows share most of their taps,
    // so the grey rows they read are L1 hits after the first (a row-strided walk re-reads them
    // from L2 once per tap: the pass was L2-bandwidth-bound)
    const uint32_t rpb = (nh + gridDim.y - 1) / gridDim.y;
    const uint32_t oy1 = (blockIdx.y + 1) * rpb < nh ? (blockIdx.y + 1) * rpb : nh;
    for (uint32_t oy = blockIdx.y * rpb; oy < oy1; ++oy) {
        const int32_t l = r.vl[oy], n = r.vc[oy];  // row-uniform: scalar loads
        if (n > 16) {
            resize_v_px(grey + r.grey_off, r.T, r.vl, r.vc, r.vo, r.vw, tmp + r.tmp_off, x, oy);
            continue;
        }
        const float* wr = r.vw + r.vo[oy];
        const float* src = in + (uint64_t)l * r.T;
        // all tap loads in flight together; the sum in resize_v_px's order
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = i < n ? src[(uint64_t)i * r.T] : 0.0f;
        float t = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i < n) t += v[i] * wr[i];
        tmp[r.tmp_off + (uint64_t)oy * r.ts + x] = t;
    }
}


// A block owns 256 output columns of one image and walks its rows (blockIdx.y-strided). The
// block's input span [lb, lb + span) of each row is staged in LDS (one coalesced load per
// element; the taps of neighbouring columns overlap). Columns with <= kHTaps taps keep their
// weights in registers and sum branch-free; columns with more (downsampling: up to ntap, the
// group's maximum) read their weights from an LDS copy laid out tap-major (conflict-free). The
// sum runs in resize_h_rgb_px's order (t = 0; t += in * w, i ascending). The row segment's RGB
// bytes are assembled in LDS and leave as aligned 32-bit words (3-byte pixels stored lane by
// lane are byte stores at stride 3). A block whose taps do not fit takes the direct path.
constexpr int kHTaps = 16;
template <int KT>
__global__ void __launch_bounds__(256) resize_h_rgb_batch_kernel(uint32_t nh, const RenderDesc* d,
                                                                 const float* tmp,
                                                                 const uint8_t* cmap, uint8_t* rgb,
                                                                 int ntap, int span_cap, int abl) {
    extern __shared__ __attribute__((aligned(16))) float hsm[];
    float* rin = hsm;                                       // span_cap + KT floats
    float* wl = hsm + span_cap + KT;                    // ntap x 256 (when ntap > KT)
    uint8_t* seg = reinterpret_cast<uint8_t*>(wl + (ntap > KT ? ntap * 256 : 0));
    uint8_t* cm = seg + 256 * 3;
    const RenderDesc r = d[blockIdx.z];
    const uint32_t ox0 = blockIdx.x * 256;
    if (ox0 >= r.nw) return;  // block-uniform
    const int tid = threadIdx.x;
    if (tid < 30) cm[tid] = cmap[tid];
    const uint32_t ox = ox0 + tid;
    const bool act = ox < r.nw;
    int32_t l = 0, n = 0;
    float w[KT];
    const float* wr = r.hw;
    if (act) {
        l = r.hl[ox];
        n = r.hc[ox];
        wr = r.hw + r.ho[ox];
    }
#pragma unroll
    for (int i = 0; i < KT; ++i) w[i] = (i < n && n <= KT) ? wr[i] : 0.0f;
    const bool wide = n > KT && n <= ntap && ntap > KT;
    if (wide)
        for (int i = 0; i < n; ++i) wl[i * 256 + tid] = wr[i];
    // + KT zeros after the span: the register sum runs all KT terms branch-free, the
    // terms past a column's count being (+0 weight) x (finite value) = +-0, which leave the
    // sum's bits unchanged (t is never -0: it starts at +0 and x + -x rounds to +0)
    for (int k = tid; k < span_cap + KT; k += 256) rin[k] = 0.0f;
    const uint32_t npx = r.nw - ox0 < 256u ? r.nw - ox0 : 256u;
    const uint32_t nb = 3 * npx;
    const int32_t lb = r.hl[ox0];
    const uint32_t last = ox0 + npx - 1;
    int32_t span = r.hl[last] + r.hc[last] - lb;  // supports are monotone in ox
    span = span < 0 ? 0 : (span > span_cap ? span_cap : span);
    const bool fits = !act || (l >= lb && l + n <= lb + span && (n <= KT || wide));
    const bool staged = __syncthreads_and(fits) != 0;
    // the next row's span is loaded into registers while this row is summed (one HBM latency
    // per row otherwise: the pass was latency-bound), when it fits kHPf floats per thread
    constexpr int kHPf = 8;
    const bool pf = staged && span <= kHPf * 256;
    float nx[kHPf];
    auto load_row = [&](uint32_t yy) {
        const float* src = tmp + r.tmp_off + (uint64_t)yy * r.ts + lb;
#pragma unroll
        for (int p = 0; p < kHPf; ++p) {
            const int32_t k = tid + 256 * p;
            nx[p] = k < span ? src[k] : 0.0f;
        }
    };
    auto store_row = [&](uint32_t yy, const uint8_t* sg) {
        uint8_t* g = rgb + r.rgb_off + ((uint64_t)yy * r.nw + ox0) * 3;
        const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(g) & 3);
        const uint32_t head = mis ? (4 - mis < nb ? 4 - mis : nb) : 0;
        if ((uint32_t)tid < head) g[tid] = sg[tid];
        const uint32_t nwords = (nb - head) / 4;
        uint32_t* gw = reinterpret_cast<uint32_t*>(g + head);
        for (uint32_t k = tid; k < nwords; k += 256) {
            const uint32_t b = head + 4 * k;
            gw[k] = (uint32_t)sg[b] | ((uint32_t)sg[b + 1] << 8) | ((uint32_t)sg[b + 2] << 16) |
                    ((uint32_t)sg[b + 3] << 24);
        }
        for (uint32_t b = head + 4 * nwords + tid; b < nb; b += 256) g[b] = sg[b];
    };
    // rows below oz: their tmp rows are +0 (never formed) -> colormap(+0), no tmp reads
    uint32_t ys = blockIdx.y;
    if (r.oz > ys) {
        if (act) colormap_px(0.0f, cm, seg + 3 * tid);
        __syncthreads();
        for (; ys < r.oz && ys < nh; ys += gridDim.y) store_row(ys, seg);
        __syncthreads();
    }
#if THESIA_H_2ROW
    if (pf && abl == 0) {
        // two rows per step (y and y + G): two independent sum chains per column over the
        // same weights, both rows' spans prefetched a step ahead
        float* rin1 = reinterpret_cast<float*>(cm + 32);
#if !THESIA_H_DIRECT
        uint8_t* seg1 = reinterpret_cast<uint8_t*>(rin1 + span_cap + KT);
#endif
        for (int k = tid; k < span_cap + KT; k += 256) rin1[k] = 0.0f;
        const uint32_t G = gridDim.y;
        float nx1[kHPf];
        auto load_row1 = [&](uint32_t yy) {
            const float* src = tmp + r.tmp_off + (uint64_t)yy * r.ts + lb;
#pragma unroll
            for (int p = 0; p < kHPf; ++p) {
                const int32_t k = tid + 256 * p;
                nx1[p] = k < span ? src[k] : 0.0f;
            }
        };
        if (ys < nh) load_row(ys);
        if (ys + G < nh) load_row1(ys + G);
        for (uint32_t y = ys; y < nh; y += 2 * G) {
            const bool two = y + G < nh;
#pragma unroll
            for (int p = 0; p < kHPf; ++p) {
                const int32_t k = tid + 256 * p;
                if (k < span) {
                    rin[k] = nx[p];
                    rin1[k] = nx1[p];
                }
            }
            __syncthreads();
#if !(THESIA_H_ABL & 4)  // ablation (timing only): no span loads
            if (y + 2 * G < nh) load_row(y + 2 * G);
            if (y + 3 * G < nh) load_row1(y + 3 * G);
#endif
            if (act) {
                float t0 = 0.0f, t1 = 0.0f;
                const int base = l - lb;
                if (THESIA_H_ABL & 1) {  // ablation (timing only): no sums
                } else if (n <= KT) {
#pragma unroll
                    for (int i = 0; i < KT; ++i) {
                        t0 += rin[base + i] * w[i];
                        t1 += rin1[base + i] * w[i];
                    }
                } else {
                    for (int i = 0; i < n; ++i) {
                        const float wi = wl[i * 256 + tid];
                        t0 += rin[base + i] * wi;
                        t1 += rin1[base + i] * wi;
                    }
                }
#if THESIA_H_DIRECT
                // RGB bytes straight to HBM (three byte stores per pixel: a wave's 192 bytes are
                // contiguous, L2 merges them), no LDS assembly and one barrier less per step
                uint8_t px[6];
                colormap_px(t0, cm, px);
                colormap_px(t1, cm, px + 3);
                uint8_t* g0 = rgb + r.rgb_off + ((uint64_t)y * r.nw + ox) * 3;
                if (THESIA_H_ABL & 2) {  // ablation (timing only): no stores
                    if (px[0] == 255 && px[1] == 1 && px[2] == 254) g0[0] = 7;
                } else {
                g0[0] = px[0]; g0[1] = px[1]; g0[2] = px[2];
                }
                if (two && !(THESIA_H_ABL & 2)) {
                    uint8_t* g1 = g0 + (uint64_t)G * r.nw * 3;
                    g1[0] = px[3]; g1[1] = px[4]; g1[2] = px[5];
                }
#else
                colormap_px(t0, cm, seg + 3 * tid);
                colormap_px(t1, cm, seg1 + 3 * tid);
#endif
            }
            __syncthreads();
#if !THESIA_H_DIRECT
            store_row(y, seg);
            if (two) store_row(y + G, seg1);
            __syncthreads();
#endif
        }
        return;
    }
#endif
    if (pf && ys < nh) load_row(ys);
    for (uint32_t y = ys; y < nh; y += gridDim.y) {
        if (pf) {
#pragma unroll
            for (int p = 0; p < kHPf; ++p) {
                const int32_t k = tid + 256 * p;
                if (k < span) rin[k] = nx[p];
            }
            __syncthreads();
            if (y + gridDim.y < nh) load_row(y + gridDim.y);
        } else if (staged) {
            const float* src = tmp + r.tmp_off + (uint64_t)y * r.ts + lb;
            if (!(abl & 4))  // ablation (timing only): no row loads
                for (int32_t k = tid; k < span; k += 256) rin[k] = src[k];
            __syncthreads();
        }
        if (act) {
            float t = 0.0f;
            if (staged) {
                const int base = l - lb;
                if (n <= KT) {
#pragma unroll
                    for (int i = 0; i < KT; ++i) t += rin[base + i] * w[i];
                } else {
                    for (int i = 0; i < n; ++i) t += rin[base + i] * wl[i * 256 + tid];
                }
            } else {
                const float* row = tmp + r.tmp_off + (uint64_t)y * r.ts + l;
                for (int32_t i = 0; i < n; ++i) t += row[i] * wr[i];
            }
            if (abl & 1) {  // ablation (timing only): no colormap
                seg[3 * tid] = (uint8_t)t;
            } else {
                colormap_px(t, cm, seg + 3 * tid);
            }
        }
        __syncthreads();
        if (abl & 2) { __syncthreads(); continue; }  // ablation: no global stores
        store_row(y, seg);
        __syncthreads();
    }
}

// thesia_ranges_global: one block; each thread folds a stride of the tracks' slots (NaN tracks
// skipped: ndarray-stats' max/min error -> unwrap_or, lib.rs:198-199), a shared-memory tree
// folds the threads, thread 0 applies lib.rs:208-209 in the order thesia.shard.global_db_range
// does (Python's min / max argument order, the difference in double, the result rounded to f32)
__global__ void __launch_bounds__(256) range_global_kernel(const int* trk, uint32_t n, double db_range,
                                                           float* out) {
    __shared__ float smx[256], smn[256];
    float mx = -INFINITY, mn = INFINITY;
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        if (trk[3 * i + 2]) continue;
        mx = fmaxf(mx, range_unord(trk[3 * i]));
        mn = fminf(mn, range_unord(trk[3 * i + 1]));
    }
    smx[threadIdx.x] = mx;
    smn[threadIdx.x] = mn;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + w]);
            smn[threadIdx.x] = fminf(smn[threadIdx.x], smn[threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float gx = smx[0], gn = smn[0];
        const float gmax = 0.0f < gx ? 0.0f : gx;               // min(mx, 0.0)
        const double t = (double)gmax - db_range;
        const double m = t > (double)gn ? t : (double)gn;         // max(mn, gmax - db_range)
        out[0] = gmax;
        out[1] = (float)m;
    }
}

int launch_range_global(const int* trk_range, uint32_t n, double db_range, float* out, hipStream_t s) {
    hipLaunchKernelGGL(range_global_kernel, dim3(1), dim3(256), 0, s, trk_range, n, db_range, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_render_batch(const float* spec, uint32_t bins, float max, float min,
                        const RenderDesc* d_desc, uint32_t n, uint32_t T_max, uint32_t H_max,
                        uint32_t nw_max, uint32_t nh, int h_taps, int h_span, float* grey,
                        float* tmp, const uint8_t* cmap, uint8_t* rgb, hipStream_t s) {
    if (n == 0 || nh == 0) return 0;
    if (n > 65535) return -2;
    uint32_t ry = 64;  // grid.y: row blocks per image (strided row loop inside)
    bool ry_set = false;
    int abl = 0;
#ifdef THESIA_EXPERIMENTS
    if (const char* e = getenv("THESIA_RENDER_RY")) { ry = (uint32_t)atoi(e) > 0 ? (uint32_t)atoi(e) : 64; ry_set = true; }
    if (const char* e = getenv("THESIA_RENDER_ABL")) abl = atoi(e);  // ablations (timing only)
#endif
    dim3 g1((T_max + 63) / 64, (H_max + 63) / 64, n);
    hipLaunchKernelGGL(spec_to_grey_batch_kernel, g1, dim3(256), 0, s, spec, bins, max, min, d_desc, grey);
    dim3 g2((T_max + 255) / 256, nh < ry ? nh : ry, n);
    hipLaunchKernelGGL(resize_v_batch_kernel, g2, dim3(256), 0, s, nh, d_desc, grey, tmp);
    // the horizontal pass prefers fewer, longer row walks (one LDS weight / tap setup per block
    // amortised over more rows): 16 row blocks per image measured 3.96 vs 4.46 ms at 64
    const uint32_t ry_h = ry_set ? ry : 16;
    dim3 g3((nw_max + 255) / 256, nh < ry_h ? nh : ry_h, n);
    // LDS: the staged span (+ kHTaps zeros), tap-major weights for > kHTaps taps, RGB segment,
    // colormap; beyond 64 KiB the weights (then the span) stay in HBM (direct path)
    int taps = h_taps > kHTaps ? h_taps : 0;
    int span = h_span;
    // span + zeros, wide weights, RGB segment, colormap; then the second row's span + segment
    auto lds = [&]() { return (2 * (span + kHTaps) + taps * 256) * 4 + 2 * 256 * 3 + 32; };
    if (lds() > 65536) taps = 0;
    if (lds() > 65536) span = 4096;
    hipLaunchKernelGGL(resize_h_rgb_batch_kernel<kHTaps>, g3, dim3(256), lds(), s, nh, d_desc, tmp, cmap, rgb,
                       taps, span, abl);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// Fused display path (launch_render_batch2): grey + vertical Lanczos3 in one pass
// ------------------------------------------------------------------------------------
// K4+K5v: a block owns 64 frames x `band` output rows of one track (band: the widest band
// whose grey rows and weights fit the LDS tile, chosen per launch by the host). The grey values those rows'
// taps reach (display.rs:44-54: rows above the track's band are the image's zero fill) are formed
// from the dB spectrogram straight into an LDS tile [grey row][frame] (each frame's bins read
// contiguously), the band's tap weights into LDS; lane = frame, each wave walks its output rows:
// tmp[oy][x] = sum_i grey[l + i][x] * w[i] in resize_v_px's order (t = 0; t += in * w), stored
// along frames (coalesced). The grey image itself is never written (7.7 GB of the C5 step's
// display traffic in the three-stage path).
__global__ void __launch_bounds__(256) grey_vert_kernel(const float* spec, uint32_t bins, float max,
                                                        float min, uint32_t nh, const RenderDesc* d,
                                                        float* tmp, int tile_cap, int kv, uint32_t band) {
    extern __shared__ __attribute__((aligned(16))) float vsm[];
    const RenderDesc r = d[blockIdx.z];
    if (r.grange) {  // the device-side global range (RenderDesc::grange)
        max = r.grange[0];
        min = r.grange[1];
    }
    const GreyMap gm(max, min);
    const uint32_t x0 = blockIdx.x * 64, ob = blockIdx.y * band;
    const uint32_t oy1 = ob + band < nh ? ob + band : nh;
    const uint32_t oy0 = ob > r.oz ? ob : r.oz;  // rows below oz: +0, never formed (RenderDesc)
    if (x0 >= r.T || oy0 >= oy1) return;  // block-uniform
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // grey rows [ya, ya + rows) reached by the band's taps, each row's taps padded to kv (a
    // multiple of 4) with zero weights: supports are monotone in oy, so the last row's padded
    // support ends the tile. A padded term adds +-0 (zero weight x finite grey) to the sum,
    // which leaves its bits unchanged (t starts at +0 and x + -x rounds to +0): the sum equals
    // resize_v_px's t = 0; t += in * w over the row's own taps.
    const int32_t ya = r.vl[oy0];
    const int32_t rows = r.vl[oy1 - 1] - ya + kv;
    const uint32_t nb = oy1 - oy0;
    constexpr int TS = 65;                    // tile row stride: staging writes walk rows
    const int mrows = ((int)band + 3) & ~3;   // meta entries, rounded for 16-byte alignment
    int* meta = reinterpret_cast<int*>(vsm);  // per band row: its first tile row
    float* tile = vsm + mrows;                // [tile_cap][TS]
    float* wl = tile + ((tile_cap * TS + 3) & ~3);  // [band][kv], zero-padded per row
    const bool staged = rows <= tile_cap;
    const uint32_t x = x0 + lane;
    const int32_t H = (int32_t)r.H, top = (int32_t)r.H - (int32_t)bins;
    const float* sp = spec + r.spec_off;
    if (staged && rows <= 128) {
        // Tile row k holds bin hy - k (hy = H - 1 - ya). The in-band bins [blo, bhi] are read as
        // groups of four consecutive bins [4m, 4m + 3] (16-byte loads, never below bin 0: a
        // buffer load whose offset wraps below the base returns 0 in every dword, measured; past
        // the frame's last bin it reads the next frame's or, past the block's frames, +0 per
        // dword -- rows never stored): thread -> (group g = tid mod ng, frame phase p = tid / ng),
        // P = 256 / ng phases walk the block's frames p, p + P, ...; consecutive threads read
        // consecutive 16 bytes of one frame row (coalesced). An element costs a quarter of a
        // load, its grey value and an LDS store. Rows outside the band (the image's zero fill
        // above it, padded taps below the image) are zero-filled on their own.
        constexpr int D = THESIA_VDEPTH;
        const int32_t hy = H - 1 - ya;
        const int32_t blo = hy - rows + 1 > 0 ? hy - rows + 1 : 0;
        const int32_t bhi = hy < (int32_t)bins - 1 ? hy : (int32_t)bins - 1;
        // zero rows: k < hy - bhi (above the band) and k > hy - blo (below the image)
        const int32_t kz0 = hy - bhi < rows ? (hy - bhi > 0 ? hy - bhi : 0) : rows;
        const int32_t kz1 = blo <= bhi ? hy - blo + 1 : kz0;  // first zero row below the band
        {
            const int nz0 = kz0, nz1 = rows - (kz1 > kz0 ? kz1 : kz0);
            for (int e = tid; e < (nz0 + nz1) * 64; e += 256) {
                const int z = e >> 6, f = e & 63;
                const int kk = z < nz0 ? z : (kz1 > kz0 ? kz1 : kz0) + (z - nz0);
                tile[kk * TS + f] = 0.0f;
            }
        }
        if (blo <= bhi) {
            const int mlo = blo >> 2, ng = (bhi >> 2) - mlo + 1;  // <= 34
            const int P = __builtin_amdgcn_readfirstlane(256 / ng);
            const int g = tid % ng, p = tid / ng;
            const uint32_t nf = r.T - x0 < 64u ? r.T - x0 : 64u;  // the block's frames (uniform)
            if (p < P) {
                const int32_t b0 = 4 * (mlo + g);
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<float*>(sp + (uint64_t)x0 * bins), (short)0, (int)(nf * bins * 4u), 0x00020000);
                const uint32_t vo = ((uint32_t)p * bins + (uint32_t)b0) * 4u;  // this thread's first load
                const uint32_t step = __builtin_amdgcn_readfirstlane((uint32_t)P * bins * 4u);  // per phase step
                bool ok[4];
                float* trow[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    ok[q] = b0 + q >= blo && b0 + q <= bhi;
                    trow[q] = tile + (hy - (b0 + q)) * TS + p;
                }
                const int nit = (64 + P - 1) / P;  // phase steps covering 64 frames (uniform)
                typedef float v4f __attribute__((ext_vector_type(4)));
                for (int i0 = 0; i0 < nit; i0 += D) {
                    v4f v[D];
#pragma unroll
                    for (int i = 0; i < D; ++i)
                        v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (i0 + i) * step, 0);
#pragma unroll
                    for (int i = 0; i < D; ++i) {
                        const int f = p + P * (i0 + i);
                        if (f < 64) {
                            if (ok[0]) trow[0][P * (i0 + i)] = gm(v[i].x);
                            if (ok[1]) trow[1][P * (i0 + i)] = gm(v[i].y);
                            if (ok[2]) trow[2][P * (i0 + i)] = gm(v[i].z);
                            if (ok[3]) trow[3][P * (i0 + i)] = gm(v[i].w);
                        }
                    }
                }
            }
        }
        for (uint32_t e = tid; e < nb * (uint32_t)kv; e += 256) {
            const uint32_t j = e / (uint32_t)kv, i = e - j * (uint32_t)kv;
            const int32_t n = r.vc[oy0 + j];
            wl[e] = (int32_t)i < n ? r.vw[r.vo[oy0 + j] + i] : 0.0f;
        }
        for (uint32_t j = tid; j < nb; j += 256) meta[j] = r.vl[oy0 + j] - ya;
    } else if (staged) {
        // (frame, row) pairs flattened over the block's 256 threads (f = e / rows by a
        // multiply-high, exact for e < 2^14): consecutive threads read consecutive bins of one
        // frame (coalesced), a thread's THESIA_VDEPTH loads in flight together. Branch-free:
        // indices past the tile repeat its last element (same value to the same slot), frames
        // past T read frame T - 1 (their lanes store nothing), rows outside the track's band
        // read a clamped bin and store +0 (the image's zero fill; padded taps below the image)
        constexpr int D = THESIA_VDEPTH;
        const int total = 64 * rows;  // rows >= kv >= 4 (host): the reciprocal below is exact
        const uint32_t mrec = (uint32_t)((0x100000000ull + rows - 1) / (uint32_t)rows);
        const uint32_t emax = (uint32_t)total - 1;
        const uint32_t flast = r.T - 1 - x0;  // x0 < T (block-uniform exit above)
        // the block's frames as a buffer resource: 32-bit byte offsets from frame x0 (at most
        // 64 frames x bins floats), one buffer_load per element
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(sp + (uint64_t)x0 * bins), (short)0, -1, 0x00020000);
        const int32_t hy = H - 1 - ya;  // bin of tile row k: hy - k
        for (int e0 = 0; e0 < total; e0 += 256 * D) {
            float v[D];
            uint32_t fk[D];  // (frame, tile row) of each element: f | k << 8 (f < 64, k < 256)
#pragma unroll
            for (int i = 0; i < D; ++i) {
                uint32_t e = (uint32_t)(e0 + 256 * i + tid);
                e = e < emax ? e : emax;
                const uint32_t f = __umulhi(e, mrec);
                const int32_t k = (int32_t)(e - f * (uint32_t)rows);
                fk[i] = f | ((uint32_t)k << 8);
                const uint32_t fl = f < flast ? f : flast;
                int32_t b = hy - k;
                b = b < 0 ? 0 : b < (int32_t)bins ? b : (int32_t)bins - 1;
                v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (fl * bins + (uint32_t)b) * 4u, 0, 0));
            }
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const uint32_t f = fk[i] & 255u;
                const int32_t k = (int32_t)(fk[i] >> 8);
                const int32_t y = ya + k;
                // formed for every element (pinned: a select, not a branch around the grey value)
                float g = gm(v[i]);
                asm volatile("" : "+v"(g));
                tile[k * TS + (int32_t)f] = (y >= top && y < H) ? g : 0.0f;
            }
        }
        for (uint32_t e = tid; e < nb * (uint32_t)kv; e += 256) {
            const uint32_t j = e / (uint32_t)kv, i = e - j * (uint32_t)kv;
            const int32_t n = r.vc[oy0 + j];
            wl[e] = (int32_t)i < n ? r.vw[r.vo[oy0 + j] + i] : 0.0f;
        }
        for (uint32_t j = tid; j < nb; j += 256) meta[j] = r.vl[oy0 + j] - ya;
    }
    __syncthreads();
    if (x >= r.T) return;  // no block barrier below
    float* out = tmp + r.tmp_off + x;
    uint32_t oy = oy0 + wave;
    if (staged) {
        const float4* wl4 = reinterpret_cast<const float4*>(wl);
        const int kv4 = kv >> 2;
        const float* col = tile + lane;
        // four output rows per wave step: four independent chains (each in its own order); a
        // row's first tile row and its weights are wave-uniform (LDS broadcasts), the grey
        // values one conflict-free LDS read per tap
        for (; oy + 12 < oy1; oy += 16) {
            int lq[4];
            const float4* wq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t j = oy - oy0 + 4 * q;
                lq[q] = __builtin_amdgcn_readfirstlane(meta[j]);
                wq[q] = wl4 + j * kv4;
            }
            float t[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#if !(THESIA_V_ABL & 2)  // ablation (timing only): no sums
            for (int i4 = 0; i4 < kv4; ++i4) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 w = wq[q][i4];
                    const float* c = col + (lq[q] + 4 * i4) * TS;
                    t[q] += c[0] * w.x;
                    t[q] += c[TS] * w.y;
                    t[q] += c[2 * TS] * w.z;
                    t[q] += c[3 * TS] * w.w;
                }
            }
#endif
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#if THESIA_V_ABL & 1  // ablation (timing only): no tmp stores
                if (t[q] == 1.2345e-30f)
#endif
                    out[(uint64_t)(oy + 4 * q) * r.ts] = t[q];
            }
        }
        for (; oy < oy1; oy += 4) {
            const uint32_t j = oy - oy0;
            const int l = __builtin_amdgcn_readfirstlane(meta[j]);
            const float4* w4 = wl4 + j * kv4;
            float t = 0.0f;
            for (int i4 = 0; i4 < kv4; ++i4) {
                const float4 w = w4[i4];
                const float* c = col + (l + 4 * i4) * TS;
                t += c[0] * w.x;
                t += c[TS] * w.y;
                t += c[2 * TS] * w.z;
                t += c[3 * TS] * w.w;
            }
            out[(uint64_t)oy * r.ts] = t;
        }
        return;
    }
    // direct path (a band whose tile does not fit): taps straight from HBM, scalar weights
    for (; oy < oy1; oy += 4) {
        const int32_t l = r.vl[oy], n = r.vc[oy];
        const float* wr = r.vw + r.vo[oy];
        const float* srow = sp + (uint64_t)x * bins;
        float t = 0.0f;
        for (int32_t i = 0; i < n; ++i) {
            const int32_t y = l + i;
            t += (y >= top ? gm(srow[H - 1 - y]) : 0.0f) * wr[i];
        }
        out[(uint64_t)oy * r.ts] = t;
    }
}

// K4+K5v, wide: grey_vert_kernel with FPL consecutive frames per lane (a block owns 64 * FPL
// frames x `band` output rows). A tap reads the lane's FPL grey values of one tile row with one
// ds_read_b64 / ds_read_b128 (256 B/clk, against 128 for the narrow kernel's ds_read_b32) and an
// output row leaves as one FPL * 4-byte store per lane: 512 B / 1 KiB contiguous per wave
// instead of 256 B. Same staging, zero-padded weights and per-element summation order as
// grey_vert_kernel (identical bytes). Lanes whose frames start past T store nothing; frames past
// T inside a stored vector land in the row padding [T, ts) as finite values (their tile columns
// are grey(+0)), which the horizontal pass only ever multiplies by zero weights.
template <int FPL>
struct FVec;
template <>
struct FVec<2> {
    using T = float2;
};
template <>
struct FVec<4> {
    using T = float4;
};
template <int FPL>
__device__ __forceinline__ float& fv(typename FVec<FPL>::T& v, int c) {
    return reinterpret_cast<float*>(&v)[c];
}
template <int FPL>
__global__ void __launch_bounds__(256) grey_vert_wide_kernel(const float* spec, uint32_t bins, float max,
                                                             float min, uint32_t nh, const RenderDesc* d,
                                                             float* tmp, int tile_cap, int kv, uint32_t band) {
    using VT = typename FVec<FPL>::T;
    constexpr int FW = 64 * FPL;  // frames per block
    constexpr int TS = FW + 4;    // tile row stride (16-byte aligned rows)
    extern __shared__ __attribute__((aligned(16))) float vsm[];
    const RenderDesc r = d[blockIdx.z];
    if (r.grange) {  // the device-side global range (RenderDesc::grange)
        max = r.grange[0];
        min = r.grange[1];
    }
    const GreyMap gm(max, min);
    const uint32_t x0 = blockIdx.x * FW, ob = blockIdx.y * band;
    const uint32_t oy1 = ob + band < nh ? ob + band : nh;
    const uint32_t oy0 = ob > r.oz ? ob : r.oz;  // rows below oz: +0, never formed (RenderDesc)
    if (x0 >= r.T || oy0 >= oy1) return;         // block-uniform
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t ya = r.vl[oy0];
    const int32_t rows = r.vl[oy1 - 1] - ya + kv;  // <= tile_cap (host)
    const uint32_t nb = oy1 - oy0;
    const int mrows = ((int)band + 3) & ~3;
    int* meta = reinterpret_cast<int*>(vsm);
    float* tile = vsm + mrows;                      // [tile_cap][TS]
    float* wl = tile + tile_cap * TS;               // [band][kv], zero-padded per row
    const int32_t H = (int32_t)r.H, top = (int32_t)r.H - (int32_t)bins;
    const float* sp = spec + r.spec_off;
    {
        // (frame, row) pairs in quads of frames: element e = (quad q, row k, frame 4q + c), c
        // fastest. A wave reads 16 consecutive bins of 4 frames (4 x 64 B) and its LDS stores
        // k * TS + 4q + c (TS = 4 mod 32) fall on 32 distinct banks; THESIA_VDEPTH loads in
        // flight per thread. The zero fill above the track's band, rows past the image and
        // frames past T are never loaded.
        constexpr int D = THESIA_VDEPTH;
        const int total = FW * rows;
        const uint32_t r4 = 4u * (uint32_t)rows;
        const uint32_t mrec = (uint32_t)((0x100000000ull + r4 - 1) / r4);
        auto split = [&](uint32_t e, uint32_t& f, int32_t& k) {
            const uint32_t q = __umulhi(e, mrec), rem = e - q * r4;
            k = (int32_t)(rem >> 2);
            f = 4 * q + (rem & 3);
        };
        for (int e0 = 0; e0 < total; e0 += 256 * D) {
            float v[D];
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const uint32_t e = (uint32_t)(e0 + 256 * i + tid);
                uint32_t f;
                int32_t k;
                split(e, f, k);
                const int32_t y = ya + k;
                v[i] = 0.0f;
                if ((int)e < total && y >= top && y < H && x0 + f < r.T)
                    v[i] = sp[(uint64_t)(x0 + f) * bins + (uint32_t)(H - 1 - y)];
            }
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const uint32_t e = (uint32_t)(e0 + 256 * i + tid);
                uint32_t f;
                int32_t k;
                split(e, f, k);
                const int32_t y = ya + k;
                if ((int)e < total) tile[k * TS + f] = (y >= top && y < H) ? gm(v[i]) : 0.0f;
            }
        }
        for (uint32_t e = tid; e < nb * (uint32_t)kv; e += 256) {
            const uint32_t j = e / (uint32_t)kv, i = e - j * (uint32_t)kv;
            const int32_t n = r.vc[oy0 + j];
            wl[e] = (int32_t)i < n ? r.vw[r.vo[oy0 + j] + i] : 0.0f;
        }
        for (uint32_t j = tid; j < nb; j += 256) meta[j] = r.vl[oy0 + j] - ya;
    }
    __syncthreads();
    const uint32_t xl = x0 + (uint32_t)(FPL * lane);
    const bool st = xl < r.T;  // (no block barrier below)
    float* out = tmp + r.tmp_off + xl;
    const float4* wl4 = reinterpret_cast<const float4*>(wl);
    const int kv4 = kv >> 2;
    const float* col = tile + FPL * lane;
    auto tap = [&](VT& t, const float* c, float w) {
        const VT g = *reinterpret_cast<const VT*>(c);
        const float* gp = reinterpret_cast<const float*>(&g);
#pragma unroll
        for (int u = 0; u < FPL; ++u) fv<FPL>(t, u) += gp[u] * w;
    };
    uint32_t oy = oy0 + wave;
    // four output rows per wave step (four independent chains per frame, each in its own order)
    for (; oy + 12 < oy1; oy += 16) {
        int lq[4];
        const float4* wq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t j = oy - oy0 + 4 * q;
            lq[q] = __builtin_amdgcn_readfirstlane(meta[j]);
            wq[q] = wl4 + j * kv4;
        }
        VT t[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int u = 0; u < FPL; ++u) fv<FPL>(t[q], u) = 0.0f;
        for (int i4 = 0; i4 < kv4; ++i4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 w = wq[q][i4];
                const float* c = col + (lq[q] + 4 * i4) * TS;
                tap(t[q], c, w.x);
                tap(t[q], c + TS, w.y);
                tap(t[q], c + 2 * TS, w.z);
                tap(t[q], c + 3 * TS, w.w);
            }
        }
        if (st) {
#pragma unroll
            for (int q = 0; q < 4; ++q) *reinterpret_cast<VT*>(out + (uint64_t)(oy + 4 * q) * r.ts) = t[q];
        }
    }
    for (; oy < oy1; oy += 4) {
        const uint32_t j = oy - oy0;
        const int l = __builtin_amdgcn_readfirstlane(meta[j]);
        const float4* w4 = wl4 + j * kv4;
        VT t;
#pragma unroll
        for (int u = 0; u < FPL; ++u) fv<FPL>(t, u) = 0.0f;
        for (int i4 = 0; i4 < kv4; ++i4) {
            const float4 w = w4[i4];
            const float* c = col + (l + 4 * i4) * TS;
            tap(t, c, w.x);
            tap(t, c + TS, w.y);
            tap(t, c + 2 * TS, w.z);
            tap(t, c + 3 * TS, w.w);
        }
        if (st) *reinterpret_cast<VT*>(out + (uint64_t)oy * r.ts) = t;
    }
}

int grey_vert_wide_lds_bytes(int fpl, uint32_t band, int tile_cap, int kv) {
    return ((((int)band + 3) & ~3) + tile_cap * (64 * fpl + 4) + (int)band * kv) * 4;
}

// The horizontal pass with its row spans staged by LDS-DMA (global_load_lds_dwordx4, no VGPRs):
// NB row buffers per block, NB - 1 rows in flight while a row is summed, one barrier per row.
// A block owns 256 output columns of one image (thread = column, <= KT zero-padded register
// weights: n <= KT for every column of the launch) and walks its rows (blockIdx.y-strided). Row
// k's span [lb4, lb4 + span4) (16-byte aligned) lands in buffer k % NB: wave w issues the chunks
// (m * 4 + w) * 64 + lane, m < K; chunks past the span re-read the span's last chunk (finite
// values in the buffer's tail, summed with zero weights: bits unchanged, as in the staged pass;
// the intermediate's row padding is zeroed when its workspace is allocated). Each wave waits for
// its own chunks of row k (vmcnt((NB - 2) K): all but the wave's (NB - 2) K youngest
// vector-memory ops retire, in issue order; the RGB stores interleaved with the DMAs make that
// wait stricter than row k alone — counting them exactly measured no faster), then
// the barrier makes the whole row visible and frees the buffer of row k - 1 for row k + NB - 1.
// Same sums and colormap as resize_h_rgb_batch_kernel (identical bytes).
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// RP rows per barrier (groups of RP rows in NB x RP buffers). The launcher uses 1: two rows per
// barrier, both rows' sums and colormaps interleaved, measured no faster (C5 step 3.86 vs 3.81 ms,
// profiles/r04_display/ab_experiments.txt).
template <int KT, int K, int NB, int RP = 1>
__global__ void __launch_bounds__(256) resize_h_dma_kernel(uint32_t nh, const RenderDesc* d, const float* tmp,
                                                           const uint8_t* cmap, uint8_t* rgb) {
    extern __shared__ __attribute__((aligned(16))) float hsm[];
    constexpr int BUF = K * 1024;  // floats per row buffer: K chunks of 64 lanes x 16 B per wave
    uint2* lut = reinterpret_cast<uint2*>(hsm + NB * RP * BUF);  // colormap_rgb's stop pairs
    const RenderDesc r = d[blockIdx.z];
    const uint32_t ox0 = blockIdx.x * 256;
    if (ox0 >= r.nw) return;  // block-uniform
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 10) lut[tid] = colormap_pair(cmap, tid);
    const uint32_t ox = ox0 + tid;
    const bool act = ox < r.nw;
    int32_t l = 0, n = 0;
    const float* wr = r.hw;
    if (act) {
        l = r.hl[ox];
        n = r.hc[ox];
        wr = r.hw + r.ho[ox];
    }
    float w[KT];
#pragma unroll
    for (int i = 0; i < KT; ++i) w[i] = i < n ? wr[i] : 0.0f;
    const uint32_t npx = r.nw - ox0 < 256u ? r.nw - ox0 : 256u;
    const int32_t lb4 = r.hl[ox0] & ~3;
    const uint32_t last = ox0 + npx - 1;
    const int32_t span4 = (r.hl[last] + r.hc[last] - lb4 + 3) & ~3;  // <= BUF - KT (host)
    const int nchunk = span4 > 0 ? span4 >> 2 : 1;
    const int base = l - lb4;
    __syncthreads();  // colormap pairs
    const uint32_t lut_lds = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint2*)lut);
    // a pixel's 3 bytes (colormap_rgb packs them r | g << 8 | b << 16)
    auto put = [](uint8_t* o, uint32_t px) {
        o[0] = (uint8_t)px;
        o[1] = (uint8_t)(px >> 8);
        o[2] = (uint8_t)(px >> 16);
    };
    // rows below oz: their intermediate rows are +0 (never formed) -> colormap(+0)
    const uint32_t G = gridDim.y;
    const uint64_t ostep = (uint64_t)G * r.nw * 3;  // bytes between the block's rows
    uint8_t* o = rgb + r.rgb_off + (uint64_t)ox * 3 + (uint64_t)blockIdx.y * r.nw * 3;
    uint32_t y0 = blockIdx.y;
    // where the image's rows start 4-byte aligned (nwidth and the RGB offset multiples of 4), a
    // wave's 64 pixels (192 bytes) leave as 48 dword stores instead of 64 byte + 64 short stores (a
    // third of the addresses for the texture addresser): the summed rows packed through LDS (inline
    // asm: the compiler cannot tell plain LDS accesses from the DMA's targets and would wait for
    // every DMA in flight before them), the colormap(+0) rows below oz as the repeating pattern
    const bool drgb = ((r.nw | (uint32_t)r.rgb_off) & 3u) == 0;  // block-uniform
    const uint32_t wb = ox0 + 64u * (uint32_t)wave;              // the wave's first column
    const uint32_t wpx = wb < r.nw ? (r.nw - wb < 64u ? r.nw - wb : 64u) : 0u;
    const int nd = (int)(3u * wpx) >> 2, ntail = (int)(3u * wpx) & 3;  // the wave's dwords, tail bytes
    const uint32_t stg = lut_lds + 128u + 192u * (uint32_t)wave;        // the wave's 192 staging bytes
    if (r.oz > y0) {
        const uint32_t px = colormap_rgb(0.0f, lut);
        if (drgb) {
            // byte i of the row piece is component i mod 3 of px; dword lane = bytes 4 lane ..
            auto comp = [&](int i) { return (px >> (8 * (i % 3))) & 0xFFu; };
            const int b0 = 4 * lane;
            const uint32_t dw = comp(b0) | comp(b0 + 1) << 8 | comp(b0 + 2) << 16 | comp(b0 + 3) << 24;
            const uint32_t tb = comp(4 * nd + lane);
            uint8_t* ow = o - 3 * tid + 192 * wave;  // the wave's first pixel (o = base + 3 ox)
            for (; y0 < r.oz && y0 < nh; y0 += G, ow += ostep, o += ostep) {
                if (lane < nd) reinterpret_cast<uint32_t*>(ow)[lane] = dw;
                if (lane < ntail) ow[4 * nd + lane] = (uint8_t)tb;
            }
        } else {
            for (; y0 < r.oz && y0 < nh; y0 += G, o += ostep)
                if (act) put(o, px);
        }
    }
    const int nrows = y0 < nh ? (int)((nh - 1 - y0) / G) + 1 : 0;
    const float* rows0 = tmp + r.tmp_off + lb4;
    // group g = rows g RP .. g RP + RP - 1 in buffers (g % NB) RP + i; rows past the last repeat
    // it (same DMA count per group, so the counted waits hold; never summed)
    auto dma = [&](int g) {
#pragma unroll
        for (int i = 0; i < RP; ++i) {
            int k = g * RP + i;
            k = k < nrows ? k : nrows - 1;
            const float* row = rows0 + (uint64_t)(y0 + G * (uint32_t)k) * r.ts;
            float* buf = hsm + ((g % NB) * RP + i) * BUF;
#pragma unroll
            for (int m = 0; m < K; ++m) {
                const int c = (m * 4 + wave) * 64 + lane;
                const int cc = c < nchunk ? c : nchunk - 1;
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(row + 4 * cc),
                                                 (__attribute__((address_space(3))) void*)(buf + (m * 4 + wave) * 256),
                                                 16, 0, 0);
            }
        }
    };
    const int ng = (nrows + RP - 1) / RP;
    for (int g = 0; g < NB - 1 && g < ng; ++g) dma(g);
    for (int g = 0; g < ng; ++g, o += RP * ostep) {
        if (g + NB - 2 < ng) wait_vm<(NB - 2) * K * RP>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (g + NB - 1 < ng) dma(g + NB - 1);
        if (act) {
            float t[RP];
#pragma unroll
            for (int q = 0; q < RP; ++q) {
                const float* rin = hsm + ((g % NB) * RP + q) * BUF + base;
                t[q] = 0.0f;
#pragma unroll
                for (int i = 0; i < KT; ++i) t[q] += rin[i] * w[i];
            }
#pragma unroll
            for (int q = 0; q < RP; ++q) {
                if (g * RP + q < nrows) {  // uniform
                    // the pair read in asm: the compiler cannot tell it from the DMA's LDS targets
                    // and would wait for every DMA in flight (vmcnt(0)) before a plain read
                    const CmapPos cp = colormap_pos(t[q]);
                    uint2 e;
                    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(e) : "v"(lut_lds + 8u * (uint32_t)cp.index));
                    const uint32_t px = colormap_lerp(e, cp.ratio);
                    if (drgb) {
                        uint8_t* ow = o + q * ostep - 3 * lane;  // the wave's first pixel
                        uint32_t dw;
                        asm volatile(
                            "ds_write_b8 %1, %2\n\t"
                            "ds_write_b8 %1, %3 offset:1\n\t"
                            "ds_write_b8 %1, %4 offset:2\n\t"
                            "ds_read_b32 %0, %5\n\t"
                            "s_waitcnt lgkmcnt(0)"
                            : "=&v"(dw)
                            : "v"(stg + 3u * (uint32_t)lane), "v"(px), "v"(px >> 8), "v"(px >> 16),
                              "v"(stg + 4u * (uint32_t)lane)
                            : "memory");
                        if (lane < nd) reinterpret_cast<uint32_t*>(ow)[lane] = dw;
                        if (lane < ntail) {
                            uint32_t b;
                            asm volatile("ds_read_u8 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                                         : "=v"(b) : "v"(stg + 4u * (uint32_t)nd + (uint32_t)lane) : "memory");
                            ow[4 * nd + lane] = (uint8_t)b;
                        }
                    } else {
                        put(o + q * ostep, px);
                    }
                }
            }
        }
    }
}

// the LDS-DMA horizontal pass for a launch (h_taps <= 48, span + taps <= 4 096 floats), else -2
static int launch_resize_h_dma(uint32_t nh, const RenderDesc* d_desc, uint32_t n, uint32_t nw_max, int h_taps,
                               int h_span, const float* tmp, const uint8_t* cmap, uint8_t* rgb, dim3 g3,
                               hipStream_t s) {
    // 8 taps: the groups that upsample along time (Lanczos3's 6-7 taps per column); 10 / 12: the
    // groups that downsample 1.2-2x (9-12 taps)
    const int kt = h_taps <= 8 ? 8 : h_taps <= 10 ? 10 : h_taps <= 12 ? 12 : h_taps <= 16 ? 16
                 : h_taps <= 32 ? 32 : h_taps <= 48 ? 48 : 0;
    if (!kt) return -2;
    const int need = h_span + 4 + kt;
    const int K = need <= 1024 ? 1 : need <= 2048 ? 2 : need <= 4096 ? 4 : 0;
    if (!K) return -2;
    // row buffers (3 and 6 measured slower: 3.40 / 3.42 vs 3.36 ms per C5 step; round 4, 8 for the
    // one-chunk spans: 3.88 vs 3.84 ms, profiles/r04_display/ab_experiments.txt)
    constexpr int NB = 4;
    const int lds = NB * K * 1024 * 4 + 128 + 4 * 192;  // + the colormap pairs, the RGB staging
    const void* kern = nullptr;
#define THESIA_HDMA(KT_, K_) \
    if (kt == KT_ && K == K_) kern = reinterpret_cast<const void*>(resize_h_dma_kernel<KT_, K_, NB>);
    THESIA_HDMA(8, 1) THESIA_HDMA(8, 2) THESIA_HDMA(8, 4)
    THESIA_HDMA(10, 1) THESIA_HDMA(10, 2) THESIA_HDMA(10, 4)
    THESIA_HDMA(12, 1) THESIA_HDMA(12, 2) THESIA_HDMA(12, 4)
    THESIA_HDMA(16, 1) THESIA_HDMA(16, 2) THESIA_HDMA(16, 4)
    THESIA_HDMA(32, 1) THESIA_HDMA(32, 2) THESIA_HDMA(32, 4)
    THESIA_HDMA(48, 1) THESIA_HDMA(48, 2) THESIA_HDMA(48, 4)
#undef THESIA_HDMA
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    void* args[] = {&nh, &d_desc, &tmp, &cmap, &rgb};
    if (hipLaunchKernel(kern, g3, dim3(256), args, lds, s) != hipSuccess) return -1;
    (void)n;
    (void)nw_max;
    return 0;
}

int launch_render_batch2(const float* spec, uint32_t bins, float max, float min,
                         const RenderDesc* d_desc, uint32_t n, uint32_t T_max, uint32_t H_max,
                         uint32_t nw_max, uint32_t nh, int h_taps, int h_span, uint32_t v_band,
                         int v_rows, int v_kv, float* tmp, const uint8_t* cmap, uint8_t* rgb,
                         hipStream_t s, bool h_dma, int v_fpl) {
    if (n == 0 || nh == 0 || v_band == 0) return 0;
    if (n > 65535) return -2;
    (void)H_max;
    const int kv = (v_kv + 3) & ~3;
    if (v_fpl == 4 || v_fpl == 2) {
        // K4+K5v wide: every band's grey rows fit the tile (host: v_rows <= the FPL's cap)
        const int lds1 = grey_vert_wide_lds_bytes(v_fpl, v_band, v_rows, kv);
        if (lds1 > 163840) return -2;
        const void* kern = v_fpl == 4 ? reinterpret_cast<const void*>(grey_vert_wide_kernel<4>)
                                      : reinterpret_cast<const void*>(grey_vert_wide_kernel<2>);
        if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds1) != hipSuccess) return -1;
        const uint32_t fw = 64u * (uint32_t)v_fpl;
        dim3 g1((T_max + fw - 1) / fw, (nh + v_band - 1) / v_band, n);
        int tile_cap = v_rows;
        void* args[] = {&spec, &bins, &max, &min, &nh, &d_desc, &tmp, &tile_cap, const_cast<int*>(&kv), &v_band};
        if (hipLaunchKernel(kern, g1, dim3(256), args, lds1, s) != hipSuccess) return -1;
    } else {
        // K4+K5v: the band's grey tile, meta and zero-padded weights in LDS (a band whose tile
        // does not fit reads HBM directly)
        const int tile_cap = v_rows < 256 ? v_rows : 256;
        const int lds1 = ((((int)v_band + 3) & ~3) + ((tile_cap * 65 + 3) & ~3) + (int)v_band * kv) * 4;
        if (lds1 > 163840) return -2;
        const void* vk = reinterpret_cast<const void*>(grey_vert_kernel);
        if (hipFuncSetAttribute(vk, hipFuncAttributeMaxDynamicSharedMemorySize, lds1) != hipSuccess) return -1;
        dim3 g1((T_max + 63) / 64, (nh + v_band - 1) / v_band, n);
        void* vargs[] = {&spec, &bins, &max, &min, &nh, &d_desc, &tmp, const_cast<int*>(&tile_cap),
                         const_cast<int*>(&kv), &v_band};
        if (hipLaunchKernel(vk, g1, dim3(256), vargs, lds1, s) != hipSuccess) return -1;
    }
    // K5h + K6: the three-stage path's horizontal pass (same intermediate layout [nh][T])
    // row blocks per image: THESIA_RYH, more when few images would leave CUs idle
    uint32_t ry_h = THESIA_RYH;  // (8 rows blocks: same time with the LDS-DMA pass; 32: +4 %)
    const uint32_t nxb = (nw_max + 255) / 256;
    while (ry_h < 128 && (uint64_t)nxb * ry_h * n < 4096) ry_h *= 2;
    dim3 g3(nxb, nh < ry_h ? nh : ry_h, n);
    // register weights up to THESIA_HKT_MAX taps (a downsampling group's 20-48 taps as an LDS
    // weight table took 44 KiB per block: two blocks per CU); more taps: the LDS table
    if (h_dma) {
        const int rc = launch_resize_h_dma(nh, d_desc, n, nw_max, h_taps, h_span, tmp, cmap, rgb, g3, s);
        if (rc != -2) return rc;
    }
    const int kt = h_taps <= 16 ? 16 : h_taps <= 32 && THESIA_HKT_MAX >= 32 ? 32
                 : h_taps <= 48 && THESIA_HKT_MAX >= 48 ? 48 : 16;
    int taps = h_taps > kt ? h_taps : 0;
    int span = h_span;
    // span + zeros, wide weights, RGB segment, colormap; then the second row's span + segment
    auto lds = [&]() { return (2 * (span + kt) + taps * 256) * 4 + 2 * 256 * 3 + 32; };
    if (lds() > 65536) taps = 0;
    if (lds() > 65536) span = 4096;
    auto kern = kt == 48 ? resize_h_rgb_batch_kernel<48>
              : kt == 32 ? resize_h_rgb_batch_kernel<32> : resize_h_rgb_batch_kernel<16>;
    hipLaunchKernelGGL(kern, g3, dim3(256), lds(), s, nh, d_desc, tmp, cmap, rgb, taps, span, 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_resize_h_rgb(const float* in, uint32_t w, uint32_t nh, uint32_t nw,
                        const int32_t* left, const int32_t* cnt, const int32_t* woff,
                        const float* wts, int max_taps, const uint8_t* cmap, uint8_t* out,
                        hipStream_t s) {
    (void)max_taps;
    if (nw == 0 || nh == 0) return 0;
    dim3 grid((nw + 255) / 256, nh);
    hipLaunchKernelGGL(resize_h_rgb_kernel, grid, dim3(256), 0, s, in, w, nh, nw, left, cnt, woff,
                       wts, cmap, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// waveform image (display.rs:63-115)
// ------------------------------------------------------------------------------------
__global__ void wav_upsample_kernel(const float* wav, uint64_t n, uint32_t factor, float* out) {
    const uint64_t total = (uint64_t)factor * n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t q = i / factor, r = i % factor;
        const float b = (q + 1 < n) ? wav[q + 1] : 0.0f;
        out[i] = b * ((float)r / (float)factor) + wav[q] * (1.0f - (float)r / (float)factor);
    }
}

int launch_wav_upsample(const float* wav, uint64_t n, uint32_t factor, float* out, hipStream_t s) {
    const uint64_t total = (uint64_t)factor * n;
    if (total == 0) return 0;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(wav_upsample_kernel, dim3((unsigned)blocks), dim3(256), 0, s, wav, n, factor, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// one thread per pixel column: envelope extent, then paint the column
__global__ void wav_image_kernel(const float* wav, uint64_t wlen, uint32_t nwidth, uint32_t nheight,
                                 float spp, float amp_min, float amp_max, uint8_t* out,
                                 int* panicked) {
    const uint32_t ipx = blockIdx.x * blockDim.x + threadIdx.x;
    if (ipx >= nwidth) return;
    float s = roundf(((float)ipx - 1.5f) * spp);
    s = fmaxf(s, 0.0f);
    const uint64_t i_start = (uint64_t)s;
    const float e = roundf(((float)ipx + 1.5f) * spp);
    uint64_t i_end = e <= 0.0f ? 0 : (uint64_t)e;
    if (i_end > wlen) i_end = wlen;
    for (uint32_t y = 0; y < nheight; ++y) {
        uint8_t* o = out + ((uint64_t)y * nwidth + ipx) * 4;
        o[0] = 0; o[1] = 0; o[2] = 0; o[3] = 0;
    }
    if (i_start >= i_end) { atomicOr(panicked, 1); return; }
    float mx = wav[i_start], mn = wav[i_start];
    bool nan = false;
    for (uint64_t i = i_start; i < i_end; ++i) {
        const float v = wav[i];
        if (v != v) nan = true;
        if (v > mx) mx = v;
        if (v < mn) mn = v;
    }
    if (nan) { atomicOr(panicked, 1); return; }
    const float fh = (float)nheight, rng = amp_max - amp_min;
    long long top = (long long)roundf((amp_max - mx) * fh / rng);
    long long bottom = (long long)roundf((amp_max - mn) * fh / rng);
    if (bottom - top < 3) {
        const float d = (float)(3 - bottom + top) / 2.0f;
        const long long pad_bottom = (long long)ceilf(d), pad_top = (long long)floorf(d);
        top -= pad_top;
        bottom += pad_bottom;
    }
    if (top < 0) top = 0;
    if (bottom > (long long)nheight) bottom = (long long)nheight;
    if (bottom + 1 > (long long)nheight) { atomicOr(panicked, 1); bottom = (long long)nheight - 1; }
    if (top > bottom + 1) { atomicOr(panicked, 1); return; }
    for (long long y = top; y <= bottom; ++y) {
        uint8_t* o = out + ((uint64_t)y * nwidth + ipx) * 4;
        o[0] = 200; o[1] = 21; o[2] = 103; o[3] = 255;  // WAVECOLOR display.rs:22
    }
}

int launch_wav_image(const float* wav, uint64_t n, const float* wav_up, uint64_t n_up,
                     uint32_t nwidth, uint32_t nheight, float spp, float amp_min, float amp_max,
                     uint8_t* out, int* panicked, hipStream_t s) {
    if (nwidth == 0) return 0;
    const float* src = wav_up ? wav_up : wav;
    const uint64_t len = wav_up ? n_up : n;
    hipLaunchKernelGGL(wav_image_kernel, dim3((nwidth + 127) / 128), dim3(128), 0, s, src, len,
                       nwidth, nheight, spp, amp_min, amp_max, out, panicked);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------------------
// deterministic integer PCM generator (bench / tests): chirp from an int16 sine LUT with a
// 64-bit fixed-point phase, plus Irwin-Hall noise from a splitmix64 hash. Host and device
// produce identical int16 samples (host twin in engine.cpp).
// ------------------------------------------------------------------------------------
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__host__ __device__ inline int16_t synth_sample(uint64_t track, uint32_t ch, uint64_t i,
                                                uint64_t ph_a, uint64_t ph_b, uint64_t seed,
                                                const int16_t* lut /*4096*/) {
    // chirp phase in Q64 turns: ph = A*i + B*i^2 (mod 2^64), A, B from synth_phase_coeffs()
    const uint64_t ph = ph_a * i + ph_b * (i * i);
    const int32_t chirp = lut[ph >> 52] / 4;  // 0.25 full scale
    const uint64_t h = splitmix64(seed ^ splitmix64(track * 0x100000001B3ull + ch) ^ (i * 0xD6E8FEB86659FD93ull));
    // Irwin-Hall (4 x 16-bit uniforms): mean 2*65535, sd ~ 37837 -> scale to ~0.05 FS
    const int64_t u = (int64_t)(h & 0xFFFF) + (int64_t)((h >> 16) & 0xFFFF) +
                      (int64_t)((h >> 32) & 0xFFFF) + (int64_t)((h >> 48) & 0xFFFF) - 131070;
    const int64_t noise = (u * 1638) / 37837;
    int64_t v = (int64_t)chirp + noise;
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    return (int16_t)v;
}

__global__ void synth_kernel(void* out, int out_format, uint32_t C, uint64_t n_tracks,
                             uint64_t n, uint64_t ph_a, uint64_t ph_b, uint64_t seed,
                             const int16_t* lut) {
    const uint64_t total = n_tracks * n * C;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t track = e / (n * C);
        const uint64_t rem = e % (n * C);
        const uint64_t i = rem / C;
        const uint32_t ch = (uint32_t)(rem % C);
        const int16_t v = synth_sample(track, ch, i, ph_a, ph_b, seed, lut);
        if (out_format == IN_S16) static_cast<int16_t*>(out)[e] = v;
        else static_cast<float*>(out)[e] = (float)v / 32768.0f;
    }
}

void synth_phase_coeffs(uint64_t n, uint32_t sr, uint64_t* ph_a, uint64_t* ph_b) {
    // f(t) sweeps 50 Hz -> 0.45 sr linearly over the track: phase(i) = a*i + b*i^2 turns
    const double f0 = 50.0, f1 = 0.45 * (double)sr;
    const double b = (f1 - f0) / (2.0 * (double)n * (double)sr);
    const double a = f0 / (double)sr - b;
    const double two64 = 18446744073709551616.0;
    *ph_a = (uint64_t)(int64_t)(a * two64 / 4.0) * 4u;
    *ph_b = (uint64_t)(b * two64);
}

int launch_synth_pcm(void* out, int out_format, uint32_t channels, uint64_t n_tracks,
                     uint64_t n_samples, uint32_t sr, uint64_t seed, const int16_t* sine_lut,
                     hipStream_t s) {
    uint64_t pa = 0, pb = 0;
    synth_phase_coeffs(n_samples, sr, &pa, &pb);
    hipLaunchKernelGGL(synth_kernel, dim3(16384), dim3(256), 0, s, out, out_format, channels,
                       n_tracks, n_samples, pa, pb, seed, sine_lut);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace thesia

// host twin of the generator (same integer arithmetic)
namespace thesia {
void synth_host(int16_t* out, uint32_t C, uint64_t track, uint64_t n, uint32_t sr, uint64_t seed,
                const int16_t* lut) {
    uint64_t pa = 0, pb = 0;
    synth_phase_coeffs(n, sr, &pa, &pb);
    for (uint64_t i = 0; i < n; ++i)
        for (uint32_t c = 0; c < C; ++c) out[i * C + c] = synth_sample(track, c, i, pa, pb, seed, lut);
}
}  // namespace thesia
