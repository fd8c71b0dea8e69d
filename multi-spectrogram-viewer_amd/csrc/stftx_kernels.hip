// stftx_kernels.hip -- the reference-order STFT ("exact" kernel, batch kernel 9): every f32
// operation of the reference path in the reference's order, so the device result is the
// oracle's bit for bit.
//
// What the fast kernels (stft3/stft5, stft2, stft) reorder, this one does not:
//   framing / window  x_ref[...] * w[k], zero outside the window            lib.rs:367-435
//   real FFT          rustfft 4.0 Radix4 as restated by the oracle            realfft.rs:126-138
//                     (oracle/thesia_oracle.c cfft_tab: prepare_radix4 digit order, base
//                     butterfly_4 / butterfly_8, radix-4 passes with table twiddles), products as
//                     num-complex Mul (no fused multiply-add anywhere: -ffp-contract=off)
//   untangle          realfft.rs:140-157 expression by expression
//   |X|, |X|^2        hypotf (num-complex norm -> glibc, exact_math.hpp), re*re + im*im
//   mel               lib.rs:131 as the oracle's dot: one k-ascending fma chain per mel
//   dB                decibel.rs:49-55 / :65 / :75 with glibc 2.35 log10f (exact_math.hpp)
// Downstream (grey, Lanczos3, colormap) is bit-exact already, so MultiTrack images from this
// kernel equal the oracle pipeline's bytes (tests/test_gpu_exact.py).
//
// Layout: one wave per frame, 4 waves per block. The frame's NC complex points live in the
// wave's LDS buffer, loaded straight into their prepare_radix4 positions (host table xpos);
// a butterfly per lane per step, wave-level LDS syncs between passes. Throughput is secondary
// here (the viewer path: a few tracks); the batch engine's fast kernels stay the default.
#include "exact_math.hpp"
#include "stft_common.hpp"

namespace thesia {

namespace {

constexpr int kXWaves = 4;
constexpr int kXMagRegs = 17;  // |X| values per lane held in registers (F <= 1088: n_fft <= 2048)

struct Cx {
    float re, im;
};
__device__ __forceinline__ Cx xadd(Cx a, Cx b) { return Cx{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ Cx xsub(Cx a, Cx b) { return Cx{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ Cx xmul(Cx a, Cx b) {  // num-complex Mul
    return Cx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ Cx xrot90(Cx v) { return Cx{v.im, -v.re}; }  // forward: * (-i)
__device__ __forceinline__ void xbfly2(Cx& a, Cx& b) {
    const Cx t = xadd(a, b);
    b = xsub(a, b);
    a = t;
}
__device__ __forceinline__ void xbfly4(Cx* buf) {
    Cx v0 = buf[0], v1 = buf[1], v2 = buf[2], v3 = buf[3];
    xbfly2(v0, v2);
    xbfly2(v1, v3);
    v3 = xrot90(v3);
    xbfly2(v0, v1);
    xbfly2(v2, v3);
    buf[0] = v0; buf[1] = v2; buf[2] = v1; buf[3] = v3;
}
__device__ __forceinline__ void xbfly8(Cx* buf, Cx w1, Cx w3) {
    Cx s[8] = {buf[0], buf[2], buf[4], buf[6], buf[1], buf[3], buf[5], buf[7]};
    xbfly4(s);
    xbfly4(s + 4);
    s[5] = xmul(s[5], w1);
    s[6] = xrot90(s[6]);
    s[7] = xmul(s[7], w3);
    for (int i = 0; i < 4; ++i) xbfly2(s[i], s[i + 4]);
    for (int i = 0; i < 8; ++i) buf[i] = s[i];
}

__device__ __forceinline__ float xdb(float x, float log_amin, float amin, float factor) {
    // decibel.rs:49-55 (ref 1: log_ref = 0, so y - 0 is y) then the separate factor pass
    const float y = x > amin ? exact::log10f_glibc(x) - 0.0f : log_amin - 0.0f;
    return factor * y;
}

}  // namespace

template <int INF>
__global__ void __launch_bounds__(64 * kXWaves)
stftx_kernel(StftLaunch a) {
    const int NC = a.n_fft / 2;
    const int F = NC + 1;
    const int bufl = (NC + 3) & ~3;  // complex points (realfft.rs:140's buf[NC] = buf[0]: read
                                     // through the index mod NC below)
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Cx* buf = reinterpret_cast<Cx*>(xs) + (size_t)wave * bufl;
    // the |X| row (mel kinds): in the frame's own buffer once the untangle has read it (NC <=
    // kXMagRegs x 64 - 1: the row goes through registers), else a row of its own after the
    // buffers (the other kinds' launches carry no room for it)
    float* mag = NC < 64 * kXMagRegs ? reinterpret_cast<float*>(buf)
                                     : xs + (size_t)kXWaves * bufl * 2 + (size_t)wave * ((F + 3) & ~3);
    const uint64_t g = (uint64_t)blockIdx.x * kXWaves + wave;
    if (g >= a.total_frames) return;  // wave-uniform; no block barrier below

    const int trk = find_track(a.trk_frame0, a.n_tracks, g, -1);
    const uint64_t g_beg = a.trk_frame0[trk];
    const int64_t n = (int64_t)a.trk_len[trk];
    const uint64_t base = a.trk_in_off[trk];
    const int64_t start = (int64_t)(g - g_beg) * a.hop - a.win / 2 - a.pad_left;
    const bool fold = a.fold != 0;

    // ---- the frame (lib.rs:378-383: x_ref slice * window, zero padded to n_fft), complex
    // point m = (x_2m, x_2m+1) stored at its prepare_radix4 position ----
    auto sample = [&](int jj) -> float {
        if (jj < a.pad_left || jj >= a.pad_left + a.win) return 0.0f;
        int64_t i = start + jj;
        if (i < 0) i = -i;
        if (i > n - 1) i = 2 * (n - 1) - i;
        i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
        return read_sample<INF>(a.in, base, i, a.channels, fold) * a.wpad[jj];
    };
    for (int m = lane; m < NC; m += 64) {
        const int pos = NC > 4 ? a.xpos[m] : m;
        buf[pos] = Cx{sample(2 * m), sample(2 * m + 1)};
    }
    wave_lds_sync();

    // ---- rustfft Radix4 (oracle cfft_tab) ----
    const Cx* tw = reinterpret_cast<const Cx*>(a.tw1);  // twiddle(i, NC), f64-evaluated
    if (NC == 2) {
        if (lane == 0) xbfly2(buf[0], buf[1]);
    } else if (NC == 4) {
        if (lane == 0) xbfly4(buf);
    } else if (NC >= 8) {
        int bits = 0;
        while ((1 << bits) < NC) ++bits;
        int cur;
        if (bits % 2 == 0) {
            for (int c = 4 * lane; c < NC; c += 256) xbfly4(buf + c);
            cur = 16;
        } else {
            const Cx w1 = Cx{a.xw8[0], a.xw8[1]}, w3 = Cx{a.xw8[2], a.xw8[3]};
            for (int c = 8 * lane; c < NC; c += 512) xbfly8(buf + c, w1, w3);
            cur = 32;
        }
        for (; cur <= NC; cur *= 4) {
            wave_lds_sync();
            const int q = cur / 4, tstride = NC / cur;
            const int lq = __builtin_ctz((unsigned)q);  // q, cur: powers of two (no divisions)
            for (int b = lane; b < NC / 4; b += 64) {
                const int row = b >> lq, j = b & (q - 1);
                Cx* d = buf + (size_t)row * cur;
                // rustfft butterfly_4, forward (oracle cfft_tab)
                const Cx s0 = xmul(d[j + q], tw[j * 1 * tstride]);
                const Cx s1 = xmul(d[j + 2 * q], tw[j * 2 * tstride]);
                const Cx s2 = xmul(d[j + 3 * q], tw[j * 3 * tstride]);
                const Cx s5 = xsub(d[j], s1);
                Cx d0 = xadd(d[j], s1);
                const Cx s3 = xadd(s0, s2);
                const Cx s4 = xsub(s0, s2);
                d[j + 2 * q] = xsub(d0, s3);
                d0 = xadd(d0, s3);
                d[j] = d0;
                d[j + q] = Cx{s5.re + s4.im, s5.im - s4.re};
                d[j + 3 * q] = Cx{s5.re - s4.im, s5.im + s4.re};
            }
        }
    }
    wave_lds_sync();

    // ---- realfft untangle (realfft.rs:142-157) and the output kind ----
    const int kind = a.out_kind;
    const float2* sc = a.sincos;
    auto bin = [&](int k) -> Cx {
        if (k == NC) return Cx{buf[0].re - buf[0].im, 0.0f};
        const float s = sc[k].x, c = sc[k].y;
        const Cx b = buf[k], r = buf[(NC - k) & (NC - 1)];  // k = 0: buf[NC] = buf[0]
        const float xr = 0.5f * (((b.re + r.re) + c * (b.im + r.im)) - s * (b.re - r.re));
        const float xi = 0.5f * (((b.im - r.im) - s * (b.im + r.im)) - c * (b.re - r.re));
        return Cx{xr, xi};
    };
    if (kind == OUT_COMPLEX) {
        float2* row = reinterpret_cast<float2*>(a.out) + g * (uint64_t)F;
        for (int k = lane; k < F; k += 64) {
            const Cx x = bin(k);
            row[k] = make_float2(x.re, x.im);
        }
        return;
    }
    const bool mel = kind == OUT_MEL || kind == OUT_MEL_AMP_DB;
    const bool power = kind == OUT_POWER || kind == OUT_POWER_DB;
    const bool db = kind == OUT_AMP_DB || kind == OUT_POWER_DB || kind == OUT_MEL_AMP_DB;
    if (!mel) {
        float* row = static_cast<float*>(a.out) + g * (uint64_t)F;
        for (int k = lane; k < F; k += 64) {
            const Cx x = bin(k);
            float v = power ? x.re * x.re + x.im * x.im : exact::hypotf_glibc(x.re, x.im);
            if (db) v = power ? xdb(v, a.log_amin, 1e-36f, 10.0f) : xdb(v, a.log_amin, 1e-18f, 20.0f);
            row[k] = v;
        }
        return;
    }
    if (NC < 64 * kXMagRegs) {
        float mr[kXMagRegs];
#pragma unroll
        for (int i = 0; i < kXMagRegs; ++i) {
            const int k = lane + 64 * i;
            if (k < F) {
                const Cx x = bin(k);
                mr[i] = exact::hypotf_glibc(x.re, x.im);
            }
        }
        wave_lds_sync();  // every lane's untangle reads are done: the buffer takes the row
#pragma unroll
        for (int i = 0; i < kXMagRegs; ++i)
            if (lane + 64 * i < F) mag[lane + 64 * i] = mr[i];
    } else {
        for (int k = lane; k < F; k += 64) {
            const Cx x = bin(k);
            mag[k] = exact::hypotf_glibc(x.re, x.im);
        }
    }
    wave_lds_sync();
    // lib.rs:131: out[m] = fma chain over k ascending of |X|[k] * fb[k][m] (the oracle's dot);
    // terms outside the filter's nonzero band are fma(x, 0, acc) = acc and are skipped
    float* row = static_cast<float*>(a.out) + g * (uint64_t)a.n_mels;
    for (int m = lane; m < a.n_mels; m += 64) {
        const int4 bd = a.xmel_band[m];  // {first bin, bins, weight offset}
        float acc = 0.0f;
        // unrolled: the weight reads (global) of 8 taps issue ahead of their fma chain
#pragma unroll 8
        for (int t = 0; t < bd.y; ++t) acc = __builtin_fmaf(mag[bd.x + t], a.xmel_w[bd.z + t], acc);
        row[m] = db ? xdb(acc, a.log_amin, 1e-18f, 20.0f) : acc;
    }
}

// ------------------------------------------------------------------------------------
// InvRealFFT (realfft.rs:167-241): spectrum of NC+1 bins -> 2*NC real samples, unnormalised
// (the reference's complex_to_real test: 0.5 * Re(full inverse DFT)). Same structure as
// stftx: one wave per frame; the realfft pre-twiddle (realfft.rs:210-219) written straight to
// the prepare_radix4 positions, then rustfft 4.0 Radix4 with inverse = true: conjugated
// twiddles (compute_twiddle(..).conj(), exact), rotate_90 by +i, and butterfly_4's inverse
// output pair; the complex result is the real output, pairs interleaved (realfft.rs:225-230).
// ------------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ Cx xconj(Cx a) { return Cx{a.re, -a.im}; }
__device__ __forceinline__ Cx xrot90i(Cx v) { return Cx{-v.im, v.re}; }  // inverse: * (+i)
__device__ __forceinline__ void xbfly4i(Cx* buf) {
    Cx v0 = buf[0], v1 = buf[1], v2 = buf[2], v3 = buf[3];
    xbfly2(v0, v2);
    xbfly2(v1, v3);
    v3 = xrot90i(v3);
    xbfly2(v0, v1);
    xbfly2(v2, v3);
    buf[0] = v0; buf[1] = v2; buf[2] = v1; buf[3] = v3;
}
__device__ __forceinline__ void xbfly8i(Cx* buf, Cx w1, Cx w3) {
    Cx s[8] = {buf[0], buf[2], buf[4], buf[6], buf[1], buf[3], buf[5], buf[7]};
    xbfly4i(s);
    xbfly4i(s + 4);
    s[5] = xmul(s[5], w1);
    s[6] = xrot90i(s[6]);
    s[7] = xmul(s[7], w3);
    for (int i = 0; i < 4; ++i) xbfly2(s[i], s[i + 4]);
    for (int i = 0; i < 8; ++i) buf[i] = s[i];
}
}  // namespace

__global__ void __launch_bounds__(64 * kXWaves)
irfftx_kernel(const float2* in, uint64_t n_frames, int NC, const int* xpos, const float2* tw1,
              const float2* sincos, float4 w8, float* out) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int bufl = (NC + 3) & ~3;
    Cx* buf = reinterpret_cast<Cx*>(xs) + (size_t)wave * bufl;
    const uint64_t g = (uint64_t)blockIdx.x * kXWaves + wave;
    if (g >= n_frames) return;  // wave-uniform; no block barrier below
    const float2* X = in + g * (uint64_t)(NC + 1);
    // realfft.rs:210-219 (zip4 of input, input.rev(), sin_cos, buffer_in: k = 0 .. NC-1)
    for (int k = lane; k < NC; k += 64) {
        const float2 b = X[k], r = X[NC - k];
        const float s = sincos[k].x, c = sincos[k].y;
        const float xr = 0.5f * (((b.x + r.x) - c * (b.y + r.y)) - s * (b.x - r.x));
        const float xi = 0.5f * (((b.y - r.y) + c * (b.x - r.x)) - s * (b.y + r.y));
        buf[NC > 4 ? xpos[k] : k] = Cx{xr, xi};
    }
    wave_lds_sync();
    if (NC == 2) {
        if (lane == 0) xbfly2(buf[0], buf[1]);
    } else if (NC == 4) {
        if (lane == 0) xbfly4i(buf);
    } else if (NC >= 8) {
        const Cx* tw = reinterpret_cast<const Cx*>(tw1);  // forward twiddle(i, NC); conjugated below
        int bits = 0;
        while ((1 << bits) < NC) ++bits;
        int cur;
        if (bits % 2 == 0) {
            for (int c = 4 * lane; c < NC; c += 256) xbfly4i(buf + c);
            cur = 16;
        } else {
            const Cx w1 = xconj(Cx{w8.x, w8.y}), w3 = xconj(Cx{w8.z, w8.w});
            for (int c = 8 * lane; c < NC; c += 512) xbfly8i(buf + c, w1, w3);
            cur = 32;
        }
        for (; cur <= NC; cur *= 4) {
            wave_lds_sync();
            const int q = cur / 4, tstride = NC / cur;
            const int lq = __builtin_ctz((unsigned)q);  // q, cur: powers of two (no divisions)
            for (int b = lane; b < NC / 4; b += 64) {
                const int row = b >> lq, j = b & (q - 1);
                Cx* d = buf + (size_t)row * cur;
                // rustfft butterfly_4, inverse
                const Cx s0 = xmul(d[j + q], xconj(tw[j * 1 * tstride]));
                const Cx s1 = xmul(d[j + 2 * q], xconj(tw[j * 2 * tstride]));
                const Cx s2 = xmul(d[j + 3 * q], xconj(tw[j * 3 * tstride]));
                const Cx s5 = xsub(d[j], s1);
                Cx d0 = xadd(d[j], s1);
                const Cx s3 = xadd(s0, s2);
                const Cx s4 = xsub(s0, s2);
                d[j + 2 * q] = xsub(d0, s3);
                d0 = xadd(d0, s3);
                d[j] = d0;
                d[j + q] = Cx{s5.re - s4.im, s5.im + s4.re};
                d[j + 3 * q] = Cx{s5.re + s4.im, s5.im - s4.re};
            }
        }
    }
    wave_lds_sync();
    float2* o = reinterpret_cast<float2*>(out + g * (uint64_t)(2 * NC));
    for (int m = lane; m < NC; m += 64) o[m] = make_float2(buf[m].re, buf[m].im);
}

int launch_irfftx(const float* in, uint64_t n_frames, int length, const int* xpos, const float* tw1,
                  const float* sincos, const float* xw8, float* out, hipStream_t s) {
    if (length < 2 || (length & (length - 1))) return -2;
    const int NC = length / 2;
    const int lds = kXWaves * ((NC + 3) & ~3) * 8;
    if (lds > 163840) return -2;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(irfftx_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
    if (n_frames == 0) return 0;
    const uint64_t blocks = (n_frames + kXWaves - 1) / kXWaves;
    if (blocks > 0x7fffffffULL) return -2;
    hipLaunchKernelGGL(irfftx_kernel, dim3((unsigned)blocks), dim3(64 * kXWaves), lds, s,
                       reinterpret_cast<const float2*>(in), n_frames, NC, xpos,
                       reinterpret_cast<const float2*>(tw1), reinterpret_cast<const float2*>(sincos),
                       make_float4(xw8[0], xw8[1], xw8[2], xw8[3]), out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int stftx_lds_bytes(int n_fft, bool mel) {
    const int NC = n_fft / 2, F = NC + 1;
    const int bufl = (NC + 3) & ~3;
    return kXWaves * (bufl * 8 + (mel && NC >= 64 * kXMagRegs ? ((F + 3) & ~3) * 4 : 0));
}

int launch_stftx(const StftLaunch& a, hipStream_t s) {
    if (a.n_fft < 2 || (a.n_fft & (a.n_fft - 1))) return -2;
    // a separate |X| row only for the mel kinds at n_fft 4096: otherwise a frame's wave takes
    // 8 KiB at n_fft 2048 (16 waves per CU instead of 12)
    const int lds = stftx_lds_bytes(a.n_fft, a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB);
    if (lds > 163840) return -2;
    auto kern = a.in_format == IN_S16 ? stftx_kernel<IN_S16> : stftx_kernel<IN_F32>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    const uint64_t blocks = (a.total_frames + kXWaves - 1) / kXWaves;
    if (blocks > 0x7fffffffULL) return -2;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * kXWaves), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace thesia
