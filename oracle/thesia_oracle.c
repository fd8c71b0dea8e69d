/*
 * thesia_oracle.c -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Parity checker for the MI355X engine; never linked into the product, never measured as
 * the product. See thesia_oracle.h for the pinning status of every function.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off). All citations are to
 * /root/reference/src_rust/ unless stated.
 */
#include "thesia_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------------------------ */
/* windows.rs:7-30 cosine_window / hann                                                  */
/* ------------------------------------------------------------------------------------ */
void or_hann_f32(size_t size, int symmetric, float* out) {
    /* windows.rs:8 pi = T::from(PI f64); size2 = size (symmetric) or size+1 */
    const float pi = (float)M_PI;
    const size_t size2 = symmetric ? size : size + 1;
    const float a = 0.5f, b = 0.5f, c = 0.0f, d = 0.0f;
    for (size_t i = 0; i < size; ++i) {
        /* windows.rs:12: x = pi * i / (size2 - 1)  (left to right) */
        float x = pi * (float)i / (float)(size2 - 1);
        float b_ = b * cosf(2.0f * x);
        float c_ = c * cosf(4.0f * x);
        float d_ = d * cosf(6.0f * x);
        out[i] = (a - b_) + (c_ - d_); /* windows.rs:16 */
    }
}

void or_hann_f64(size_t size, int symmetric, double* out) {
    const double pi = M_PI;
    const size_t size2 = symmetric ? size : size + 1;
    for (size_t i = 0; i < size; ++i) {
        double x = pi * (double)i / (double)(size2 - 1);
        double b_ = 0.5 * cos(2.0 * x);
        double c_ = 0.0 * cos(4.0 * x);
        double d_ = 0.0 * cos(6.0 * x);
        out[i] = (0.5 - b_) + (c_ - d_);
    }
}

/* ------------------------------------------------------------------------------------ */
/* utils.rs                                                                             */
/* ------------------------------------------------------------------------------------ */
size_t or_calc_proper_n_fft(size_t win_length) {
    /* utils.rs:17-19: 2usize.pow((win_length as f32).log2().ceil() as u32) */
    float e = ceilf(log2f((float)win_length));
    unsigned ue = e > 0.0f ? (unsigned)e : 0u;
    return (size_t)1 << ue;
}

int or_pad_constant_f32(const float* x, size_t n, size_t left, size_t right, float c, float* out) {
    /* utils.rs:63-71: concatenate![axis, pad_left, array, pad_right] */
    for (size_t i = 0; i < left; ++i) out[i] = c;
    memcpy(out + left, x, n * sizeof(float));
    for (size_t i = 0; i < right; ++i) out[left + n + i] = c;
    return 0;
}

int or_pad_reflect_f32(const float* x, size_t n, size_t left, size_t right, float* out) {
    /* utils.rs:72-78: s_left = Slice(1, left+1, -1) -> x[1..=left] reversed;
     * s_right = Slice(-(right+1), -1, -1) -> x[n-1-right .. n-1) reversed.
     * ndarray panics when a slice bound exceeds the axis length. */
    if (left + 1 > n || right + 1 > n) return -1;
    for (size_t i = 0; i < left; ++i) out[i] = x[left - i];
    memcpy(out + left, x, n * sizeof(float));
    for (size_t i = 0; i < right; ++i) out[left + n + i] = x[n - 2 - i];
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* rustfft 4.0 Radix4 (third-party, restated) + realfft.rs                               */
/* Twiddles follow rustfft twiddles::single_twiddle (f64 cos/sin of -2*pi*i/len).       */
/* The exact rustfft butterfly op order is not reproducible here (no toolchain): parity */
/* for the FFT is by tolerance.                                             */
/* ------------------------------------------------------------------------------------ */
/* The twiddles every butterfly uses come from a table built once per length (tw[i] =
 * twiddle(i, len), i < len): the values are the ones the butterflies would compute inline, so
 * planned and unplanned transforms are bit-identical. RealFFT::new (realfft.rs:80-101) builds
 * the Radix4 plan (its twiddles) and the sin_cos table once; the reference reuses one plan per
 * track on its multi-track path (lib.rs:459-467) and re-plans per frame only when a single
 * track is added (lib.rs:449-458). */
#define DEFINE_FFT(T, SUF)                                                                   \
    typedef struct { T re, im; } cx_##SUF;                                                   \
    static inline cx_##SUF cadd_##SUF(cx_##SUF a, cx_##SUF b) {                              \
        cx_##SUF r = {a.re + b.re, a.im + b.im}; return r; }                                 \
    static inline cx_##SUF csub_##SUF(cx_##SUF a, cx_##SUF b) {                              \
        cx_##SUF r = {a.re - b.re, a.im - b.im}; return r; }                                 \
    static inline cx_##SUF cmul_##SUF(cx_##SUF a, cx_##SUF b) { /* num-complex Mul */        \
        cx_##SUF r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; return r; }     \
    static inline cx_##SUF rot90_##SUF(cx_##SUF v) { /* forward: multiply by -i */           \
        cx_##SUF r = {v.im, -v.re}; return r; }                                              \
    static inline cx_##SUF twiddle_##SUF(size_t i, size_t len) {                             \
        double ang = -2.0 * M_PI * (double)i / (double)len;                                  \
        cx_##SUF r = {(T)cos(ang), (T)sin(ang)}; return r; }                                 \
    static inline void bfly2_##SUF(cx_##SUF* a, cx_##SUF* b) {                               \
        cx_##SUF t = cadd_##SUF(*a, *b); *b = csub_##SUF(*a, *b); *a = t; }                  \
    static void bfly4_##SUF(cx_##SUF* buf) {                                                 \
        cx_##SUF v0 = buf[0], v1 = buf[1], v2 = buf[2], v3 = buf[3];                         \
        bfly2_##SUF(&v0, &v2); bfly2_##SUF(&v1, &v3);                                        \
        v3 = rot90_##SUF(v3);                                                                \
        bfly2_##SUF(&v0, &v1); bfly2_##SUF(&v2, &v3);                                        \
        buf[0] = v0; buf[1] = v2; buf[2] = v1; buf[3] = v3; }                                \
    static void bfly8_##SUF(cx_##SUF* buf, cx_##SUF w1, cx_##SUF w3) {                       \
        cx_##SUF s[8] = {buf[0], buf[2], buf[4], buf[6], buf[1], buf[3], buf[5], buf[7]};    \
        bfly4_##SUF(s); bfly4_##SUF(s + 4);                                                  \
        s[5] = cmul_##SUF(s[5], w1);                       /* twiddle(1, 8) */               \
        s[6] = rot90_##SUF(s[6]);                                                            \
        s[7] = cmul_##SUF(s[7], w3);                       /* twiddle(3, 8) */               \
        for (int i = 0; i < 4; ++i) bfly2_##SUF(&s[i], &s[i + 4]);                           \
        for (int i = 0; i < 8; ++i) buf[i] = s[i]; }                                         \
    static void prepare_radix4_##SUF(size_t size, const cx_##SUF* sig, cx_##SUF* spec,       \
                                     size_t stride) {                                        \
        if (size == 16) {                                                                    \
            for (size_t i = 0; i < 4; ++i)                                                   \
                prepare_radix4_##SUF(4, sig + i * stride, spec + i * 4, stride * 4);         \
        } else if (size == 8 || size == 4) {                                                 \
            for (size_t i = 0; i < size; ++i) spec[i] = sig[i * stride];                     \
        } else {                                                                             \
            for (size_t i = 0; i < 4; ++i)                                                   \
                prepare_radix4_##SUF(size / 4, sig + i * stride, spec + i * (size / 4),      \
                                     stride * 4);                                            \
        }                                                                                    \
    }                                                                                        \
    /* tw: [len] twiddle(i, len); w8: {twiddle(1, 8), twiddle(3, 8)} */                      \
    static void cfft_tab_##SUF(const cx_##SUF* in, size_t len, cx_##SUF* out,                \
                               const cx_##SUF* tw, const cx_##SUF* w8) {                     \
        if (len == 1) { out[0] = in[0]; return; }                                            \
        if (len == 2) { out[0] = in[0]; out[1] = in[1]; bfly2_##SUF(&out[0], &out[1]); return; } \
        if (len == 4) { memcpy(out, in, 4 * sizeof(cx_##SUF)); bfly4_##SUF(out); return; }   \
        prepare_radix4_##SUF(len, in, out, 1);                                               \
        unsigned bits = 0; while (((size_t)1 << bits) < len) ++bits;                         \
        size_t cur;                                                                          \
        if (bits % 2 == 0) { for (size_t c = 0; c < len; c += 4) bfly4_##SUF(out + c); cur = 16; } \
        else { for (size_t c = 0; c < len; c += 8) bfly8_##SUF(out + c, w8[0], w8[1]); cur = 32; } \
        for (; cur <= len; cur *= 4) {                                                       \
            size_t q = cur / 4, tstride = len / cur;                                         \
            for (size_t row = 0; row < len / cur; ++row) {                                   \
                cx_##SUF* d = out + row * cur;                                               \
                for (size_t j = 0; j < q; ++j) { /* rustfft butterfly_4, forward */          \
                    cx_##SUF s0 = cmul_##SUF(d[j + q], tw[j * 1 * tstride]);                 \
                    cx_##SUF s1 = cmul_##SUF(d[j + 2 * q], tw[j * 2 * tstride]);             \
                    cx_##SUF s2 = cmul_##SUF(d[j + 3 * q], tw[j * 3 * tstride]);             \
                    cx_##SUF s5 = csub_##SUF(d[j], s1);                                      \
                    d[j] = cadd_##SUF(d[j], s1);                                             \
                    cx_##SUF s3 = cadd_##SUF(s0, s2);                                        \
                    cx_##SUF s4 = csub_##SUF(s0, s2);                                        \
                    d[j + 2 * q] = csub_##SUF(d[j], s3);                                     \
                    d[j] = cadd_##SUF(d[j], s3);                                             \
                    d[j + q].re = s5.re + s4.im; d[j + q].im = s5.im - s4.re;                \
                    d[j + 3 * q].re = s5.re - s4.im; d[j + 3 * q].im = s5.im + s4.re;        \
                }                                                                            \
            }                                                                                \
        }                                                                                    \
    }                                                                                        \
    /* RealFFT::new (realfft.rs:80-101): Radix4 twiddles of length n/2, sin_cos table */     \
    typedef struct { size_t n, half; cx_##SUF* tw; cx_##SUF w8[2]; T* sn; T* cs; cx_##SUF* buf; } plan_##SUF; \
    static plan_##SUF* plan_new_##SUF(size_t n) {                                            \
        if (n % 2 || n < 2) return NULL;                                                     \
        size_t half = n / 2;                                                                 \
        if (half & (half - 1)) return NULL; /* Radix4 asserts a power of two */              \
        plan_##SUF* p = (plan_##SUF*)calloc(1, sizeof(plan_##SUF));                          \
        p->n = n; p->half = half;                                                            \
        p->tw = (cx_##SUF*)malloc(half * sizeof(cx_##SUF));                                  \
        for (size_t i = 0; i < half; ++i) p->tw[i] = twiddle_##SUF(i, half);                 \
        p->w8[0] = twiddle_##SUF(1, 8); p->w8[1] = twiddle_##SUF(3, 8);                      \
        p->sn = (T*)malloc(half * sizeof(T)); p->cs = (T*)malloc(half * sizeof(T));          \
        const T pi = (T)M_PI; const T halflen = (T)half;                                     \
        for (size_t k = 0; k < half; ++k) {           /* realfft.rs:88-93 */                 \
            T ang = (T)k * pi / halflen;                                                     \
            p->sn[k] = SUF##_sin(ang); p->cs[k] = SUF##_cos(ang);                            \
        }                                                                                    \
        p->buf = (cx_##SUF*)malloc((half + 1) * sizeof(cx_##SUF));                           \
        return p;                                                                            \
    }                                                                                        \
    static void plan_free_##SUF(plan_##SUF* p) {                                             \
        if (!p) return;                                                                      \
        free(p->tw); free(p->sn); free(p->cs); free(p->buf); free(p);                        \
    }                                                                                        \
    int or_cfft_radix4_##SUF(const T* in, size_t len, T* out) {                              \
        if (len == 0 || (len & (len - 1))) return -1;                                        \
        cx_##SUF* tw = (cx_##SUF*)malloc(len * sizeof(cx_##SUF));                            \
        for (size_t i = 0; i < len; ++i) tw[i] = twiddle_##SUF(i, len);                      \
        cx_##SUF w8[2] = {twiddle_##SUF(1, 8), twiddle_##SUF(3, 8)};                         \
        cfft_tab_##SUF((const cx_##SUF*)in, len, (cx_##SUF*)out, tw, w8);                    \
        free(tw);                                                                            \
        return 0;                                                                            \
    }                                                                                        \
    /* realfft.rs:105-159 RealFFT::process with a plan */                                    \
    static void rfft_plan_##SUF(plan_##SUF* p, const T* in, T* out) {                        \
        const size_t half = p->half;                                                         \
        cx_##SUF* buf = p->buf;                                                              \
        cfft_tab_##SUF((const cx_##SUF*)in, half, buf, p->tw, p->w8); /* realfft.rs:130-138 */ \
        buf[half] = buf[0];                                 /* realfft.rs:140 */             \
        cx_##SUF* o = (cx_##SUF*)out;                                                        \
        for (size_t k = 0; k < half; ++k) { /* realfft.rs:142-156 (zip4 over rev) */         \
            T s = p->sn[k], c = p->cs[k];                                                    \
            cx_##SUF b = buf[k], r = buf[half - k];                                          \
            T xr = (T)0.5 * (((b.re + r.re) + c * (b.im + r.im)) - s * (b.re - r.re));       \
            T xi = (T)0.5 * (((b.im - r.im) - s * (b.im + r.im)) - c * (b.re - r.re));       \
            o[k].re = xr; o[k].im = xi;                                                      \
        }                                                                                    \
        o[half].re = buf[0].re - buf[0].im; o[half].im = (T)0; /* realfft.rs:157 */          \
    }                                                                                        \
    /* rustfft 4.0 Radix4 with inverse = true: twiddles compute_twiddle(..).conj(),          \
     * rotate_90 by +i, butterfly_4's inverse output pair (same passes as cfft_tab) */      \
    static inline cx_##SUF rot90i_##SUF(cx_##SUF v) { cx_##SUF r = {-v.im, v.re}; return r; } \
    static inline cx_##SUF conj_##SUF(cx_##SUF v) { cx_##SUF r = {v.re, -v.im}; return r; } \
    static void bfly4i_##SUF(cx_##SUF* buf) {                                                \
        cx_##SUF v0 = buf[0], v1 = buf[1], v2 = buf[2], v3 = buf[3];                         \
        bfly2_##SUF(&v0, &v2); bfly2_##SUF(&v1, &v3);                                        \
        v3 = rot90i_##SUF(v3);                                                               \
        bfly2_##SUF(&v0, &v1); bfly2_##SUF(&v2, &v3);                                        \
        buf[0] = v0; buf[1] = v2; buf[2] = v1; buf[3] = v3; }                                \
    static void bfly8i_##SUF(cx_##SUF* buf, cx_##SUF w1, cx_##SUF w3) {                      \
        cx_##SUF s[8] = {buf[0], buf[2], buf[4], buf[6], buf[1], buf[3], buf[5], buf[7]};    \
        bfly4i_##SUF(s); bfly4i_##SUF(s + 4);                                                \
        s[5] = cmul_##SUF(s[5], w1); s[6] = rot90i_##SUF(s[6]); s[7] = cmul_##SUF(s[7], w3); \
        for (int i = 0; i < 4; ++i) bfly2_##SUF(&s[i], &s[i + 4]);                           \
        for (int i = 0; i < 8; ++i) buf[i] = s[i]; }                                         \
    static void cifft_tab_##SUF(const cx_##SUF* in, size_t len, cx_##SUF* out,               \
                                const cx_##SUF* tw, const cx_##SUF* w8) {                    \
        if (len == 1) { out[0] = in[0]; return; }                                            \
        if (len == 2) { out[0] = in[0]; out[1] = in[1]; bfly2_##SUF(&out[0], &out[1]); return; } \
        if (len == 4) { memcpy(out, in, 4 * sizeof(cx_##SUF)); bfly4i_##SUF(out); return; }  \
        prepare_radix4_##SUF(len, in, out, 1);                                               \
        unsigned bits = 0; while (((size_t)1 << bits) < len) ++bits;                         \
        size_t cur;                                                                          \
        if (bits % 2 == 0) { for (size_t c = 0; c < len; c += 4) bfly4i_##SUF(out + c); cur = 16; } \
        else {                                                                               \
            const cx_##SUF w1 = conj_##SUF(w8[0]), w3 = conj_##SUF(w8[1]);                   \
            for (size_t c = 0; c < len; c += 8) bfly8i_##SUF(out + c, w1, w3);               \
            cur = 32;                                                                        \
        }                                                                                    \
        for (; cur <= len; cur *= 4) {                                                       \
            size_t q = cur / 4, tstride = len / cur;                                         \
            for (size_t row = 0; row < len / cur; ++row) {                                   \
                cx_##SUF* d = out + row * cur;                                               \
                for (size_t j = 0; j < q; ++j) { /* rustfft butterfly_4, inverse */          \
                    cx_##SUF s0 = cmul_##SUF(d[j + q], conj_##SUF(tw[j * 1 * tstride]));     \
                    cx_##SUF s1 = cmul_##SUF(d[j + 2 * q], conj_##SUF(tw[j * 2 * tstride])); \
                    cx_##SUF s2 = cmul_##SUF(d[j + 3 * q], conj_##SUF(tw[j * 3 * tstride])); \
                    cx_##SUF s5 = csub_##SUF(d[j], s1);                                      \
                    d[j] = cadd_##SUF(d[j], s1);                                             \
                    cx_##SUF s3 = cadd_##SUF(s0, s2);                                        \
                    cx_##SUF s4 = csub_##SUF(s0, s2);                                        \
                    d[j + 2 * q] = csub_##SUF(d[j], s3);                                     \
                    d[j] = cadd_##SUF(d[j], s3);                                             \
                    d[j + q].re = s5.re - s4.im; d[j + q].im = s5.im + s4.re;                \
                    d[j + 3 * q].re = s5.re + s4.im; d[j + 3 * q].im = s5.im - s4.re;        \
                }                                                                            \
            }                                                                                \
        }                                                                                    \
    }                                                                                        \
    /* realfft.rs:167-241 InvRealFFT::new + process: in [n/2+1] complex, out [n] real */    \
    int or_irfft_##SUF(const T* in, size_t n, T* out) {                                      \
        plan_##SUF* p = plan_new_##SUF(n);                                                   \
        if (!p) return -1;                                                                   \
        const size_t half = p->half;                                                         \
        const cx_##SUF* X = (const cx_##SUF*)in;                                             \
        for (size_t k = 0; k < half; ++k) { /* realfft.rs:210-219 (zip4 over rev) */         \
            T s = p->sn[k], c = p->cs[k];                                                    \
            cx_##SUF b = X[k], r = X[half - k];                                              \
            p->buf[k].re = (T)0.5 * (((b.re + r.re) - c * (b.im + r.im)) - s * (b.re - r.re)); \
            p->buf[k].im = (T)0.5 * (((b.im - r.im) + c * (b.re - r.re)) - s * (b.im + r.im)); \
        }                                                                                    \
        cifft_tab_##SUF(p->buf, half, (cx_##SUF*)out, p->tw, p->w8); /* realfft.rs:225-230 */ \
        plan_free_##SUF(p);                                                                  \
        return 0;                                                                            \
    }                                                                                        \
    /* one RealFFT::new per call (the reference's per-frame re-plan, lib.rs:455) */          \
    int or_rfft_##SUF(const T* in, size_t n, T* out) {                                       \
        plan_##SUF* p = plan_new_##SUF(n);                                                   \
        if (!p) return -1;                                                                   \
        rfft_plan_##SUF(p, in, out);                                                         \
        plan_free_##SUF(p);                                                                  \
        return 0;                                                                            \
    }

static inline float f32_sin(float x) { return sinf(x); }
static inline float f32_cos(float x) { return cosf(x); }
static inline double f64_sin(double x) { return sin(x); }
static inline double f64_cos(double x) { return cos(x); }

DEFINE_FFT(float, f32)
DEFINE_FFT(double, f64)

void or_rfft_sin_cos_f32(size_t n, float* out) {
    const float pi = (float)M_PI;
    const float halflen = (float)(n / 2);
    for (size_t k = 0; k < n / 2; ++k) {
        float ang = (float)k * pi / halflen;
        out[2 * k] = sinf(ang);
        out[2 * k + 1] = cosf(ang);
    }
}

/* ------------------------------------------------------------------------------------ */
/* lib.rs:367-471 to_windowed_frames / perform_stft                                     */
/* ------------------------------------------------------------------------------------ */
static size_t n_windows(size_t len, size_t win, size_t hop) {
    /* input.windows(win).into_iter().step_by(hop).count() */
    if (len < win) return 0;
    return (len - win) / hop + 1;
}

/* Emits the frames of one segment (to_windowed_frames, lib.rs:367-386) into out. */
static size_t emit_frames(const float* seg, size_t len, const float* window, size_t win,
                          size_t hop, size_t pad_l, size_t pad_r, float* out) {
    size_t nf = n_windows(len, win, hop);
    size_t n_fft = pad_l + win + pad_r;
    for (size_t f = 0; f < nf; ++f) {
        float* o = out + f * n_fft;
        for (size_t i = 0; i < pad_l; ++i) o[i] = 0.0f;
        for (size_t k = 0; k < win; ++k) o[pad_l + k] = seg[f * hop + k] * window[k]; /* &x * &window */
        for (size_t i = 0; i < pad_r; ++i) o[pad_l + win + i] = 0.0f;
    }
    return nf;
}

static void default_window(size_t win, size_t n_fft, float* w) {
    /* lib.rs:407 windows::hann(win_length, false) / A::from(n_fft) */
    or_hann_f32(win, 0, w);
    for (size_t i = 0; i < win; ++i) w[i] = w[i] / (float)n_fft;
}

/* Literal front / middle / back construction, lib.rs:400-435. out may be NULL (count). */
size_t or_frames_literal_f32(const float* x, size_t n, size_t win, size_t hop, size_t n_fft,
                             const float* window, float* out) {
    if (win == 0 || hop == 0 || n_fft < win || win < 1) return 0;
    if (n + 1 < win) return 0;                       /* input.slice(s![..win-1]) panics */
    size_t pad_l = (n_fft - win) / 2;                                   /* lib.rs:400 */
    size_t pad_r = (size_t)ceilf((float)(n_fft - win) / 2.0f);          /* lib.rs:401 */
    float* wbuf = NULL;
    if (!window) { wbuf = (float*)malloc(win * sizeof(float)); default_window(win, n_fft, wbuf); window = wbuf; }
    size_t half = win / 2;
    float* zeros = NULL;
    if (!x) { zeros = (float*)calloc(n + 1, sizeof(float)); x = zeros; out = NULL; }
    /* front_wav = pad(input[..win-1], (win/2, 0), Reflect)  lib.rs:412-417 */
    size_t flen = (win - 1) + half;
    float* front = (float*)malloc((flen + 1) * sizeof(float));
    if (or_pad_reflect_f32(x, win - 1, half, 0, front) != 0) { free(front); free(wbuf); free(zeros); return 0; }
    size_t nfront = n_windows(flen, win, hop);
    if (nfront * hop < half) { free(front); free(wbuf); free(zeros); return 0; }     /* usize underflow */
    size_t first_idx = nfront * hop - half;                             /* lib.rs:420 */
    if (first_idx > n) { free(front); free(wbuf); free(zeros); return 0; }
    size_t nmid = n_windows(n - first_idx, win, hop);                   /* lib.rs:421 */
    size_t mid_start = first_idx;
    first_idx += nmid * hop;                                            /* lib.rs:423 */
    if (n < half + 1) { free(front); free(wbuf); free(zeros); return 0; }
    size_t back_start = first_idx < n - half - 1 ? first_idx : n - half - 1; /* lib.rs:424 */
    size_t blen0 = n - back_start;
    float* back = (float*)malloc((blen0 + half + 1) * sizeof(float));
    if (or_pad_reflect_f32(x + back_start, blen0, 0, half, back) != 0) {
        free(front); free(back); free(wbuf); free(zeros); return 0;
    }
    size_t skip = first_idx - back_start;                               /* lib.rs:432 */
    size_t blen = blen0 + half;
    if (skip > blen) { free(front); free(back); free(wbuf); free(zeros); return 0; }
    size_t nback = n_windows(blen - skip, win, hop);
    size_t total = nfront + nmid + nback;
    if (out) {
        float* o = out;
        o += emit_frames(front, flen, window, win, hop, pad_l, pad_r, o) * n_fft;
        o += emit_frames(x + mid_start, n - mid_start, window, win, hop, pad_l, pad_r, o) * n_fft;
        emit_frames(back + skip, blen - skip, window, win, hop, pad_l, pad_r, o);
    }
    free(front); free(back); free(wbuf); free(zeros);
    return total;
}

size_t or_stft_n_frames(size_t n, size_t win, size_t hop) {
    return or_frames_literal_f32(NULL, n, win, hop, win, NULL, NULL);
}

/* The uniform rule: frame t, k<win: x_ref[t*hop - win/2 + k] * w[k] at pad_l + k, where
 * x_ref reflects about sample 0 and sample n-1. Count = (n + 2*(win/2) - win)/hop + 1. */
size_t or_frames_uniform_f32(const float* x, size_t n, size_t win, size_t hop, size_t n_fft,
                             const float* window, float* out) {
    if (win == 0 || hop == 0 || n_fft < win || n + 1 < win || n < 2) return 0;
    size_t half = win / 2;
    size_t T = (n + 2 * half - win) / hop + 1;
    size_t pad_l = (n_fft - win) / 2;
    float* wbuf = NULL;
    if (!window) { wbuf = (float*)malloc(win * sizeof(float)); default_window(win, n_fft, wbuf); window = wbuf; }
    if (out) {
        for (size_t t = 0; t < T; ++t) {
            float* o = out + t * n_fft;
            for (size_t m = 0; m < n_fft; ++m) o[m] = 0.0f;
            for (size_t k = 0; k < win; ++k) {
                long long i = (long long)(t * hop) - (long long)half + (long long)k;
                if (i < 0) i = -i;
                if (i > (long long)n - 1) i = 2 * ((long long)n - 1) - i;
                if (i < 0) i = 0;
                o[pad_l + k] = x[i] * window[k];
            }
        }
    }
    free(wbuf);
    return T;
}

size_t or_perform_stft_f32(const float* x, size_t n, size_t win, size_t hop, size_t n_fft,
                           const float* window, float* out) {
    size_t T = or_frames_literal_f32(x, n, win, hop, n_fft, window, NULL);
    if (T == 0) return 0;
    plan_f32* p = plan_new_f32(n_fft);                 /* RealFFT::new returns Err -> unwrap */
    if (!p) return 0;
    float* frames = (float*)malloc(T * n_fft * sizeof(float));
    or_frames_literal_f32(x, n, win, hop, n_fft, window, frames);
    size_t F = n_fft / 2 + 1;
    /* lib.rs:459-467: one plan for every frame (bit-identical to a plan per frame, :449-458) */
    for (size_t t = 0; t < T; ++t) rfft_plan_f32(p, frames + t * n_fft, out + t * F * 2);
    free(frames);
    plan_free_f32(p);
    return T;
}

/* ------------------------------------------------------------------------------------ */
/* lib.rs:124 norm (num-complex: re.hypot(im) -> glibc hypotf), norm_sqr; decibel.rs    */
/* ------------------------------------------------------------------------------------ */
void or_norm_f32(const float* c, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = hypotf(c[2 * i], c[2 * i + 1]);
}
void or_norm_sqr_f32(const float* c, size_t n, float* out) {
    for (size_t i = 0; i < n; ++i) out[i] = c[2 * i] * c[2 * i] + c[2 * i + 1] * c[2 * i + 1];
}

int or_log_for_db_f32(float* x, size_t n, float ref, float amin) {
    for (size_t i = 0; i < n; ++i)                     /* decibel.rs:34 assert all x >= 0 */
        if (!(x[i] >= 0.0f)) return -1;
    float ref_value = fabsf(ref);                      /* decibel.rs:37-40 */
    float log_amin = log10f(amin);                     /* decibel.rs:43 */
    float log_ref = ref_value > amin ? log10f(ref_value) : log_amin;
    for (size_t i = 0; i < n; ++i)                     /* decibel.rs:49-55 */
        x[i] = x[i] > amin ? log10f(x[i]) - log_ref : log_amin - log_ref;
    return 0;
}
int or_amp_to_db_default_f32(float* x, size_t n) {
    if (or_log_for_db_f32(x, n, 1.0f, 1e-18f)) return -1;   /* decibel.rs:7,79-88 */
    for (size_t i = 0; i < n; ++i) x[i] = 20.0f * x[i];     /* decibel.rs:75 */
    return 0;
}
int or_power_to_db_default_f32(float* x, size_t n) {
    if (or_log_for_db_f32(x, n, 1.0f, 1e-36f)) return -1;   /* decibel.rs:8,91-100 */
    for (size_t i = 0; i < n; ++i) x[i] = 10.0f * x[i];     /* decibel.rs:65 */
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* mel.rs                                                                               */
/* ------------------------------------------------------------------------------------ */
#define MIN_LOG_MEL 15.0
#define MIN_LOG_HZ 1000.0
#define LOGSTEP 0.06875177742094912
#define LINEARSCALE (200.0 / 3.0)

float or_mel_to_hz_f32(float mel) {                    /* mel.rs:13-21 */
    const float min_log_mel = (float)MIN_LOG_MEL;
    if (mel < min_log_mel) return (float)LINEARSCALE * mel;
    return (float)MIN_LOG_HZ * expf((float)LOGSTEP * (mel - min_log_mel));
}
float or_hz_to_mel_f32(float f) {                      /* mel.rs:23-31 */
    const float min_log_hz = (float)MIN_LOG_HZ;
    if (f < min_log_hz) return f / (float)LINEARSCALE;
    return (float)MIN_LOG_MEL + logf(f / min_log_hz) / (float)LOGSTEP;
}
double or_mel_to_hz_f64(double mel) {
    if (mel < MIN_LOG_MEL) return LINEARSCALE * mel;
    return MIN_LOG_HZ * exp(LOGSTEP * (mel - MIN_LOG_MEL));
}
double or_hz_to_mel_f64(double f) {
    if (f < MIN_LOG_HZ) return f / LINEARSCALE;
    return MIN_LOG_MEL + log(f / MIN_LOG_HZ) / LOGSTEP;
}

/* ndarray::numeric_util::unrolled_fold for a contiguous column (only reached when n_mel==1) */
#define DEFINE_UNROLLED_SUM(T, SUF)                                                          \
    static T unrolled_sum_##SUF(const T* xs, size_t n, size_t stride) {                      \
        T acc = 0, p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0, p6 = 0, p7 = 0;          \
        size_t i = 0;                                                                        \
        for (; n - i >= 8; i += 8) {                                                         \
            p0 = p0 + xs[(i + 0) * stride]; p1 = p1 + xs[(i + 1) * stride];                  \
            p2 = p2 + xs[(i + 2) * stride]; p3 = p3 + xs[(i + 3) * stride];                  \
            p4 = p4 + xs[(i + 4) * stride]; p5 = p5 + xs[(i + 5) * stride];                  \
            p6 = p6 + xs[(i + 6) * stride]; p7 = p7 + xs[(i + 7) * stride];                  \
        }                                                                                    \
        acc = acc + (p0 + p4); acc = acc + (p1 + p5);                                        \
        acc = acc + (p2 + p6); acc = acc + (p3 + p7);                                        \
        for (; i < n; ++i) acc = acc + xs[i * stride];                                       \
        return acc;                                                                          \
    }
DEFINE_UNROLLED_SUM(float, f32)
DEFINE_UNROLLED_SUM(double, f64)

#define DEFINE_MEL_FB(T, SUF, EPS)                                                           \
    void or_calc_mel_fb_##SUF(uint32_t sr, size_t n_fft, size_t n_mel, T fmin, T fmax_in,    \
                              int do_norm, T* w) {                                           \
        const T f_nyq = (T)((float)sr / 2.0f);               /* mel.rs:54 */                 \
        const T fmax = fmax_in < 0 ? f_nyq : fmax_in;         /* mel.rs:55 */                \
        const size_t n_freq = n_fft / 2 + 1;                  /* mel.rs:56 */                \
        const T min_mel = or_hz_to_mel_##SUF(fmin), max_mel = or_hz_to_mel_##SUF(fmax);      \
        /* ndarray 0.14 linspace: start + step * i, step = (end-start)/(n-1) */              \
        T lstep = n_freq > 1 ? (f_nyq - (T)0) / (T)(n_freq - 1) : (T)0;                      \
        T* lin = (T*)malloc(n_freq * sizeof(T));                                             \
        for (size_t i = 0; i < n_freq; ++i) lin[i] = (T)0 + lstep * (T)i;                    \
        size_t nm2 = n_mel + 2;                                                              \
        T mstep = (max_mel - min_mel) / (T)(nm2 - 1);                                        \
        T* melf = (T*)malloc(nm2 * sizeof(T));                                               \
        for (size_t i = 0; i < nm2; ++i) melf[i] = or_mel_to_hz_##SUF(min_mel + mstep * (T)i); \
        memset(w, 0, n_freq * n_mel * sizeof(T));                                            \
        for (size_t m = 0; m < n_mel; ++m) {                  /* mel.rs:66-83 */             \
            T m0 = melf[m], m1 = melf[m + 1], m2 = melf[m + 2];                              \
            for (size_t i = 0; i < n_freq; ++i) {                                            \
                T f = lin[i];                                                                \
                if (f <= m0) continue;                                                       \
                else if (m0 < f && f < m1) w[i * n_mel + m] = (f - m0) / (m1 - m0);          \
                else if (f == m1) w[i * n_mel + m] = (T)1;                                   \
                else if (m1 < f && f < m2) w[i * n_mel + m] = (m2 - f) / (m2 - m1);          \
                else break;                                                                  \
            }                                                                                \
            if (do_norm) {                                                                   \
                T s;                                                                         \
                if (n_mel == 1) s = unrolled_sum_##SUF(w + m, n_freq, n_mel);                \
                else { s = (T)0; for (size_t i = 0; i < n_freq; ++i) s = s + w[i * n_mel + m]; } \
                T d = s > (T)EPS ? s : (T)EPS;                /* Float::max(sum, epsilon) */ \
                if (s != s) d = (T)EPS;                                                      \
                for (size_t i = 0; i < n_freq; ++i) w[i * n_mel + m] = w[i * n_mel + m] / d; \
            }                                                                                \
        }                                                                                    \
        free(lin); free(melf);                                                               \
    }
DEFINE_MEL_FB(float, f32, FLT_EPSILON)
DEFINE_MEL_FB(double, f64, DBL_EPSILON)

size_t or_calc_mel_fb_default_f32(uint32_t sr, size_t n_fft, float* out) {
    /* mel.rs:88-90 */
    float v = 2.0f * or_hz_to_mel_f32((float)sr / 2.0f) / or_hz_to_mel_f32((float)sr / (float)n_fft) - 1.0f;
    size_t n_mel = (v != v || v <= 0.0f) ? 0 : (size_t)v;
    size_t F = n_fft / 2 + 1;
    if (n_mel > F) n_mel = F;
    float* fb = (float*)malloc(F * (n_mel ? n_mel : 1) * sizeof(float));
    for (; n_mel > 0; --n_mel) {                       /* mel.rs:92-98 */
        or_calc_mel_fb_f32(sr, n_fft, n_mel, 0.0f, -1.0f, 1, fb);
        int ok = 1;
        for (size_t m = 0; m < n_mel && ok; ++m) {
            float s = 0.0f;
            for (size_t i = 0; i < F; ++i) s = s + fb[i * n_mel + m];
            if (!(s > 0.0f)) ok = 0;
        }
        if (ok) break;
    }
    if (out && n_mel) memcpy(out, fb, F * n_mel * sizeof(float));
    free(fb);
    return n_mel;
}

/* ------------------------------------------------------------------------------------ */
/* lib.rs:131 linspec.dot(mel_fb) -- fmaf chain over k ascending (order unpinned)       */
/* ------------------------------------------------------------------------------------ */
#if defined(__x86_64__) && defined(__GNUC__)
__attribute__((target("avx2,fma")))
static void dot_fma_avx2(const float* a, const float* b, size_t T, size_t K, size_t M, float* out) {
    for (size_t t = 0; t < T; ++t) {
        float* o = out + t * M;
        for (size_t m = 0; m < M; ++m) o[m] = 0.0f;
        for (size_t k = 0; k < K; ++k) {
            float av = a[t * K + k];
            const float* br = b + k * M;
            for (size_t m = 0; m < M; ++m) o[m] = __builtin_fmaf(av, br[m], o[m]);
        }
    }
}
#endif
void or_dot_f32(const float* a, const float* b, size_t T, size_t K, size_t M, float* out) {
#if defined(__x86_64__) && defined(__GNUC__)
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) {
        dot_fma_avx2(a, b, T, K, M, out);
        return;
    }
#endif
    for (size_t t = 0; t < T; ++t) {
        float* o = out + t * M;
        for (size_t m = 0; m < M; ++m) o[m] = 0.0f;
        for (size_t k = 0; k < K; ++k) {
            float av = a[t * K + k];
            for (size_t m = 0; m < M; ++m) o[m] = fmaf(av, b[k * M + m], o[m]);
        }
    }
}

/* ------------------------------------------------------------------------------------ */
/* display.rs                                                                           */
/* ------------------------------------------------------------------------------------ */
const uint8_t OR_COLORMAP[10][3] = {                   /* display.rs:10-21 (inferno, 10 stops) */
    {0, 0, 4},     {27, 12, 65},  {74, 12, 107}, {120, 28, 109}, {165, 44, 96},
    {207, 68, 70}, {237, 105, 37}, {251, 155, 6}, {247, 209, 61}, {252, 255, 164}};
const uint8_t OR_WAVECOLOR[4] = {200, 21, 103, 255};   /* display.rs:22 */

static uint8_t sat_u8(float v) {                       /* Rust `as u8`: saturating, NaN -> 0 */
    if (!(v == v)) return 0;
    if (v <= 0.0f) return 0;
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}

int or_grey_to_color(float x, uint8_t rgb[3]) {        /* display.rs:24-42 */
    int panicked = 0;
    if (!(x >= 0.0f)) { panicked = 1; x = 0.0f; }      /* assert!(x >= 0.) */
    float position = 10.0f * x;
    float fl = floorf(position);
    size_t index = fl >= 18446744073709551615.0f ? (size_t)-1 : (size_t)fl;
    if (index >= 9) {
        rgb[0] = OR_COLORMAP[9][0]; rgb[1] = OR_COLORMAP[9][1]; rgb[2] = OR_COLORMAP[9][2];
        return panicked;
    }
    float ratio = position - (float)index;
    for (int i = 0; i < 3; ++i) {
        float a = (float)OR_COLORMAP[index][i], b = (float)OR_COLORMAP[index + 1][i];
        rgb[i] = sat_u8(roundf(ratio * b + (1.0f - ratio) * a));
    }
    return panicked;
}

uint32_t or_spec_grey_height(size_t bins, float up_ratio) {
    float h = roundf((float)bins * up_ratio);          /* display.rs:45 */
    if (!(h > 0.0f)) return 0;
    if (h >= 4294967295.0f) return 4294967295u;
    return (uint32_t)h;
}

void or_spec_to_grey(const float* spec, size_t T, size_t bins, float up_ratio, float max,
                     float min, float* grey) {
    uint32_t H = or_spec_grey_height(bins, up_ratio);  /* display.rs:44-54 */
    for (uint32_t y = 0; y < H; ++y) {
        for (size_t x = 0; x < T; ++x) {
            float v = 0.0f;
            if (y >= H - (uint32_t)bins) {
                float db = spec[x * bins + (H - 1 - y)];
                v = (db - min) / (max - min);
                v = fmaxf(v, 0.0f);                    /* Rust f32::max/min ignore NaN */
                v = fminf(v, 1.0f);
            }
            grey[(size_t)y * T + x] = v;
        }
    }
}

/* image 0.23.12 imageops/sample.rs (restated): sinc / lanczos / lanczos3_kernel */
static float sinc_f(float t) {
    float a = t * (float)M_PI;
    return t == 0.0f ? 1.0f : sinf(a) / a;
}
static float lanczos3(float x) {
    return fabsf(x) < 3.0f ? sinc_f(x) * sinc_f(x / 3.0f) : 0.0f;
}

typedef struct { uint32_t left, n; float* w; } taps_t;

static taps_t* make_taps(uint32_t src, uint32_t dst) {
    taps_t* tp = (taps_t*)calloc(dst ? dst : 1, sizeof(taps_t));
    float ratio = (float)src / (float)dst;
    float sratio = ratio < 1.0f ? 1.0f : ratio;
    float support = 3.0f * sratio;
    for (uint32_t o = 0; o < dst; ++o) {
        float in = ((float)o + 0.5f) * ratio;
        long long left = (long long)floorf(in - support);
        if (left < 0) left = 0;
        if (left > (long long)src - 1) left = (long long)src - 1;
        long long right = (long long)ceilf(in + support);
        if (right < left + 1) right = left + 1;
        if (right > (long long)src) right = (long long)src;
        in = in - 0.5f;
        uint32_t n = (uint32_t)(right - left);
        tp[o].left = (uint32_t)left;
        tp[o].n = n;
        tp[o].w = (float*)malloc((n ? n : 1) * sizeof(float));
        float sum = 0.0f;
        for (uint32_t i = 0; i < n; ++i) {
            float w = lanczos3(((float)(left + i) - in) / sratio);
            tp[o].w[i] = w;
            sum += w;
        }
        for (uint32_t i = 0; i < n; ++i) tp[o].w[i] /= sum;
    }
    return tp;
}
static void free_taps(taps_t* tp, uint32_t dst) {
    for (uint32_t o = 0; o < dst; ++o) free(tp[o].w);
    free(tp);
}

void or_resize_lanczos3_f32(const float* in, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                            float* out) {
    /* resize: vertical_sample (into an f32 image) then horizontal_sample */
    float* tmp = (float*)malloc((size_t)w * nh * sizeof(float) + 4);
    taps_t* vt = make_taps(h, nh);
    for (uint32_t oy = 0; oy < nh; ++oy)
        for (uint32_t x = 0; x < w; ++x) {
            float t = 0.0f;
            for (uint32_t i = 0; i < vt[oy].n; ++i) t += in[(size_t)(vt[oy].left + i) * w + x] * vt[oy].w[i];
            tmp[(size_t)oy * w + x] = t;
        }
    free_taps(vt, nh);
    taps_t* ht = make_taps(w, nw);
    for (uint32_t ox = 0; ox < nw; ++ox)
        for (uint32_t y = 0; y < nh; ++y) {
            float t = 0.0f;
            for (uint32_t i = 0; i < ht[ox].n; ++i) t += tmp[(size_t)y * w + ht[ox].left + i] * ht[ox].w[i];
            /* clamp(t, S::min_value(), S::max_value()) for f32 subpixels: no-op on finite t */
            out[(size_t)y * nw + ox] = t;
        }
    free_taps(ht, nw);
    free(tmp);
}

size_t or_grey_to_rgb(const float* grey, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                      uint8_t* out) {
    float* r = (float*)malloc((size_t)nw * nh * sizeof(float) + 4);
    or_resize_lanczos3_f32(grey, w, h, nw, nh, r);     /* display.rs:57 */
    size_t panics = 0;
    for (size_t p = 0; p < (size_t)nw * nh; ++p)      /* display.rs:58-60 */
        panics += (size_t)or_grey_to_color(r[p], out + 3 * p);
    free(r);
    return panics;
}

int or_wav_to_image(const float* wav_in, size_t n, uint32_t nwidth, uint32_t nheight,
                    float amp_min, float amp_max, uint8_t* out) {
    /* display.rs:63-115. Returns 0 ok; -1 where the reference panics (the image written is
     * then the product policy: empty slices draw nothing, bottom clamps to nheight-1). */
    int panicked = 0;
    memset(out, 0, (size_t)nwidth * nheight * 4);
    float spp = (float)n / (float)nwidth;             /* display.rs:74 */
    const float* wav = wav_in;
    float* up = NULL;
    size_t wlen = n;
    if (spp < 1.0f) {                                  /* display.rs:76-91 */
        size_t factor = (size_t)ceilf(1.0f / spp);
        wlen = factor * n;
        up = (float*)malloc(wlen * sizeof(float));
        for (size_t i = 0; i < wlen; ++i) {
            float b = (i / factor + 1 < n) ? wav_in[i / factor + 1] : 0.0f;
            float r = (float)(i % factor) / (float)factor;
            up[i] = b * r + wav_in[i / factor] * (1.0f - (float)(i % factor) / (float)factor);
        }
        wav = up;
    }
    for (int32_t ipx = 0; ipx < (int32_t)nwidth; ++ipx) {
        float s = roundf(((float)ipx - 1.5f) * spp);
        s = fmaxf(s, 0.0f);
        size_t i_start = (size_t)s;
        float e = roundf(((float)ipx + 1.5f) * spp);
        size_t i_end = e <= 0.0f ? 0 : (size_t)e;
        if (i_end > wlen) i_end = wlen;
        if (i_start >= i_end) { panicked = 1; continue; } /* empty slice / start > end */
        float mx = wav[i_start], mn = wav[i_start];
        int nan = 0;
        for (size_t i = i_start; i < i_end; ++i) {
            float v = wav[i];
            if (v != v) nan = 1;
            if (v > mx) mx = v;
            if (v < mn) mn = v;
        }
        if (nan) { panicked = 1; continue; }
        float fh = (float)nheight, rng = amp_max - amp_min;
        long long top = (long long)roundf((amp_max - mx) * fh / rng);
        long long bottom = (long long)roundf((amp_max - mn) * fh / rng);
        if (bottom - top < 3) {
            float d = (float)(3 - bottom + top) / 2.0f;
            long long pad_bottom = (long long)ceilf(d), pad_top = (long long)floorf(d);
            top -= pad_top;
            bottom += pad_bottom;
        }
        if (top < 0) top = 0;
        if (bottom > (long long)nheight) bottom = (long long)nheight;
        if (bottom + 1 > (long long)nheight) { panicked = 1; bottom = (long long)nheight - 1; }
        if (top > bottom + 1) { panicked = 1; continue; }
        for (long long y = top; y <= bottom; ++y)
            for (int c = 0; c < 4; ++c) out[((size_t)y * nwidth + (size_t)ipx) * 4 + c] = OR_WAVECOLOR[c];
    }
    free(up);
    return panicked ? -1 : 0;
}

/* ------------------------------------------------------------------------------------ */
/* lib.rs:43-46 AudioTrack::new parameter derivation                                     */
/* ------------------------------------------------------------------------------------ */
void or_track_params(uint32_t sr, float win_ms, size_t t_overlap, size_t f_overlap,
                     size_t* win, size_t* hop, size_t* n_fft) {
    float wl = win_ms * (float)sr / 1000.0f;           /* lib.rs:43 */
    float h = roundf(wl / (float)t_overlap);           /* lib.rs:44 (.round() as usize) */
    *hop = h <= 0.0f ? 0 : (size_t)h;
    *win = *hop * t_overlap;                           /* lib.rs:45 */
    *n_fft = or_calc_proper_n_fft(*win) * f_overlap;   /* lib.rs:46 */
}

/* ------------------------------------------------------------------------------------ */
/* One track through the reference's spectrogram stage, the CPU baseline's unit of work:    */
/* channel-sum downmix of interleaved PCM (lib.rs:42), perform_stft with one plan           */
/* (lib.rs:459-467), |X| (lib.rs:124), then per `kind`: 0 |X|; 1 mel + amp dB (lib.rs:130-  */
/* 134); 2 amp dB (lib.rs:126-129); 3 power dB (decibel.rs:91-100). out: [T, F] or [T, M].  */
/* Returns T (0 where the reference panics).                                               */
/* ------------------------------------------------------------------------------------ */
size_t or_track_spec_f32(const float* pcm, size_t n, size_t channels, size_t win, size_t hop,
                         size_t n_fft, int kind, const float* mel_fb, size_t n_mel, float* out) {
    float* mono = (float*)malloc((n ? n : 1) * sizeof(float));
    for (size_t i = 0; i < n; ++i) {                   /* sum_axis(Axis(0)): 0 + c0 + c1 ... */
        float acc = 0.0f;
        for (size_t c = 0; c < channels; ++c) acc = acc + pcm[i * channels + c];
        mono[i] = acc;
    }
    size_t T = or_stft_n_frames(n, win, hop);
    size_t F = n_fft / 2 + 1;
    if (T == 0) { free(mono); return 0; }
    float* X = (float*)malloc(T * F * 2 * sizeof(float));
    if (or_perform_stft_f32(mono, n, win, hop, n_fft, NULL, X) != T) { free(mono); free(X); return 0; }
    free(mono);
    if (kind == 3) {
        or_norm_sqr_f32(X, T * F, out);
        or_power_to_db_default_f32(out, T * F);
        free(X);
        return T;
    }
    float* mag = kind == 1 ? (float*)malloc(T * F * sizeof(float)) : out;
    or_norm_f32(X, T * F, mag);
    free(X);
    if (kind == 1) {
        or_dot_f32(mag, mel_fb, T, F, n_mel, out);
        free(mag);
        or_amp_to_db_default_f32(out, T * n_mel);
    } else if (kind == 2) {
        or_amp_to_db_default_f32(out, T * F);
    }
    return T;
}

/* |X| of pre-built frames [T, n_fft] (rows t0..t1), each frame through RealFFT::process and
 * norm (lib.rs:124). replan != 0: a fresh RealFFT::new per frame, the reference's single-track
 * parallel path (lib.rs:449-458); else one plan for the rows (lib.rs:459-467). */
int or_rfft_mag_rows_f32(const float* frames, size_t n_fft, size_t t0, size_t t1, int replan,
                         float* out) {
    const size_t F = n_fft / 2 + 1;
    float* X = (float*)malloc(F * 2 * sizeof(float));
    plan_f32* p = replan ? NULL : plan_new_f32(n_fft);
    if (!replan && !p) { free(X); return -1; }
    for (size_t t = t0; t < t1; ++t) {
        if (replan) {
            if (or_rfft_f32(frames + t * n_fft, n_fft, X) != 0) { free(X); return -1; }
        } else {
            rfft_plan_f32(p, frames + t * n_fft, X);
        }
        or_norm_f32(X, F, out + t * F);
    }
    plan_free_f32(p);
    free(X);
    return 0;
}
