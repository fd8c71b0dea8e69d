/*
 * thesia_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker for the MI355X engine, never the thing measured or shipped.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Reference: Sytronik/multi-spectrogram-viewer ("thesia"), src_rust/<module>.rs. Every function
 * cites the file:line it restates. All arithmetic is f32 unless the name says f64, in
 * the reference's evaluation order, built with -ffp-contract=off (Rust never fuses a*b+c).
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   pinned by the reference's own KATs: hann (windows.rs:35-38), pad (utils.rs:125-140),
 *   rfft impulse (utils.rs:117-123), STFT impulse (lib.rs:491-514), rfft-vs-complex-FFT at
 *   1e-15 in f64 (realfft.rs:253-272), hz<->mel (mel.rs:107-113), default n_mel property
 *   (mel.rs:135-165).
 *   parity unpinned (third-party arithmetic absent from /root/reference, restated from the
 *   crates' published algorithms): rustfft 4.0 Radix4 op order, num-complex norm (hypot),
 *   ndarray 0.14 dot (matrixmultiply sgemm order), image 0.23.12 Lanczos3 resize.
 */
#ifndef THESIA_ORACLE_H
#define THESIA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- windows.rs ---- */
void or_hann_f32(size_t size, int symmetric, float* out);             /* windows.rs:7-30 */
void or_hann_f64(size_t size, int symmetric, double* out);

/* ---- utils.rs ---- */
size_t or_calc_proper_n_fft(size_t win_length);                        /* utils.rs:17-19 */
/* 1-D pad; returns 0 on success, -1 where ndarray would panic (reflect pad >= len). */
int or_pad_reflect_f32(const float* x, size_t n, size_t left, size_t right, float* out); /* utils.rs:72-78 */
int or_pad_constant_f32(const float* x, size_t n, size_t left, size_t right, float c, float* out); /* utils.rs:63-71 */

/* ---- realfft.rs + rustfft 4.0 Radix4 (restated) ---- */
/* Complex FFT, forward, len power of two (rustfft Radix4::process). Interleaved re,im. */
int or_cfft_radix4_f32(const float* in, size_t len, float* out);
int or_cfft_radix4_f64(const double* in, size_t len, double* out);
/* RealFFT::process (realfft.rs:105-159). in: n reals (n even), out: (n/2+1) complex. */
int or_rfft_f32(const float* in, size_t n, float* out);
int or_rfft_f64(const double* in, size_t n, double* out);
int or_irfft_f32(const float* in, size_t n, float* out);   /* realfft.rs:167-241 InvRealFFT */
int or_irfft_f64(const double* in, size_t n, double* out);
/* RealFFT::new sin_cos table (realfft.rs:85-93): out[2k]=sin, out[2k+1]=cos, k<n/2. */
void or_rfft_sin_cos_f32(size_t n, float* out);

/* ---- lib.rs perform_stft ---- */
/* Number of frames the reference's front/middle/back construction yields (lib.rs:410-435);
 * returns 0 where the reference panics (input shorter than win-1, etc.). */
size_t or_stft_n_frames(size_t n, size_t win, size_t hop);
/* perform_stft (lib.rs:388-471) with the literal front/middle/back framing.
 * window may be NULL (default hann(win)/n_fft, lib.rs:407). out: T x (n_fft/2+1) complex.
 * Returns number of frames, or 0 on a reference panic condition. */
size_t or_perform_stft_f32(const float* x, size_t n, size_t win, size_t hop, size_t n_fft,
                           const float* window, float* out);
/* The same frames by the uniform reflect rule (the rule the GPU kernel implements);
 * used only to prove the rule equals the literal construction. out: T x n_fft reals. */
size_t or_frames_uniform_f32(const float* x, size_t n, size_t win, size_t hop, size_t n_fft,
                             const float* window, float* out);
size_t or_frames_literal_f32(const float* x, size_t n, size_t win, size_t hop, size_t n_fft,
                             const float* window, float* out);

/* ---- lib.rs:124, decibel.rs ---- */
void or_norm_f32(const float* cplx, size_t n, float* out);             /* num-complex norm = hypot */
void or_norm_sqr_f32(const float* cplx, size_t n, float* out);         /* num-complex norm_sqr */
/* log_for_db (decibel.rs:33-56) with reference Value(ref); returns -1 on the x>=0 assert. */
int or_log_for_db_f32(float* x, size_t n, float ref, float amin);
int or_amp_to_db_default_f32(float* x, size_t n);                      /* decibel.rs:79-88 */
int or_power_to_db_default_f32(float* x, size_t n);                    /* decibel.rs:91-100 */

/* ---- mel.rs ---- */
float or_hz_to_mel_f32(float f);                                        /* mel.rs:23-31 */
float or_mel_to_hz_f32(float m);                                        /* mel.rs:13-21 */
double or_hz_to_mel_f64(double f);
double or_mel_to_hz_f64(double m);
/* calc_mel_fb (mel.rs:33-85); out is [n_fft/2+1, n_mel] row-major. fmax<0 => None. */
void or_calc_mel_fb_f32(uint32_t sr, size_t n_fft, size_t n_mel, float fmin, float fmax,
                        int do_norm, float* out);
void or_calc_mel_fb_f64(uint32_t sr, size_t n_fft, size_t n_mel, double fmin, double fmax,
                        int do_norm, double* out);
/* calc_mel_fb_default (mel.rs:87-99): returns n_mel; out (may be NULL) needs F*F floats. */
size_t or_calc_mel_fb_default_f32(uint32_t sr, size_t n_fft, float* out);

/* ---- lib.rs:131 dense mel projection ---- */
/* out[t,m] = fma-chain over k ascending of a[t,k]*b[k,m] (ndarray dot order is unpinned). */
void or_dot_f32(const float* a, const float* b, size_t T, size_t K, size_t M, float* out);

/* ---- display.rs ---- */
extern const uint8_t OR_COLORMAP[10][3];                                /* display.rs:10-21 */
extern const uint8_t OR_WAVECOLOR[4];                                   /* display.rs:22 */
/* convert_grey_to_color (display.rs:24-42). Returns 1 where the reference's assert
 * (x >= 0) would panic; the colour then written is the product's policy (x treated as 0). */
int or_grey_to_color(float x, uint8_t rgb[3]);
/* spec_to_grey (display.rs:44-54): spec [T, bins]; grey [H, T]; returns H. */
uint32_t or_spec_grey_height(size_t bins, float up_ratio);
void or_spec_to_grey(const float* spec, size_t T, size_t bins, float up_ratio, float max,
                     float min, float* grey);
/* image 0.23.12 imageops::resize(.., Lanczos3) on a Luma<f32> image (restated). */
void or_resize_lanczos3_f32(const float* in, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                            float* out);
/* grey_to_rgb (display.rs:56-61); returns the number of pixels that would have panicked. */
size_t or_grey_to_rgb(const float* grey, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                      uint8_t* out);
/* wav_to_image (display.rs:63-115): RGBA [nheight, nwidth, 4]. Returns -1 on a panic path. */
int or_wav_to_image(const float* wav, size_t n, uint32_t nwidth, uint32_t nheight,
                    float amp_min, float amp_max, uint8_t* out);

/* ---- lib.rs:43-46 param derivation (AudioTrack::new) ---- */
void or_track_params(uint32_t sr, float win_ms, size_t t_overlap, size_t f_overlap,
                     size_t* win, size_t* hop, size_t* n_fft);

/* ---- one track through the spectrogram stage (CPU baseline unit of work) ----
 * interleaved PCM -> channel sum (lib.rs:42) -> perform_stft, one plan (lib.rs:459-467) -> |X|
 * (lib.rs:124) -> kind 0 |X|, 1 mel + amp dB (lib.rs:130-134), 2 amp dB, 3 power dB. */
size_t or_track_spec_f32(const float* pcm, size_t n, size_t channels, size_t win, size_t hop,
                         size_t n_fft, int kind, const float* mel_fb, size_t n_mel, float* out);

/* |X| of pre-built frames [T, n_fft], rows t0..t1 (replan: RealFFT::new per frame, lib.rs:455). */
int or_rfft_mag_rows_f32(const float* frames, size_t n_fft, size_t t0, size_t t1, int replan,
                         float* out);

#ifdef __cplusplus
}
#endif
#endif
