// host_tables.hpp -- host-side table builders of the engine (window, mel filterbank, FFT
// twiddles, realfft untangle table, Lanczos3 taps). f32 formulas in the reference's
// evaluation order with glibc libm (what Rust's f32 methods call on Linux) and
// -ffp-contract=off, so every table is bit-identical to the reference's.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace thesia {

// windows.rs:7-30
std::vector<float> hann(size_t size, bool symmetric);
// utils.rs:17-19
size_t calc_proper_n_fft(size_t win_length);
// mel.rs:13-31 (f32 instantiation)
float hz_to_mel(float f);
float mel_to_hz(float m);
// mel.rs:33-85 -> [n_fft/2+1, n_mel] row-major; fmax < 0 => Nyquist
std::vector<float> calc_mel_fb(uint32_t sr, size_t n_fft, size_t n_mel, float fmin, float fmax,
                               bool do_norm);
// mel.rs:87-99
std::vector<float> calc_mel_fb_default(uint32_t sr, size_t n_fft, size_t* n_mel);
// lib.rs:43-46
void track_params(uint32_t sr, float win_ms, size_t t_overlap, size_t f_overlap, size_t* win,
                  size_t* hop, size_t* n_fft);
// realfft.rs:85-93: (sin, cos) pairs, k < n/2
std::vector<float> rfft_sin_cos(size_t n_fft);
// W_NC^{n2*k1} for the stage-1 twiddles, [P][L] complex (f64-evaluated, rounded to f32)
std::vector<float> stage1_twiddles(size_t NC, int L, int P);
// Frame count of the reference's framing (lib.rs:410-435); 0 where it panics.
uint64_t stft_n_frames(uint64_t n, uint64_t win, uint64_t hop);

// image 0.23.12 resize taps for one axis (src -> dst) with Lanczos3 weights
struct Taps {
    std::vector<int32_t> left, count, offset;
    std::vector<float> weights;
    int max_taps = 0;
};
Taps lanczos3_taps(uint32_t src, uint32_t dst);

extern const uint8_t kColormap[10][3];  // display.rs:10-21

}  // namespace thesia
