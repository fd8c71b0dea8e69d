// host_tables.cpp -- see host_tables.hpp. Compiled with -ffp-contract=off.
#include "host_tables.hpp"

#include <cfloat>
#include <cmath>

namespace thesia {

namespace {
constexpr double kPi = 3.14159265358979323846;
constexpr double kMinLogMel = 15.0;                // mel.rs:8
constexpr double kMinLogHz = 1000.0;               // mel.rs:9
constexpr double kLogStep = 0.06875177742094912;   // mel.rs:10
constexpr double kLinearScale = 200.0 / 3.0;       // mel.rs:11
}  // namespace

const uint8_t kColormap[10][3] = {
    {0, 0, 4},     {27, 12, 65},  {74, 12, 107}, {120, 28, 109}, {165, 44, 96},
    {207, 68, 70}, {237, 105, 37}, {251, 155, 6}, {247, 209, 61}, {252, 255, 164}};

std::vector<float> hann(size_t size, bool symmetric) {
    // cosine_window(0.5, 0.5, 0, 0, size, symmetric), windows.rs:7-19
    std::vector<float> w(size);
    const float pi = (float)kPi;
    const size_t size2 = symmetric ? size : size + 1;
    const float a = 0.5f, b = 0.5f, c = 0.0f, d = 0.0f;
    for (size_t i = 0; i < size; ++i) {
        const float x = pi * (float)i / (float)(size2 - 1);
        const float b_ = b * cosf(2.0f * x);
        const float c_ = c * cosf(4.0f * x);
        const float d_ = d * cosf(6.0f * x);
        w[i] = (a - b_) + (c_ - d_);
    }
    return w;
}

size_t calc_proper_n_fft(size_t win_length) {
    const float e = ceilf(log2f((float)win_length));
    const unsigned ue = e > 0.0f ? (unsigned)e : 0u;
    return (size_t)1 << ue;
}

float mel_to_hz(float mel) {
    const float min_log_mel = (float)kMinLogMel;
    if (mel < min_log_mel) return (float)kLinearScale * mel;
    return (float)kMinLogHz * expf((float)kLogStep * (mel - min_log_mel));
}

float hz_to_mel(float f) {
    const float min_log_hz = (float)kMinLogHz;
    if (f < min_log_hz) return f / (float)kLinearScale;
    return (float)kMinLogMel + logf(f / min_log_hz) / (float)kLogStep;
}

std::vector<float> calc_mel_fb(uint32_t sr, size_t n_fft, size_t n_mel, float fmin, float fmax_in,
                               bool do_norm) {
    const size_t n_freq = n_fft / 2 + 1;
    std::vector<float> w(n_freq * n_mel, 0.0f);
    if (n_mel == 0) return w;
    const float f_nyq = (float)sr / 2.0f;
    const float fmax = fmax_in < 0.0f ? f_nyq : fmax_in;
    const float min_mel = hz_to_mel(fmin), max_mel = hz_to_mel(fmax);
    // ndarray 0.14 linspace: start + step * i
    const float lstep = n_freq > 1 ? (f_nyq - 0.0f) / (float)(n_freq - 1) : 0.0f;
    std::vector<float> lin(n_freq);
    for (size_t i = 0; i < n_freq; ++i) lin[i] = 0.0f + lstep * (float)i;
    const size_t nm2 = n_mel + 2;
    const float mstep = (max_mel - min_mel) / (float)(nm2 - 1);
    std::vector<float> melf(nm2);
    for (size_t i = 0; i < nm2; ++i) melf[i] = mel_to_hz(min_mel + mstep * (float)i);
    for (size_t m = 0; m < n_mel; ++m) {  // mel.rs:66-83
        const float m0 = melf[m], m1 = melf[m + 1], m2 = melf[m + 2];
        for (size_t i = 0; i < n_freq; ++i) {
            const float f = lin[i];
            if (f <= m0) continue;
            else if (m0 < f && f < m1) w[i * n_mel + m] = (f - m0) / (m1 - m0);
            else if (f == m1) w[i * n_mel + m] = 1.0f;
            else if (m1 < f && f < m2) w[i * n_mel + m] = (m2 - f) / (m2 - m1);
            else break;
        }
        if (do_norm) {
            float s = 0.0f;
            if (n_mel == 1) {  // contiguous column -> ndarray unrolled_fold
                float p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                size_t i = 0;
                for (; n_freq - i >= 8; i += 8)
                    for (int u = 0; u < 8; ++u) p[u] = p[u] + w[i + u];
                float acc = 0.0f;
                acc = acc + (p[0] + p[4]);
                acc = acc + (p[1] + p[5]);
                acc = acc + (p[2] + p[6]);
                acc = acc + (p[3] + p[7]);
                for (; i < n_freq; ++i) acc = acc + w[i];
                s = acc;
            } else {
                for (size_t i = 0; i < n_freq; ++i) s = s + w[i * n_mel + m];
            }
            float d = s > FLT_EPSILON ? s : FLT_EPSILON;  // Float::max(sum, epsilon)
            if (s != s) d = FLT_EPSILON;
            for (size_t i = 0; i < n_freq; ++i) w[i * n_mel + m] = w[i * n_mel + m] / d;
        }
    }
    return w;
}

std::vector<float> calc_mel_fb_default(uint32_t sr, size_t n_fft, size_t* n_mel_out) {
    const float v = 2.0f * hz_to_mel((float)sr / 2.0f) / hz_to_mel((float)sr / (float)n_fft) - 1.0f;
    size_t n_mel = (v != v || v <= 0.0f) ? 0 : (size_t)v;
    const size_t F = n_fft / 2 + 1;
    if (n_mel > F) n_mel = F;
    std::vector<float> fb;
    for (; n_mel > 0; --n_mel) {
        fb = calc_mel_fb(sr, n_fft, n_mel, 0.0f, -1.0f, true);
        bool ok = true;
        for (size_t m = 0; m < n_mel && ok; ++m) {
            float s = 0.0f;
            for (size_t i = 0; i < F; ++i) s = s + fb[i * n_mel + m];
            if (!(s > 0.0f)) ok = false;
        }
        if (ok) break;
    }
    *n_mel_out = n_mel;
    if (n_mel == 0) fb.clear();
    return fb;
}

void track_params(uint32_t sr, float win_ms, size_t t_overlap, size_t f_overlap, size_t* win,
                  size_t* hop, size_t* n_fft) {
    const float wl = win_ms * (float)sr / 1000.0f;
    const float h = roundf(wl / (float)t_overlap);
    *hop = h <= 0.0f ? 0 : (size_t)h;
    *win = *hop * t_overlap;
    *n_fft = calc_proper_n_fft(*win) * f_overlap;
}

std::vector<float> rfft_sin_cos(size_t n_fft) {
    const size_t half = n_fft / 2;
    std::vector<float> t(2 * (half ? half : 1), 0.0f);
    const float pi = (float)kPi;
    const float halflen = (float)half;
    for (size_t k = 0; k < half; ++k) {
        const float ang = (float)k * pi / halflen;  // realfft.rs:90-91
        t[2 * k] = sinf(ang);
        t[2 * k + 1] = cosf(ang);
    }
    return t;
}

std::vector<float> stage1_twiddles(size_t NC, int L, int P) {
    std::vector<float> t(2 * (size_t)L * P);
    for (int k1 = 0; k1 < P; ++k1)
        for (int n2 = 0; n2 < L; ++n2) {
            const size_t e = ((size_t)n2 * (size_t)k1) % NC;
            const double ang = -2.0 * kPi * (double)e / (double)NC;  // rustfft single_twiddle
            t[2 * ((size_t)k1 * L + n2)] = (float)cos(ang);
            t[2 * ((size_t)k1 * L + n2) + 1] = (float)sin(ang);
        }
    return t;
}

static uint64_t n_windows(uint64_t len, uint64_t win, uint64_t hop) {
    return len < win ? 0 : (len - win) / hop + 1;
}

uint64_t stft_n_frames(uint64_t n, uint64_t win, uint64_t hop) {
    // lib.rs:410-435, counting only (the frames themselves follow the uniform reflect rule,
    // proved equal to this construction in tests/test_oracle.py)
    if (win == 0 || hop == 0 || n + 1 < win) return 0;
    const uint64_t half = win / 2;
    if (half + 1 > win - 1) return 0;   // reflect pad on input[..win-1] panics
    const uint64_t flen = (win - 1) + half;
    const uint64_t nfront = n_windows(flen, win, hop);
    if (nfront * hop < half) return 0;
    uint64_t first = nfront * hop - half;
    if (first > n) return 0;
    const uint64_t nmid = n_windows(n - first, win, hop);
    first += nmid * hop;
    if (n < half + 1) return 0;
    const uint64_t back_start = first < n - half - 1 ? first : n - half - 1;
    const uint64_t blen0 = n - back_start;
    if (half + 1 > blen0) return 0;
    const uint64_t skip = first - back_start;
    const uint64_t blen = blen0 + half;
    if (skip > blen) return 0;
    const uint64_t nback = n_windows(blen - skip, win, hop);
    return nfront + nmid + nback;
}

// image 0.23.12 imageops::sample: sinc, lanczos(x, 3), vertical/horizontal_sample taps
static float sinc_f(float t) {
    const float a = t * (float)kPi;
    return t == 0.0f ? 1.0f : sinf(a) / a;
}
static float lanczos3(float x) { return fabsf(x) < 3.0f ? sinc_f(x) * sinc_f(x / 3.0f) : 0.0f; }

Taps lanczos3_taps(uint32_t src, uint32_t dst) {
    Taps tp;
    tp.left.resize(dst);
    tp.count.resize(dst);
    tp.offset.resize(dst);
    const float ratio = (float)src / (float)dst;
    const float sratio = ratio < 1.0f ? 1.0f : ratio;
    const float support = 3.0f * sratio;
    for (uint32_t o = 0; o < dst; ++o) {
        float in = ((float)o + 0.5f) * ratio;
        long long left = (long long)floorf(in - support);
        if (left < 0) left = 0;
        if (left > (long long)src - 1) left = (long long)src - 1;
        long long right = (long long)ceilf(in + support);
        if (right < left + 1) right = left + 1;
        if (right > (long long)src) right = (long long)src;
        in = in - 0.5f;
        const int32_t n = (int32_t)(right - left);
        tp.left[o] = (int32_t)left;
        tp.count[o] = n;
        tp.offset[o] = (int32_t)tp.weights.size();
        float sum = 0.0f;
        const size_t base = tp.weights.size();
        for (int32_t i = 0; i < n; ++i) {
            const float w = lanczos3(((float)(left + i) - in) / sratio);
            tp.weights.push_back(w);
            sum += w;
        }
        for (int32_t i = 0; i < n; ++i) tp.weights[base + i] /= sum;
        if (n > tp.max_taps) tp.max_taps = n;
    }
    if (tp.weights.empty()) tp.weights.push_back(0.0f);
    return tp;
}

}  // namespace thesia
