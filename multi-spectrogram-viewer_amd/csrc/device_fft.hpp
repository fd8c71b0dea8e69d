// device_fft.hpp -- register-resident complex FFT building blocks for gfx950 (CDNA4).
//
// A length-NC complex FFT (NC = n_fft/2, the half-length transform realfft.rs:126-138 runs)
// is split NC = L x P: stage 1 is a P-point DFT held in one lane's registers (lane = n2),
// then an LDS transpose, then stage 2 is P/L L-point DFTs per lane. Twiddles inside a
// lane's DFT are compile-time constants (rounded once from a double evaluation, like
// rustfft's twiddles::single_twiddle); nothing here depends on runtime trig.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace thesia {

// ------------------------------------------------------------------------------------
// constexpr trig (double), used only to build compile-time twiddle constants.
// ------------------------------------------------------------------------------------
constexpr double kPiD = 3.14159265358979323846264338327950288;

constexpr double ce_sin_small(double x) {  // |x| <= pi/4
    double x2 = x * x, term = x, sum = x;
    for (int i = 1; i < 14; ++i) {
        term *= -x2 / double((2 * i) * (2 * i + 1));
        sum += term;
    }
    return sum;
}
constexpr double ce_cos_small(double x) {  // |x| <= pi/4
    double x2 = x * x, term = 1.0, sum = 1.0;
    for (int i = 1; i < 14; ++i) {
        term *= -x2 / double((2 * i - 1) * (2 * i));
        sum += term;
    }
    return sum;
}
// cos / sin of 2*pi*num/den with exact rational octant reduction.
constexpr void ce_cis(long long num, long long den, double& c, double& s) {
    num %= den;
    if (num < 0) num += den;
    // angle in [0, 2pi) = 2pi*num/den; octant o = floor(8*num/den)
    long long o = (8 * num) / den;
    // remainder angle r = 2pi*(num/den - o/8) in [0, pi/4)
    double r = 2.0 * kPiD * (double(8 * num - o * den) / double(8 * den));
    double sr = ce_sin_small(r), cr = ce_cos_small(r);
    // rotate by o * pi/4
    constexpr double h = 0.70710678118654752440084436210484903;
    double cc = cr, ss = sr;
    switch (o) {
        case 0: cc = cr; ss = sr; break;
        case 1: cc = h * (cr - sr); ss = h * (cr + sr); break;
        case 2: cc = -sr; ss = cr; break;
        case 3: cc = -h * (cr + sr); ss = h * (cr - sr); break;
        case 4: cc = -cr; ss = -sr; break;
        case 5: cc = -h * (cr - sr); ss = -h * (cr + sr); break;
        case 6: cc = sr; ss = -cr; break;
        default: cc = h * (cr + sr); ss = -h * (cr - sr); break;
    }
    c = cc;
    s = ss;
}
// Forward twiddle W_N^j = exp(-2*pi*i*j/N) as f32 components.
constexpr float ce_tw_re(int j, int N) {
    double c = 0, s = 0;
    ce_cis(j, N, c, s);
    return float(c);
}
constexpr float ce_tw_im(int j, int N) {
    double c = 0, s = 0;
    ce_cis(j, N, c, s);
    return float(-s);
}

// ------------------------------------------------------------------------------------
// complex helpers (float2 = re, im)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
    return make_float2(__builtin_fmaf(a.x, w.x, -(a.y * w.y)), __builtin_fmaf(a.x, w.y, a.y * w.x));
}
__device__ __forceinline__ float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }  // * (-i)
__device__ __forceinline__ float2 mul_posi(float2 a) { return make_float2(-a.y, a.x); }  // * (+i)

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// a * W_N^J with compile-time J, N (trivial rotations folded).
template <int N, int J>
__device__ __forceinline__ float2 twc(float2 a) {
    constexpr int r = ((J % N) + N) % N;
    if constexpr (r == 0) {
        return a;
    } else if constexpr (4 * r == N) {
        return mul_negi(a);
    } else if constexpr (2 * r == N) {
        return make_float2(-a.x, -a.y);
    } else if constexpr (4 * r == 3 * N) {
        return mul_posi(a);
    } else if constexpr (8 * r == N) {  // (1 - i)/sqrt2
        constexpr float h = ce_tw_re(1, 8);
        return make_float2((a.x + a.y) * h, (a.y - a.x) * h);
    } else if constexpr (8 * r == 3 * N) {  // (-1 - i)/sqrt2
        constexpr float h = ce_tw_re(1, 8);
        return make_float2((a.y - a.x) * h, -(a.x + a.y) * h);
    } else {
        constexpr float wr = ce_tw_re(r, N), wi = ce_tw_im(r, N);
        return cmul(a, make_float2(wr, wi));
    }
}

// ------------------------------------------------------------------------------------
// In-register DIF FFT over v[O + i*S], i < N (compile-time). Output in digit-reversed
// positions; ce_pos<N>(k) gives the position of X[k] relative to O (in units of S).
// ------------------------------------------------------------------------------------
constexpr int ce_pos(int N, int k) {
    if (N <= 1) return 0;
    if (N == 2) return k;
    if (N % 4 == 0) {
        const int Q = N / 4;
        return (k % 4) * Q + ce_pos(Q, k / 4);
    }
    const int H = N / 2;
    return (k % 2) * H + ce_pos(H, k / 2);
}

template <int I, int N>
__device__ __forceinline__ void pin_rec(float2 (&v)[N]) {
    if constexpr (I < N) {
        asm volatile("" : "+v"(v[I].x), "+v"(v[I].y));
        pin_rec<I + 1, N>(v);
    }
}
// Register "pin": an empty asm that reads and writes every value, so the scheduler cannot
// move arithmetic across it. Used between FFT stages to bound live ranges.
template <int N>
__device__ __forceinline__ void pin(float2 (&v)[N]) { pin_rec<0, N>(v); }
template <int N>
__device__ __forceinline__ void pin_f(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}
template <int B, int E, int N>
__device__ __forceinline__ void pin_range(float2 (&v)[N]) {
    if constexpr (B < E) {
        asm volatile("" : "+v"(v[B].x), "+v"(v[B].y));
        pin_range<B + 1, E, N>(v);
    }
}

template <int N, int S, int O, int TOT, int PIN_MIN = 1 << 30>
__device__ __forceinline__ void dif_fft(float2 (&v)[TOT]) {
    if constexpr (N <= 1) {
        return;
    } else if constexpr (N == 2) {
        float2 a = v[O], b = v[O + S];
        v[O] = cadd(a, b);
        v[O + S] = csub(a, b);
    } else if constexpr (N % 4 == 0) {
        constexpr int Q = N / 4;
        static_for<0, Q>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            float2 a0 = v[O + j * S], a1 = v[O + (j + Q) * S];
            float2 a2 = v[O + (j + 2 * Q) * S], a3 = v[O + (j + 3 * Q) * S];
            float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
            float2 t2 = cadd(a1, a3), t3 = mul_negi(csub(a1, a3));
            v[O + j * S] = cadd(t0, t2);
            v[O + (j + Q) * S] = twc<N, j>(cadd(t1, t3));
            v[O + (j + 2 * Q) * S] = twc<N, 2 * j>(csub(t0, t2));
            v[O + (j + 3 * Q) * S] = twc<N, 3 * j>(csub(t1, t3));
        });
        if constexpr (N * S >= PIN_MIN) pin(v);
        dif_fft<Q, S, O, TOT, PIN_MIN>(v);
        dif_fft<Q, S, O + Q * S, TOT, PIN_MIN>(v);
        dif_fft<Q, S, O + 2 * Q * S, TOT, PIN_MIN>(v);
        dif_fft<Q, S, O + 3 * Q * S, TOT, PIN_MIN>(v);
    } else {
        constexpr int H = N / 2;
        static_for<0, H>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            float2 a = v[O + j * S], b = v[O + (j + H) * S];
            v[O + j * S] = cadd(a, b);
            v[O + (j + H) * S] = twc<N, j>(csub(a, b));
        });
        if constexpr (N * S >= PIN_MIN) pin(v);
        dif_fft<H, S, O, TOT, PIN_MIN>(v);
        dif_fft<H, S, O + H * S, TOT, PIN_MIN>(v);
    }
}

// NC = L x P factorisation used by the STFT kernels (P % L == 0, P <= 64).
constexpr int geo_L(int NC) {
    return NC <= 1 ? 1 : NC == 2 ? 1 : NC == 4 ? 2 : NC == 8 ? 2 : NC == 16 ? 4 : NC == 32 ? 4
         : NC == 64 ? 8 : NC == 128 ? 8 : NC == 256 ? 16 : NC == 512 ? 16 : 32;
}
constexpr int geo_P(int NC) { return NC / geo_L(NC); }

}  // namespace thesia
