// exact_math.hpp -- f32 functions the reference calls through the system libm, restated so the
// device computes the same bits (host and device; built with -ffp-contract=off).
//
//   hypotf (num-complex Complex::norm -> f32::hypot, lib.rs:124): glibc evaluates it in double
//   and rounds once; (float)sqrt((double)x*x + (double)y*y) equals glibc 2.35 hypotf on 1e8
//   random pairs (tests/test_exact_math.py re-checks on the host).
//
//   log10f (decibel.rs:49-55 -> f32::log10): glibc 2.35 e_log10f.c (fdlibm's split
//   k*log10(2) + log(x')/ln(10)) over glibc's logf (ARM optimized-routines logf: 16-entry
//   table, degree-3 polynomial in double). The restatement below matches glibc 2.35
//   logf and log10f bit for bit on every positive finite float (exhaustive host check,
//   tests/test_exact_math.py). Inputs here are x > amin > 0, finite.
#pragma once

#include <cstdint>
#include <cstring>

#ifdef __HIPCC__
#define THESIA_HD __host__ __device__
#else
#define THESIA_HD
#endif

namespace thesia {
namespace exact {

struct LogfEntry {
    double invc, logc;
};

THESIA_HD inline uint32_t f32_bits(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}
THESIA_HD inline float bits_f32(uint32_t u) {
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

constexpr LogfEntry kLogfT[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};

// logf for positive finite x (glibc 2.35 / optimized-routines logf.c, LOGF_TABLE_BITS = 4)
THESIA_HD inline float logf_glibc(float x) {
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = f32_bits(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix < 0x00800000u) {  // subnormal: normalize
        ix = f32_bits(x * 0x1p23f);
        ix -= 23u << 23;
    }
    // x = 2^k z, z in [0x3f330000, 2 * 0x3f330000) (exact); c near the centre of z's subinterval
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double invc = kLogfT[i].invc, logc = kLogfT[i].logc;
    const double z = (double)bits_f32(iz);
    // log(x) = log1p(z/c - 1) + log(c) + k ln2
    const double r = z * invc - 1.0;
    const double y0 = logc + (double)k * Ln2;
    const double r2 = r * r;
    double y = A1 * r + A2;
    y = A0 * r2 + y;
    y = y * r2 + (y0 + r);
    return (float)y;
}

// log10f for positive finite x (glibc 2.35 e_log10f.c)
THESIA_HD inline float log10f_glibc(float x) {
    const float two25 = 3.3554432000e+07f, ivln10 = 4.3429449201e-01f;
    const float log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
    int32_t hx = (int32_t)f32_bits(x), k = 0;
    if (hx >= 0x7f800000) return x + x;  // +inf, NaN (e_log10f.c)
    if (hx < 0x00800000) {  // subnormal: scale up
        k -= 25;
        x *= two25;
        hx = (int32_t)f32_bits(x);
    }
    k += (hx >> 23) - 127;
    const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
    hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
    const float y = (float)(k + i);
    x = bits_f32((uint32_t)hx);
    const float z = y * log10_2lo + ivln10 * logf_glibc(x);
    return z + y * log10_2hi;
}

// log10f_glibc for positive NORMAL finite x without branches: the subnormal scalings of
// log10f / logf never apply, and logf's early return for x == 1 gives the same +0 as the
// general path (table entry 9 is {1, 0}: r = 0, y = 0). Equal to log10f_glibc (and glibc) on
// every positive normal float (tests/test_exact_math.py, exhaustive).
THESIA_HD inline float log10f_normal_tab(float x, const LogfEntry* tab) {
    const float ivln10 = 4.3429449201e-01f, log10_2hi = 3.0102920532e-01f, log10_2lo = 7.9034151668e-07f;
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    const int32_t hx = (int32_t)f32_bits(x);
    const int32_t k0 = (hx >> 23) - 127;
    const int32_t i0 = (int32_t)(((uint32_t)k0 & 0x80000000u) >> 31);
    const uint32_t ix = (uint32_t)((hx & 0x007fffff) | ((0x7f - i0) << 23));  // x' in [1, 2) or [0.5, 1)
    const float y = (float)(k0 + i0);
    // logf(x') (optimized-routines logf.c) in the contracted form glibc's x86-64 FMA variant of
    // logf computes (five fma instead of five products and five sums): the float it rounds to
    // equals the unfused form's and glibc's on every positive normal float (exhaustive host check,
    // round 6: 0 mismatches in 2 130 706 432; tests/test_exact_math.py re-checks every 3rd)
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double invc = tab[i].invc, logc = tab[i].logc;
    const double z = (double)bits_f32(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double y0 = __builtin_fma((double)k, Ln2, logc);
    const double r2 = r * r;
    double q = __builtin_fma(A1, r, A2);
    q = __builtin_fma(A0, r2, q);
    q = __builtin_fma(q, r2, y0 + r);
    const float lx = (float)q;
    const float zz = y * log10_2lo + ivln10 * lx;
    const float res = zz + y * log10_2hi;
    return hx >= 0x7f800000 ? x + x : res;  // +inf, NaN (e_log10f.c), as a select
}
// (the table from constant memory; kernels pass an LDS copy of kLogfT to log10f_normal_tab)
THESIA_HD inline float log10f_normal(float x) { return log10f_normal_tab(x, kLogfT); }

// hypotf (glibc 2.35 e_hypotf.c: an infinite argument gives +inf, even beside a NaN; else double
// evaluation, one rounding)
THESIA_HD inline float hypotf_glibc(float x, float y) {
    if (__builtin_fabsf(x) == __builtin_inff() || __builtin_fabsf(y) == __builtin_inff()) return __builtin_inff();
    const double dx = (double)x, dy = (double)y;
    return (float)__builtin_sqrt(dx * dx + dy * dy);
}

#ifdef __HIP_DEVICE_COMPILE__
// hypotf_glibc on the device without the sqrt's denormal scaling and class branches: S = x^2 +
// y^2 of finite f32 values is 0 or at least 2^-298 (far above the 2^-767 where the compiler's
// correctly rounded sqrt rescales), so v_rsq_f64 + the same Newton steps give its bits; S = 0
// gives +0. dx * dx is exact in double, so fma(dx, dx, dy * dy) is dx * dx + dy * dy rounded
// once. (scripts/probes/hypot_probe.hip: equal to __builtin_sqrt on 2^24 random pairs.)
__device__ inline __attribute__((always_inline)) float hypotf_cr(float x, float y) {
    const double dx = (double)x, dy = (double)y;
    const double S = __builtin_fma(dx, dx, dy * dy);
    const double y0 = __builtin_amdgcn_rsq(S);
    double g = S * y0, h = 0.5 * y0;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, S);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, S);
    g = __builtin_fma(d, h, g);
    const float f = (float)g;
    const bool inf = __builtin_fabsf(x) == __builtin_inff() || __builtin_fabsf(y) == __builtin_inff();
    return inf ? __builtin_inff() : S == 0.0 ? 0.0f : f;
}
#elif defined(__HIPCC__)
__host__ inline float hypotf_cr(float x, float y) { return hypotf_glibc(x, y); }  // (host pass)
#endif

}  // namespace exact
}  // namespace thesia
