// Host check of multi-spectrogram-viewer_amd/csrc/exact_math.hpp against the system libm
// (glibc, the library Rust's f32::log10 / f32::hypot call on Linux). Built and run by
// tests/test_exact_math.py. Usage: exact_math_check STRIDE -> prints mismatch counts.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "exact_math.hpp"

int main(int argc, char** argv) {
    const unsigned stride = argc > 1 ? (unsigned)atoi(argv[1]) : 1;
    long n = 0, bad_log = 0, bad_log10 = 0, bad_hyp = 0, bad_norm = 0;
    for (unsigned long u = 1; u < 0x7f800000ul; u += stride) {
        float x;
        const unsigned v = (unsigned)u;
        memcpy(&x, &v, 4);
        if (thesia::exact::f32_bits(logf(x)) != thesia::exact::f32_bits(thesia::exact::logf_glibc(x))) ++bad_log;
        if (thesia::exact::f32_bits(log10f(x)) != thesia::exact::f32_bits(thesia::exact::log10f_glibc(x))) ++bad_log10;
        if (v >= 0x00800000u &&
            thesia::exact::f32_bits(log10f(x)) != thesia::exact::f32_bits(thesia::exact::log10f_normal(x)))
            ++bad_norm;  // the branch-free form, normal floats
        ++n;
    }
    unsigned s = 12345u;
    for (long i = 0; i < 20000000; ++i) {
        s ^= s << 13; s ^= s >> 17; s ^= s << 5;
        unsigned a = s;
        s ^= s << 13; s ^= s >> 17; s ^= s << 5;
        unsigned b = (s & 0x807fffffu) | ((((s >> 23) & 0xffu) % 200u + 20u) << 23);
        a = (a & 0x807fffffu) | ((((a >> 23) & 0xffu) % 200u + 20u) << 23);
        float x, y;
        memcpy(&x, &a, 4);
        memcpy(&y, &b, 4);
        if (thesia::exact::f32_bits(hypotf(x, y)) != thesia::exact::f32_bits(thesia::exact::hypotf_glibc(x, y))) ++bad_hyp;
    }
    // non-finite and zero arguments (e_hypotf.c / e_log10f.c special cases; NaN results compared
    // as NaN, not by payload)
    long bad_special = 0;
    const float sp[] = {0.0f, -0.0f, 1.5f, -3.25e-20f, 7.0e30f, __builtin_inff(), -__builtin_inff(), __builtin_nanf("")};
    auto same = [](float a, float b) {
        return (a != a && b != b) || thesia::exact::f32_bits(a) == thesia::exact::f32_bits(b);
    };
    for (float x : sp) {
        for (float y : sp)
            if (!same(hypotf(x, y), thesia::exact::hypotf_glibc(x, y))) ++bad_special;
        if (x > 0.0f || x != x) {
            if (!same(log10f(x), thesia::exact::log10f_glibc(x))) ++bad_special;
            if (x >= 1.17549435e-38f || x != x)
                if (!same(log10f(x), thesia::exact::log10f_normal(x))) ++bad_special;
        }
    }
    printf("%ld %ld %ld %ld %ld %ld\n", n, bad_log, bad_log10, bad_hyp, bad_norm, bad_special);
    return 0;
}
