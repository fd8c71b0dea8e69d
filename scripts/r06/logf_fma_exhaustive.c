/* Round 6: glibc logf (the host libm) against the optimized-routines algorithm with and without FMA
   contraction, on every positive normal float (gcc -O2 -ffp-contract=off logf_fma_exhaustive.c -lm):
   0 mismatches either way in 2 130 706 432 -- the device log10f core (exact_math.hpp) uses the
   contracted form. Test infrastructure, never linked into the library. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
typedef struct { double invc, logc; } E;
static const E T[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};
static float bf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t fb(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
/* logf for positive normal x, the optimized-routines algorithm with FMA contraction */
static float logf_fma(float x, int fma_on) {
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = fb(x);
    if (ix == 0x3f800000u) return 0.0f;
    uint32_t tmp = ix - 0x3f330000u;
    int i = (tmp >> 19) % 16;
    int k = (int32_t)tmp >> 23;
    uint32_t iz = ix - (tmp & (0x1ffu << 23));
    double invc = T[i].invc, logc = T[i].logc, z = (double)bf(iz);
    double r, y0, r2, y;
    if (fma_on) {
        r = fma(z, invc, -1.0);
        y0 = fma((double)k, Ln2, logc);
        r2 = r * r;
        y = fma(A1, r, A2);
        y = fma(A0, r2, y);
        y = fma(y, r2, y0 + r);
    } else {
        volatile double t;
        t = z * invc; r = t - 1.0;
        t = (double)k * Ln2; y0 = logc + t;
        r2 = r * r;
        t = A1 * r; y = t + A2;
        t = A0 * r2; y = t + y;
        t = y * r2; y = t + (y0 + r);
    }
    return (float)y;
}
int main(void) {
    uint64_t bad_fma = 0, bad_nofma = 0, n = 0;
    for (uint32_t u = 0x00800000u; u < 0x7f800000u; ++u) {  /* positive normal floats */
        float x = bf(u);
        float g = logf(x);
        float a = logf_fma(x, 1), b = logf_fma(x, 0);
        if (fb(a) != fb(g)) { if (bad_fma < 5) printf("fma differs at %a: %a vs glibc %a\n", x, a, g); ++bad_fma; }
        if (fb(b) != fb(g)) { if (bad_nofma < 5) printf("nofma differs at %a: %a vs glibc %a\n", x, b, g); ++bad_nofma; }
        ++n;
    }
    printf("n %llu fma mismatches %llu, non-fma mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad_fma, (unsigned long long)bad_nofma);
    return 0;
}
