// stftr_core.hpp -- the reference-order arithmetic shared by the streaming reference-order
// kernels (stftr_kernels.hip: n_fft 2048; stftq_kernels.hip: n_fft 256 / 512 / 1024): rustfft 4.0
// butterflies with num-complex products (no fused multiply-add; built with -ffp-contract=off),
// the permlane swaps, a branch-free select and the reference's dB.
#pragma once

#include "exact_math.hpp"
#include "stft_common.hpp"

namespace thesia {

// num-complex Mul (no fused multiply-add): (a.re b.re - a.im b.im, a.re b.im + a.im b.re)
__device__ __forceinline__ float2 rmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// rustfft butterfly_4 (levels >= 1, forward; oracle cfft_tab), in place
__device__ __forceinline__ void rbfly(float2& d0, float2& d1, float2& d2, float2& d3, float2 w1,
                                      float2 w2, float2 w3) {
    const float2 s0 = rmul(d1, w1), s1 = rmul(d2, w2), s2 = rmul(d3, w3);
    const float2 s5 = csub(d0, s1);
    const float2 a = cadd(d0, s1);
    const float2 s3 = cadd(s0, s2), s4 = csub(s0, s2);
    d2 = csub(a, s3);
    d0 = cadd(a, s3);
    d1 = make_float2(s5.x + s4.y, s5.y - s4.x);
    d3 = make_float2(s5.x - s4.y, s5.y + s4.x);
}

// rustfft Butterfly4 (the base level, forward): bfly2(0, 2), bfly2(1, 3), rotate 3 by -i,
// bfly2(0, 1), bfly2(2, 3), outputs (0, 2, 1, 3)
__device__ __forceinline__ void rbfly4(float2& a0, float2& a1, float2& a2, float2& a3) {
    float2 v0 = a0, v1 = a1, v2 = a2, v3 = a3;
    float2 t = cadd(v0, v2);
    v2 = csub(v0, v2);
    v0 = t;
    t = cadd(v1, v3);
    v3 = csub(v1, v3);
    v1 = t;
    v3 = make_float2(v3.y, -v3.x);
    t = cadd(v0, v1);
    v1 = csub(v0, v1);
    v0 = t;
    t = cadd(v2, v3);
    v3 = csub(v2, v3);
    v2 = t;
    a0 = v0;
    a1 = v2;
    a2 = v1;
    a3 = v3;
}

// v_permlane16_swap / v_permlane32_swap as inline asm. The builtins are mis-optimised by this
// compiler (ROCm 7.2): a lane select between the two results, `lane < 32 ? r[1] : r[0]`, folds
// to r[0], and half of a run of swaps disappeared (scripts/probes/permlane_probe.hip pins the
// hardware semantics; the fold is visible in the .s). asm keeps every swap and both results.
// s_nop 1: the two wait states a VALU write of an operand needs before the swap reads it (the
// compiler's hazard recognizer does not look inside asm).
// pl16: the odd 16-lane rows of x <-> the even rows of y; pl32: lanes 32..63 of x <-> lanes 0..31 of y
__device__ __forceinline__ void pl16(float2& x, float2& y) {
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %2\n\tv_permlane16_swap_b32 %1, %3"
                 : "+v"(x.x), "+v"(x.y), "+v"(y.x), "+v"(y.y));
}
__device__ __forceinline__ void pl32(float2& x, float2& y) {
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3"
                 : "+v"(x.x), "+v"(x.y), "+v"(y.x), "+v"(y.y));
}

// branch-free lane select (v_bfi_b32): m all ones -> a, m zero -> b (a ternary on float2 values
// next to the asm swaps became exec-mask branches)
__device__ __forceinline__ float bsel(unsigned m, float a, float b) {
    return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, a) & m) | (__builtin_bit_cast(unsigned, b) & ~m));
}
__device__ __forceinline__ float2 bsel2(unsigned m, float2 a, float2 b) {
    return make_float2(bsel(m, a.x, b.x), bsel(m, a.y, b.y));
}

// decibel.rs:49-55 (ref 1: log_ref = 0) then the factor pass (:65 / :75), glibc log10f. Branch-free:
// log10f_normal runs on max(x, amin) (amin = 1e-18 / 1e-36, normal floats; the log of x > amin is
// glibc's, the other branch is the plan's log_amin) and the select keeps the reference's order.
// tab: logf's 16-entry table (an LDS copy: a per-lane constant-memory lookup is a global load).
__device__ __forceinline__ float rdb(float x, float log_amin, float amin, float factor,
                                     const exact::LogfEntry* tab = exact::kLogfT) {
    const float l = exact::log10f_normal_tab(x > amin ? x : amin, tab);
    const float y = x > amin ? l - 0.0f : log_amin - 0.0f;
    return factor * y;
}
// the LDS copy of logf's table (64 floats at lds_tab), filled by the block's threads
__device__ __forceinline__ const exact::LogfEntry* logf_tab_to_lds(float* lds_tab) {
    exact::LogfEntry* t = reinterpret_cast<exact::LogfEntry*>(lds_tab);
    if (threadIdx.x < 16) t[threadIdx.x] = exact::kLogfT[threadIdx.x];
    return t;
}

// rustfft butterfly_8 (the base level for odd log2(NC); oracle bfly8): Butterfly4 on the even
// and the odd points, twiddle(1, 8) / -i / twiddle(3, 8) on odd outputs 1..3, then bfly2 pairs
__device__ __forceinline__ void rbfly8(float2 (&b)[8], float2 w1, float2 w3) {
    float2 s0 = b[0], s1 = b[2], s2 = b[4], s3 = b[6], s4 = b[1], s5 = b[3], s6 = b[5], s7 = b[7];
    rbfly4(s0, s1, s2, s3);
    rbfly4(s4, s5, s6, s7);
    s5 = rmul(s5, w1);
    s6 = make_float2(s6.y, -s6.x);
    s7 = rmul(s7, w3);
    b[0] = cadd(s0, s4); b[4] = csub(s0, s4);
    b[1] = cadd(s1, s5); b[5] = csub(s1, s5);
    b[2] = cadd(s2, s6); b[6] = csub(s2, s6);
    b[3] = cadd(s3, s7); b[7] = csub(s3, s7);
}

}  // namespace thesia
