// display_common.hpp -- per-pixel device helpers shared by the display kernels (display.rs):
// the grey value of one dB sample (display.rs:44-54), Rust's saturating `as u8`, and the
// 10-stop colormap lerp (display.rs:24-42). Compiled with -ffp-contract=off like every kernel:
// the same f32 operations, in the same order, as the oracle.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace thesia {

__device__ __forceinline__ uint8_t sat_u8(float v) {  // Rust `as u8`
    if (!(v == v)) return 0;
    if (v <= 0.0f) return 0;
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}

// the colormap of one horizontal-pass value (display.rs:24-42), as resize_h_rgb_px
__device__ __forceinline__ void colormap_px(float t, const uint8_t* cmap, uint8_t* o) {
    float x = t;
    if (!(x >= 0.0f)) x = 0.0f;
    const float position = 10.0f * x;
    const float fl = floorf(position);
    if (fl >= 9.0f) {
        o[0] = cmap[27];
        o[1] = cmap[28];
        o[2] = cmap[29];
        return;
    }
    const int index = (int)fl;
    const float ratio = position - (float)index;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float av = (float)cmap[index * 3 + c], bv = (float)cmap[(index + 1) * 3 + c];
        o[c] = sat_u8(roundf(ratio * bv + (1.0f - ratio) * av));
    }
}

// roundf(v) then Rust `as u8`, for a colormap lerp value 0 <= v <= 255 (a convex combination of
// two stop bytes; at most 255 (1 + 2^-24) after rounding): for v >= 0.5, floor(v + 0.5) is
// roundf(v) (the sum is exact, or rounds inside [2^k, 2^k + 1) when it crosses a binade), and
// the conversion truncates; below 0.5 roundf gives 0 while v + 0.5 may round up to 1.0. Four
// VALU, no branch (tests/test_colormap_exhaustive.py checks colormap_rgb against the oracle on every float).
__host__ __device__ __forceinline__ uint32_t round_u8(float v) {
    const uint32_t u = (uint32_t)(v + 0.5f);
    return v < 0.5f ? 0u : u;
}

// The colormap's stops as pairs {stop i, stop min(i + 1, 9)} (3 bytes each in a dword) for
// colormap_rgb: entry i of the LUT a kernel keeps in LDS.
__host__ __device__ __forceinline__ uint2 colormap_pair(const uint8_t* cmap, int i) {
    const int i2 = i < 9 ? i + 1 : 9;
    return make_uint2((uint32_t)cmap[3 * i] | (uint32_t)cmap[3 * i + 1] << 8 | (uint32_t)cmap[3 * i + 2] << 16,
                      (uint32_t)cmap[3 * i2] | (uint32_t)cmap[3 * i2 + 1] << 8 | (uint32_t)cmap[3 * i2 + 2] << 16);
}

// colormap_px (display.rs:24-42) from the paired-stop LUT: one ds_read_b64 per pixel instead of
// six byte reads, no branch; the bytes r | g << 8 | b << 16. Same operations on every value:
// t < 0 / NaN -> 0; position 10 t; below stop 9 the lerp of stops floor(position) and + 1 with
// ratio position - floor(position) (= position - (float)index: floor is integral); from stop 9
// on, the pair (stop 9, stop 9) with ratio 0, i.e. 0 * b + 1 * a = a exactly.
struct CmapPos {
    int index;    // the LUT entry
    float ratio;  // its lerp weight
};
__host__ __device__ __forceinline__ CmapPos colormap_pos(float t) {
    const float x = fmaxf(t, 0.0f);  // NaN and negatives -> 0 (-0 and +0 give the same bytes)
    const float position = 10.0f * x;
    const float fl = floorf(position);
    const bool top = fl >= 9.0f;
    return CmapPos{top ? 9 : (int)fl, top ? 0.0f : position - fl};
}
__host__ __device__ __forceinline__ uint32_t colormap_lerp(uint2 e, float ratio) {
    const float om = 1.0f - ratio;
    const uint32_t r = round_u8(ratio * (float)(e.y & 0xFF) + om * (float)(e.x & 0xFF));
    const uint32_t g = round_u8(ratio * (float)((e.y >> 8) & 0xFF) + om * (float)((e.x >> 8) & 0xFF));
    const uint32_t b = round_u8(ratio * (float)((e.y >> 16) & 0xFF) + om * (float)((e.x >> 16) & 0xFF));
    return r | (g << 8) | (b << 16);
}
__host__ __device__ __forceinline__ uint32_t colormap_rgb(float t, const uint2* lut) {
    const CmapPos p = colormap_pos(t);
    return colormap_lerp(lut[p.index], p.ratio);
}

__device__ __forceinline__ float grey_of(float db, float max, float min) {  // grey_px
    float v = (db - min) / (max - min);
    v = fmaxf(v, 0.0f);
    return fminf(v, 1.0f);
}

// grey_of without the f32 division sequence (11 VALU with a v_rcp): the f32 difference a =
// db - min times the f64 reciprocal of the f32 span b = max - min, rounded once to f32. The
// product is within 2^-52 (relative) of a / b, and for a normal quotient that is closer than any
// f32 rounding midpoint can be to a quotient of two f32 (a midpoint there has 25 significant bits,
// so a - b m is a nonzero multiple of b m's 49-bit grid: > 2^-49 relative), so the result is
// RN(a / b) bit for bit. Below the normal range exact ties exist (midpoints with few significant
// bits): those quotients, zero and non-finite ones are divided in f32 (tests/test_grey_map.py).
struct GreyMap {
    float min, span;
    double rspan;
    __host__ __device__ GreyMap(float max, float mn) : min(mn), span(max - mn), rspan(1.0 / (double)(max - mn)) {}
    __host__ __device__ __forceinline__ float operator()(float db) const {
        const float a = db - min;
        float v = (float)((double)a * rspan);
#ifdef __HIP_DEVICE_COMPILE__
        const bool normal = __builtin_amdgcn_classf(v, 0x108);  // +-normal: one v_cmp_class
#else
        const bool normal = fabsf(v) >= 1.17549435e-38f && fabsf(v) <= 3.40282347e+38f;
#endif
        if (!normal) {
            // a real branch (rarely taken), not a division formed for every element and selected
            float t = a;
#ifdef __HIP_DEVICE_COMPILE__
            asm volatile("" : "+v"(t));
#endif
            v = t / span;
        }
        v = fmaxf(v, 0.0f);
        return fminf(v, 1.0f);
    }
};

}  // namespace thesia
