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

__device__ __forceinline__ float grey_of(float db, float max, float min) {  // grey_px
    float v = (db - min) / (max - min);
    v = fmaxf(v, 0.0f);
    return fminf(v, 1.0f);
}

}  // namespace thesia
