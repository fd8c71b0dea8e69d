// stft3_core.hpp -- pieces shared by the streaming STFT kernels (stft3_kernels.hip: every
// streaming size at 2 waves/SIMD; stft5_kernels.hip: n_fft 2048 at 3 waves/SIMD): geometry of
// the register ring, the LDS-staged row stores and the reflect-padded frame load.
#pragma once

#include "stft2_core.hpp"

namespace thesia {

// WV waves per block, one block per CU: WV / 4 waves per SIMD (8: 2 waves/SIMD, 256 VGPRs;
// 12: 3 waves/SIMD, 168 VGPRs).
template <int NC, int WV = kWaves>
struct Geo3 {
    using G2 = Geo2<NC>;
    static constexpr int L = G2::L, P = G2::P, FPW = G2::FPW;
    // the wide (ds_read_b128) transpose for the headline size, L = 32 (fft2 WIDE)
    static constexpr bool WIDE = L == 32;
    // Per-frame region stride and slot offset (gfx950 banking, MI355X_MICROARCH.md LDS table).
    // The narrow transpose writes a frame's L lanes as ds_write_b32 (32-lane groups, bank = dword
    // mod 32) and reads them back as ds_read2_b64 (16-lane groups, 2 dwords each, mod 32). With
    // L = 16 the two frames of a 32-lane group must sit 16 banks apart (stride = 16 mod 32); with
    // L = 8 the four frames must take bank offsets {0, 16, 8, 24} (writes) while the two frames
    // of a 16-lane read group sit 16 apart (row stride L + 2 = 10 fills the other 16 even banks):
    // stride = 16 mod 32 and 8 more floats for slots 2, 3 mod 4. (The previous strides, = 0 mod
    // 32 for L = 16 and without the slot offset for L = 8, put every transpose write at 2-way.)
    static constexpr bool SWZ8 = !WIDE && L == 8;
    static constexpr int SWZ_MAX = SWZ8 ? 8 : 0;
    __host__ __device__ static constexpr int swz(int slot) { return SWZ8 ? 8 * ((slot >> 1) & 1) : 0; }
    static constexpr bool BANKED = !WIDE && (L == 8 || L == 16);
    static constexpr int stride_for(int need) { return BANKED ? round_to_mod32(need + SWZ_MAX, 16) : need; }
    static constexpr int RS = WIDE ? (P * fft2_stride<NC>(true) + 3) / 4 * 4
                                   : BANKED ? stride_for(G2::XREG > G2::F4 ? G2::XREG : G2::F4) : G2::RS;
    static constexpr int SH = P / 4;                      // points per lane a hop moves
    static constexpr int BLOCK = 64 * WV;
    static constexpr int STREAMS = WV * FPW;              // streams (= frames in flight) per block
    static constexpr int TW_FLOATS = 2 * P * L;           // W_NC^{j*k1}, [P][L] float2
    // window per lane: row j holds (w[2m], w[2m+1]) for m = L*n1 + j, n1 < P, read as float4;
    // row stride 2P + 4 floats keeps 16 lanes of a ds_read_b128 group on distinct banks
    static constexpr int WL_STRIDE = 2 * P + 4;
    static constexpr int WL_FLOATS = L * WL_STRIDE;
    static constexpr int BASE_FLOATS = WL_FLOATS + TW_FLOATS + STREAMS * RS;
    // linear / complex kinds stage the whole output row in the stream's region (plus up to 3
    // floats of alignment shift) so it leaves as 16-byte aligned stores
    static constexpr int ROW_FLOATS_OK(int ok) { return ok == 0 ? 2 * G2::F : G2::F; }
    // (+32: a row staged from its 128-byte line start, line_rows, is up to 31 floats in)
    static constexpr int RS_OK(bool staged, int ok) {
        return !staged ? RS
               : (RS >= (ROW_FLOATS_OK(ok) + 32 + 3) / 4 * 4 + SWZ_MAX ? RS
                                                                      : stride_for((ROW_FLOATS_OK(ok) + 32 + 3) / 4 * 4));
    }
    static constexpr int BASE_FLOATS_OK(bool staged, int ok) { return WL_FLOATS + TW_FLOATS + STREAMS * RS_OK(staged, ok); }
    static_assert(P % 4 == 0, "hop = n_fft/4 must move whole points per lane");
    static_assert(RS % 4 == 0 && SWZ_MAX % 4 == 0, "16-byte aligned regions");
    static_assert(RS >= G2::XREG + SWZ_MAX && RS >= G2::F4 + SWZ_MAX, "a slot's offset region stays in its stride");
};

// Which kinds stage their output row (measured): linear kinds yes (power dB 6.25
// vs 6.58 ms), complex no (7.50 vs 7.41 ms; HBM write traffic equals the algorithmic bytes
// either way). VAR bit10 flips the choice.
constexpr bool stage_rows(int ok, int var) {
    return ok == 1 ? (var & 1024) == 0 : ok == 0 ? (var & (1024 | 2048)) != 0 : false;
}
// complex rows staged and stored as whole 128-byte lines with the shared line carried from frame
// to frame of a stream (VAR bit11; thesia_batch_set_option ROW_STORE = 2)
constexpr bool line_rows(int ok, int var) { return ok == 0 && (var & 2048) != 0; }

// A row of nfl floats staged in LDS (row element e at stage[sh + e], sh = the row's global
// float offset mod 4) written with 16-byte aligned stores: whole float4 chunks from the L lanes
// of the frame, the row's partial first/last chunk float by float. Rows of 1025 floats
// (linear kinds) or 1025 float2 (complex) are not 16-byte aligned, so lane-wise 4- or 8-byte
// stores of them leave partial 64-byte segments that HBM writes back twice.
template <int L>
__device__ __forceinline__ void store_row_b128(float* row, int sh, const float* stage, int nfl, int j) {
    float* ab = row - sh;  // 16-byte aligned
    const int nch = (sh + nfl + 3) >> 2;
    for (int i = j; i < nch; i += L) {
        const int e0 = 4 * i;
        if (e0 >= sh && e0 + 4 <= sh + nfl) {
            const float4 v = *reinterpret_cast<const float4*>(__builtin_assume_aligned(stage + e0, 16));
            *reinterpret_cast<float4*>(__builtin_assume_aligned(ab + e0, 16)) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e0 + e >= sh && e0 + e < sh + nfl) ab[e0 + e] = stage[e0 + e];
        }
    }
}

// Reflect-padded, downmixed samples of a frame (no window): the uniform rule of
// load_frame_generic (stft_common.hpp) for win = n_fft.
template <int NC, int INF>
__device__ __forceinline__ void load_raw_generic(const StftLaunch& a, float* region, int j,
                                                 int64_t start, int64_t n, uint64_t base, int C,
                                                 bool fold, float2 (&raw)[Geo2<NC>::P]) {
    constexpr int L = Geo2<NC>::L, P = Geo2<NC>::P;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        wave_lds_sync();
        for (int n1 = 0; n1 < P; ++n1) {
            const int m = L * n1 + j;
            int64_t i = start + 2 * m + e;
            if (i < 0) i = -i;
            if (i > n - 1) i = 2 * (n - 1) - i;
            i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
            region[m] = read_sample<INF>(a.in, base, i, C, fold);
        }
        wave_lds_sync();
        static_for<0, P>([&](auto ic) {
            constexpr int n1 = decltype(ic)::value;
            const float r = region[L * n1 + j];
            if (e == 0) raw[n1].x = r; else raw[n1].y = r;
        });
    }
}

// The same load with the runtime fill loop out of line: the rare reflect / unaligned frames
// then cost the hot loop no registers (the inline loop's 64-bit index arithmetic and the
// channel fold made the register allocator spill the ring across the whole loop body).
template <int L, int P, int INF>
__device__ __attribute__((noinline)) void fill_raw_half(const void* in, float* region, int j,
                                                         int64_t start, int64_t n, uint64_t base,
                                                         int C, bool fold, int e) {
    for (int n1 = 0; n1 < P; ++n1) {
        const int m = L * n1 + j;
        int64_t i = start + 2 * m + e;
        if (i < 0) i = -i;
        if (i > n - 1) i = 2 * (n - 1) - i;
        i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
        region[m] = read_sample<INF>(in, base, i, C, fold);
    }
}

template <int NC, int INF>
__device__ __forceinline__ void load_raw_generic_ool(const StftLaunch& a, float* region, int j,
                                                     int64_t start, int64_t n, uint64_t base, int C,
                                                     bool fold, float2 (&raw)[Geo2<NC>::P], int rot = 0) {
    // rot: the ring's slot map (stft5 THESIA_RING5): slot n1 holds point (n1 - rot) mod P
    constexpr int L = Geo2<NC>::L, P = Geo2<NC>::P;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        wave_lds_sync();
        fill_raw_half<L, P, INF>(a.in, region, j, start, n, base, C, fold, e);
        wave_lds_sync();
        static_for<0, P>([&](auto ic) {
            constexpr int n1 = decltype(ic)::value;
            const float r = region[L * ((n1 + P - rot) & (P - 1)) + j];
            if (e == 0) raw[n1].x = r; else raw[n1].y = r;
        });
    }
}

}  // namespace thesia
