// stft_common.hpp -- device helpers shared by the STFT kernels (stft_kernels.hip: the
// general kernel for every n_fft; stft2_kernels.hip: the 4-waves/SIMD kernel for the large
// sizes). Input decode / downmix, track lookup, dB epilogue.
#pragma once

#include <algorithm>

#include "device_fft.hpp"
#include "kernels.hpp"

namespace thesia {

constexpr int kWaves = 8;
constexpr int kBlock = 64 * kWaves;

constexpr int round_to_mod32(int v, int r) {
    while (((v % 32) + 32) % 32 != r) ++v;
    return v;
}

template <int NC>
struct Geo {
    static constexpr int L = geo_L(NC);
    static constexpr int P = geo_P(NC);
    static constexpr int FPW = 64 / L;           // frames per wave per pass
    static constexpr int F = NC + 1;             // rfft bins
    static constexpr int XREG = P * (L + 1);     // exchange floats per frame (>= F)
    static constexpr int RS = round_to_mod32(XREG, L % 32);  // per-frame LDS region stride
    static constexpr int PASS_FRAMES = kWaves * FPW;
    static constexpr int WIN_FLOATS = ((2 * NC) + 3) / 4 * 4; // window table in LDS
    // twiddle bases: W_NC^{j*k1}, k1 = TB*a + b
    static constexpr int TB = P < 8 ? P : 8;
    static constexpr int TA = P / TB;
    static constexpr int MIN_WAVES = P >= 32 ? 2 : 4;         // VGPR cap 256 / 128
    static constexpr int LCH = P < 8 ? P : 8;                 // direct-load chunk
    static_assert(P % L == 0, "P must be a multiple of L");
    static_assert(XREG >= F, "the |X| row must fit the frame's region");
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Channel-sum downmix in ndarray's unrolled_fold order (lib.rs:42 -> sum_axis on a
// channel-contiguous view -> numeric_util::unrolled_fold).
template <int INF>
__device__ __forceinline__ float chan_val(const void* in, uint64_t idx) {
    if constexpr (INF == IN_S16) {
        return (float)static_cast<const int16_t*>(in)[idx] / 32768.0f;  // audio.rs:18
    } else {
        return static_cast<const float*>(in)[idx];
    }
}

template <int INF>
__device__ __forceinline__ float read_sample_wide(const void* in, uint64_t p, int C) {
    float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f, q4 = 0.f, q5 = 0.f, q6 = 0.f, q7 = 0.f;
    int c = 0;
    for (; C - c >= 8; c += 8) {
        q0 = q0 + chan_val<INF>(in, p + c + 0); q1 = q1 + chan_val<INF>(in, p + c + 1);
        q2 = q2 + chan_val<INF>(in, p + c + 2); q3 = q3 + chan_val<INF>(in, p + c + 3);
        q4 = q4 + chan_val<INF>(in, p + c + 4); q5 = q5 + chan_val<INF>(in, p + c + 5);
        q6 = q6 + chan_val<INF>(in, p + c + 6); q7 = q7 + chan_val<INF>(in, p + c + 7);
    }
    float acc = 0.0f;
    acc = acc + (q0 + q4);
    acc = acc + (q1 + q5);
    acc = acc + (q2 + q6);
    acc = acc + (q3 + q7);
    for (; c < C; ++c) acc = acc + chan_val<INF>(in, p + c);
    return acc;
}

template <int INF>
__device__ __forceinline__ float read_sample(const void* in, uint64_t base, int64_t i, int C,
                                             bool fold) {
    const uint64_t p = base + (uint64_t)i * (uint64_t)C;
    if (!fold) return chan_val<INF>(in, p);
    if (C == 1) return 0.0f + chan_val<INF>(in, p);
    if (C == 2) return (0.0f + chan_val<INF>(in, p)) + chan_val<INF>(in, p + 1);
    if (C < 8) {
        float acc = 0.0f;
        for (int c = 0; c < C; ++c) acc = acc + chan_val<INF>(in, p + c);
        return acc;
    }
    return read_sample_wide<INF>(in, p, C);
}

__device__ __forceinline__ int find_track(const uint64_t* f0, int n_tracks, uint64_t g, int hint) {
    if (hint < 0 || g < f0[hint]) {
        int lo = 0, hi = n_tracks;  // f0[lo] <= g < f0[hi]
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (f0[mid] <= g) lo = mid; else hi = mid;
        }
        return lo;
    }
    while (hint + 1 < n_tracks && g >= f0[hint + 1]) ++hint;
    return hint;
}

__device__ __forceinline__ float db_of(float x, float log_amin, float amin, float factor) {
    // decibel.rs:49-55 with ref = 1 (log_ref = 0) then the separate *factor pass (:65/:75).
    // log10(x) = log2(x) * log10(2) with the hardware v_log_f32: x > amin >= 1e-36 is a
    // normal float, so no denormal pre-scaling is needed; within a few ulp of glibc log10f
    // (the reference's f32::log10), i.e. <= 1e-4 dB, far inside tests/tolerances.py.
    float l = x > amin ? __builtin_amdgcn_logf(x) * 0.30102999566398119521f : log_amin;
    return factor * (l - 0.0f);
}

// Amp dB of a bin from its |X|^2 p (fast kernels): 20 log10(sqrt(p)) = 10 log10(p), and
// |X| > amin = 1e-18 <=> p > 1e-36 (a normal float), the clamp 20 log10(amin) = 10 (2 log10(amin))
// exactly (log_amin is the plan's log10(1e-18)). One v_log_f32 instead of v_sqrt + v_log: the
// rounding differs from db_of(sqrt(p)) by a few ulp of the log, inside tests/tolerances.py.
__device__ __forceinline__ float amp_db_of(float p, float log_amin) {
    const float l = p > 1e-36f ? __builtin_amdgcn_logf(p) * 0.30102999566398119521f : 2.0f * log_amin;
    return 10.0f * (l - 0.0f);
}

// Output row stores. Plain stores: non-temporal ones (THESIA_NT_STORES, experiment) measured
// slower and bimodal on the complex-output kernel (7.6 / 10.1 ms vs 6.24 ms).
#ifdef THESIA_NT_STORES
__device__ __forceinline__ void st_out(float* p, float v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_out(float2* p, float2 v) {
    typedef float v2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(v2{v.x, v.y}, reinterpret_cast<v2*>(p));
}
#else
__device__ __forceinline__ void st_out(float* p, float v) { *p = v; }
__device__ __forceinline__ void st_out(float2* p, float2 v) { *p = v; }
#endif

// |X| = hypot(re, im): v_sqrt_f32 of the f32 sum of squares (<= 1.5 ulp; the product kernel
// is parity-by-tolerance against glibc hypotf). VAR bit0 selects the correctly-rounded
// sqrt sequence instead (experiment).
template <int VAR>
__device__ __forceinline__ float vsqrt(float x) {
    if constexpr ((VAR & 1) != 0) return __builtin_sqrtf(x);
    else return __builtin_amdgcn_sqrtf(x);
}


// ------------------------------------------------------------------------------------
// frame loads (window product in the reference order: x_ref[...] * w[k], lib.rs:379)
// ------------------------------------------------------------------------------------
// Generic path (track edges / unaligned / any format): a runtime loop writes this lane's
// windowed samples into the frame's LDS region (even, then odd positions), static reads
// fill the registers. Reflection about samples 0 and n-1 (the uniform rule, proved equal
// to lib.rs:410-435 in tests/test_oracle.py).
template <int NC, int INF>
__device__ __forceinline__ void load_frame_generic(const StftLaunch& a, float* region, int j,
                                                   int64_t start, int64_t n, uint64_t base,
                                                   int C, bool fold, const float* wtab,
                                                   float2 (&v)[Geo<NC>::P]) {
    constexpr int L = Geo<NC>::L, P = Geo<NC>::P;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        wave_lds_sync();
        for (int n1 = 0; n1 < P; ++n1) {
            const int m = L * n1 + j;
            const int jj = 2 * m + e;
            float val = 0.0f;
            if (jj >= a.pad_left && jj < a.pad_left + a.win) {
                int64_t i = start + jj;
                if (i < 0) i = -i;
                if (i > n - 1) i = 2 * (n - 1) - i;
                i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
                val = read_sample<INF>(a.in, base, i, C, fold) * wtab[jj];
            }
            region[m] = val;
        }
        wave_lds_sync();
        static_for<0, P>([&](auto ic) {
            constexpr int n1 = decltype(ic)::value;
            const float r = region[L * n1 + j];
            if (e == 0) v[n1].x = r; else v[n1].y = r;
        });
    }
}

template <int NC>
__device__ __forceinline__ void twiddle_bases(const StftLaunch& a, int j, float2 (&twb)[Geo<NC>::TB],
                                              float2 (&twa)[Geo<NC>::TA],
                                              float2 (&ub)[Geo<NC>::P / Geo<NC>::L]) {
    using G = Geo<NC>;
    constexpr int L = G::L, TB = G::TB, TA = G::TA, CPL = G::P / G::L;
    // W_NC^{j*b}, W_NC^{j*TB*aa}: f64-rounded table values (like rustfft's twiddles)
#pragma unroll
    for (int b = 0; b < TB; ++b) twb[b] = a.tw1[(j * b) % NC];
#pragma unroll
    for (int aa = 0; aa < TA; ++aa) twa[aa] = a.tw1[(j * TB * aa) % NC];
    // untangle bases (sin, cos)(pi*(j + c*L)/NC) straight from the reference table (k < P)
#pragma unroll
    for (int c = 0; c < CPL; ++c) ub[c] = a.sincos[j + c * L];
}

// Grid for a persistent launch: resident blocks per CU x CUs, capped by the tile count.
// grid_req > 0: at most that many blocks; else one occupancy wave of the device, scaled by
// share in (0, 1] when several launches run side by side (thesia_batches_run: each batch on its
// share of the CUs, so its frame streams walk longer)
inline int grid_for(const void* kern, int block, int lds, uint64_t n_tiles, int grid_req, float share = 0.f) {
    int grid = grid_req;
    if (grid <= 0) {
        int dev = 0, cus = 256, per_cu = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, lds) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        grid = cus * per_cu;
        if (share > 0.f && share < 1.f) grid = std::max(1, (int)((float)grid * share + 0.5f));
    }
    if ((uint64_t)grid > n_tiles) grid = (int)n_tiles;
    return grid;
}

}  // namespace thesia
