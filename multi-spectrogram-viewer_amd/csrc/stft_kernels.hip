// stft_kernels.hip -- fused frame + window + real FFT + |X| (+ mel) + dB for gfx950.
//
// Replaces, on the device, the reference hot loop
//   perform_stft (lib.rs:388-471) -> RealFFT::process (realfft.rs:105-159)
//   -> stft.mapv(norm) (lib.rs:124) -> linspec.dot(mel_fb) (lib.rs:131)
//   -> amp_to_db_default (decibel.rs:79-88)
// for a whole batch of tracks in one launch.
//
// Layout / schedule (DESIGN.md "K1"):
//  * global frame index g runs over all tracks of a batch (packed output rows);
//  * a 64-lane wave owns FPW = 64/L frames; lane (slot, n2) holds P complex points
//    z[L*n1 + n2] = (x[2m], x[2m+1]) of its frame (the realfft.rs:130-134 packing);
//  * stage 1: P-point DFT in registers + W_NC^{n2 k1} twiddles; LDS transpose (re, im
//    halves through one per-frame region); stage 2: P/L L-point DFTs in registers;
//  * the realfft untangle (realfft.rs:140-157) pairs Z[k] with Z[NC-k]: the partner
//    lives in lane (L - j) mod L of the same frame and is fetched with ds_bpermute;
//  * every wave is independent (no block barriers after the prologue): linear kinds stream
//    rows out per bin straight from the untangle;
//  * mel kinds keep the frame's |X| row in its LDS region and project it onto the band-
//    sparse filterbank with a per-lane fma chain: round r gives lane j of the frame mel
//    r*L + j, all lanes of a round run the round's longest band (zero weights pad the
//    shorter ones), so stores are coalesced and the loop is wave-uniform. The chain runs
//    over k ascending from 0, the order of the oracle's dot (bit-exact for equal |X|).
//    (f32 MFMA runs at the VALU FMA rate on gfx950 and the filterbank is ~1.5% dense: a
//    16x16x4 MFMA tiling of it was measured slower, DESIGN.md "mel projection".)
// Built with -ffp-contract=off: arithmetic that has a reference order (window product,
// downmix, untangle, dB) is evaluated exactly in that order; FFT butterflies use explicit
// fmaf (their order is not pinned to rustfft's, parity there is by tolerance).
#include "stft_common.hpp"

#include <algorithm>
#include <cstdlib>

namespace thesia {

struct LaneCtx {
    int lane, wave, slot, j, partner;
};

template <int NC>
__device__ __forceinline__ LaneCtx lane_ctx() {
    constexpr int L = Geo<NC>::L;
    LaneCtx c;
    c.lane = threadIdx.x & 63;
    c.wave = threadIdx.x >> 6;
    c.slot = c.lane / L;
    c.j = c.lane % L;
    c.partner = c.slot * L + ((L - c.j) % L);
    return c;
}

// Direct global path for interior frames of f32 mono / stereo input (8 / 16 B per lane).
// Returns false when not applicable (caller falls back to the generic path).
template <int NC, int INF>
__device__ __forceinline__ bool load_frame_direct(const StftLaunch& a, int j, int64_t start,
                                                  int64_t n, uint64_t base, int C, bool fold,
                                                  const float* wtab, float2 (&v)[Geo<NC>::P]) {
    using G = Geo<NC>;
    constexpr int L = G::L, P = G::P, LCH = G::LCH;
    if constexpr (INF != IN_F32) {
        return false;
    } else {
        const bool interior = a.pad_left == 0 && a.win == 2 * NC && start >= 0 && start + 2 * NC <= n;
        if (!interior) return false;
        if (C == 1 && !fold && ((base + start) & 1) == 0) {
            const float2* src = reinterpret_cast<const float2*>(static_cast<const float*>(a.in) + base + start) + j;
            static_for<0, P / LCH>([&](auto gc) {
                constexpr int g8 = decltype(gc)::value;
                static_for<0, LCH>([&](auto ic) {
                    constexpr int n1 = LCH * g8 + decltype(ic)::value;
                    const int m = L * n1 + j;
                    const float2 x = src[L * n1];
                    v[n1] = make_float2(x.x * wtab[2 * m], x.y * wtab[2 * m + 1]);
                });
                pin_range<LCH * g8, LCH * g8 + LCH>(v);
            });
            return true;
        }
        if (C == 2 && fold && ((base + 2 * start) & 3) == 0) {
            const float4* src = reinterpret_cast<const float4*>(static_cast<const float*>(a.in) + base + 2 * start) + j;
            static_for<0, P / LCH>([&](auto gc) {
                constexpr int g8 = decltype(gc)::value;
                static_for<0, LCH>([&](auto ic) {
                    constexpr int n1 = LCH * g8 + decltype(ic)::value;
                    const int m = L * n1 + j;
                    const float4 x = src[L * n1];
                    const float s0 = (0.0f + x.x) + x.y, s1 = (0.0f + x.z) + x.w;
                    v[n1] = make_float2(s0 * wtab[2 * m], s1 * wtab[2 * m + 1]);
                });
                pin_range<LCH * g8, LCH * g8 + LCH>(v);
            });
            return true;
        }
        return false;
    }
}

// ------------------------------------------------------------------------------------
// FFT core: stage-1 DFT_P + twiddles, LDS transpose, stage-2 DFT_L (v -> w2r)
// ------------------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void fft_core(float2 (&v)[Geo<NC>::P], float2 (&w2r)[Geo<NC>::P],
                                         float* region, int j, const float2 (&twb)[Geo<NC>::TB],
                                         const float2 (&twa)[Geo<NC>::TA]) {
    using G = Geo<NC>;
    constexpr int L = G::L, P = G::P, TB = G::TB, CPL = P / L;
    pin(v);
    dif_fft<P, 1, 0, P>(v);
    pin(v);
    wave_lds_sync();
    static_for<0, P>([&](auto kc) {
        constexpr int k1 = decltype(kc)::value;
        constexpr int b = k1 % TB, aa = k1 / TB;
        constexpr int pk = ce_pos(P, k1);
        float2 x = v[pk];
        if constexpr (b != 0) x = cmul(x, twb[b]);
        if constexpr (aa != 0) x = cmul(x, twa[aa]);
        v[pk] = x;
        region[k1 * (L + 1) + j] = x.x;
    });
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int q = 0; q < L; ++q) w2r[c * L + q].x = region[(j + c * L) * (L + 1) + q];
    wave_lds_sync();
    static_for<0, P>([&](auto kc) {
        constexpr int k1 = decltype(kc)::value;
        constexpr int pk = ce_pos(P, k1);
        region[k1 * (L + 1) + j] = v[pk].y;
    });
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int q = 0; q < L; ++q) w2r[c * L + q].y = region[(j + c * L) * (L + 1) + q];
    wave_lds_sync();
    pin(w2r);
    static_for<0, CPL>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        dif_fft<L, 1, c * L, P>(w2r);
    });
    pin(w2r);
}

// realfft untangle (realfft.rs:140-157): calls epi(k, xr, xi) for every bin this lane owns
// (k = j + c*L + P*k2) and, on lane j == 0, the Nyquist bin NC.
template <int NC, class Epi>
__device__ __forceinline__ void untangle(float2 (&w2r)[Geo<NC>::P], int j, int partner,
                                         const float2 (&ub)[Geo<NC>::P / Geo<NC>::L], Epi&& epi) {
    using G = Geo<NC>;
    constexpr int L = G::L, P = G::P, CPL = P / L;
    static_for<0, CPL>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        static_for<0, L>([&](auto k2c) {
            constexpr int k2 = decltype(k2c)::value;
            constexpr int pb = c * L + ce_pos(L, k2);
            const float2 b = w2r[pb];
            // partner Z[NC-k] for k = j + c*L + P*k2
            constexpr int cp = CPL - 1 - c;
            constexpr int k2p = L - 1 - k2;
            constexpr int ps = cp * L + ce_pos(L, k2p);
            const float2 send = w2r[ps];
            float2 r;
            r.x = __shfl(send.x, partner, 64);
            r.y = __shfl(send.y, partner, 64);
            if (j == 0) {  // self-paired lane (k1 multiple of L)
                constexpr int c0 = (c == 0) ? 0 : CPL - c;
                constexpr int k20 = (c == 0) ? ((L - k2) % L) : (L - 1 - k2);
                constexpr int p0 = c0 * L + ce_pos(L, k20);
                r = w2r[p0];
            }
            const int k = j + c * L + P * k2;
            // (sin, cos)(pi k / NC) = base(j + cL) rotated by pi*k2/L
            float s, co;
            if constexpr (k2 == 0) {
                s = ub[c].x;
                co = ub[c].y;
            } else {
                constexpr float cb = ce_tw_re(k2, 2 * L);   // cos(pi k2 / L)
                constexpr float sb = -ce_tw_im(k2, 2 * L);  // sin(pi k2 / L)
                s = __builtin_fmaf(ub[c].x, cb, ub[c].y * sb);
                co = __builtin_fmaf(ub[c].y, cb, -(ub[c].x * sb));
            }
            // realfft.rs:148-154, evaluated in the reference's order
            const float xr = 0.5f * (((b.x + r.x) + co * (b.y + r.y)) - s * (b.x - r.x));
            const float xi = 0.5f * (((b.y - r.y) - s * (b.y + r.y)) - co * (b.x - r.x));
            epi(k, xr, xi);
            pin(w2r);
        });
    });
    if (j == 0) {  // Nyquist bin, realfft.rs:157
        const float2 z0 = w2r[0];
        epi(NC, z0.x - z0.y, 0.0f);
    }
}

// lib.rs:131-132: out[g, m] = amp_to_db(sum_k |X|[k] * fb[k, m]) for the frame whose |X|
// row sits in `region`. Round r: lane j owns mel r*L + j; its weights for bins
// k0 .. k0+len-1 (zero outside the filter's band) are rows mel_wt[row0 + it][j].
template <int NC>
__device__ __forceinline__ void mel_rounds(const StftLaunch& a, const float* region, int j,
                                           uint64_t g, bool valid) {
    constexpr int L = Geo<NC>::L;
    constexpr int U = 8;
    const int n_mels = a.n_mels;
    const bool db = a.out_kind == OUT_MEL_AMP_DB;
    float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
    for (int r = 0; r < a.mel_rounds; ++r) {
        const int2 rd = a.mel_round[r];  // {first weight row, band length}: wave-uniform
        const float* xp = region + a.mel_k0[r * L + j];
        const float* wp = a.mel_wt + (size_t)rd.x * L + j;
        float acc = 0.0f;
        int it = 0;
        for (; it + U <= rd.y; it += U) {
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = wp[(it + u) * L];
#pragma unroll
            for (int u = 0; u < U; ++u) acc = __builtin_fmaf(xp[it + u], w[u], acc);
        }
        for (; it < rd.y; ++it) acc = __builtin_fmaf(xp[it], wp[it * L], acc);
        const int m = r * L + j;
        if (valid && m < n_mels) out[m] = db ? db_of(acc, a.log_amin, 1e-18f, 20.0f) : acc;
    }
}

// ======================================================================================
// K1: every output kind (complex / |X| / |X|^2 / dB / mel). Waves are independent.
// VAR: experiment variants (THESIA_STFT_VARIANT, A/B in one process; production = 0).
// ======================================================================================
template <int NC, int OK, int INF, int VAR = 0>
__global__ void __launch_bounds__(kBlock, Geo<NC>::MIN_WAVES)
stft_kernel(StftLaunch a, uint64_t tiles_per_block) {
    using G = Geo<NC>;
    constexpr int P = G::P, FPW = G::FPW, F = G::F, L = G::L;
    constexpr int TILE = G::PASS_FRAMES;

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtab = lds;
    float* work = lds + G::WIN_FLOATS;
    const LaneCtx lc = lane_ctx<NC>();
    const int j = lc.j;

    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) wtab[i] = a.wpad[i];
    float2 twb[G::TB], twa[G::TA], ub[P / L];
    twiddle_bases<NC>(a, j, twb, twa, ub);
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t n_tiles = (total + TILE - 1) / TILE;
    const uint64_t t_begin = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t t_end = t_begin + tiles_per_block < n_tiles ? t_begin + tiles_per_block : n_tiles;
    const int half_win = a.win / 2;
    const int C = a.channels;
    const bool fold = a.fold != 0;
    int hint = -1;
    float* region = work + (lc.wave * FPW + lc.slot) * G::RS;

    for (uint64_t tile = t_begin; tile < t_end; ++tile) {
        const uint64_t g = tile * TILE + (uint64_t)(lc.wave * FPW + lc.slot);
        const bool valid = g < total;
        float2 v[P];
        if (valid) {
            hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
            const uint64_t t = g - a.trk_frame0[hint];
            const int64_t n = (int64_t)a.trk_len[hint];
            const uint64_t base = a.trk_in_off[hint];
            const int64_t start = (int64_t)t * a.hop - half_win - a.pad_left;
            if (!load_frame_direct<NC, INF>(a, j, start, n, base, C, fold, wtab, v))
                load_frame_generic<NC, INF>(a, region, j, start, n, base, C, fold, wtab, v);
        } else {
#pragma unroll
            for (int n1 = 0; n1 < P; ++n1) v[n1] = make_float2(0.f, 0.f);
        }
        float2 w2r[P];
        fft_core<NC>(v, w2r, region, j, twb, twa);
        const int kind = a.out_kind;
        if constexpr (OK == 2) {
            // |X| row of the frame into its region (lib.rs:124), then the mel rounds
            untangle<NC>(w2r, j, lc.partner, ub, [&](int k, float xr, float xi) {
                region[k] = vsqrt<VAR>(xr * xr + xi * xi);
            });
            wave_lds_sync();
            if constexpr ((VAR & 2) == 0) mel_rounds<NC>(a, region, j, g, valid);
            continue;
        }
        untangle<NC>(w2r, j, lc.partner, ub, [&](int k, float xr, float xi) {
            if constexpr (OK == 0) {
                if (valid) reinterpret_cast<float2*>(a.out)[g * F + k] = make_float2(xr, xi);
            } else {
                float val;
                if (kind == OUT_POWER || kind == OUT_POWER_DB) {
                    val = xr * xr + xi * xi;  // num-complex norm_sqr
                    if (kind == OUT_POWER_DB) val = db_of(val, a.log_amin, 1e-36f, 10.0f);
                } else {
                    val = vsqrt<VAR>(xr * xr + xi * xi);
                    if (kind == OUT_AMP_DB) val = db_of(val, a.log_amin, 1e-18f, 20.0f);
                }
                if (valid) static_cast<float*>(a.out)[g * F + k] = val;
            }
        });
    }
}

#ifndef THESIA_NO_DISPATCH
// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
static int ok_of(int out_kind) {
    if (out_kind == OUT_COMPLEX) return 0;
    if (out_kind == OUT_MEL || out_kind == OUT_MEL_AMP_DB) return 2;
    return 1;
}

template <int NC>
static int lds_bytes_nc() {
    using G = Geo<NC>;
    return (G::WIN_FLOATS + G::PASS_FRAMES * G::RS) * 4;
}

template <int NC, int OK, int INF, int VAR = 0>
static int launch_k(const StftLaunch& a, hipStream_t stream) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (VAR == 0 && NC == 1024 && INF == IN_F32 && OK == 2) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        switch (e ? atoi(e) : 0) {
            case 1: return launch_k<NC, OK, INF, 1>(a, stream);  // correctly-rounded sqrt
            case 2: return launch_k<NC, OK, INF, 2>(a, stream);  // mel projection skipped
            default: break;
        }
    }
#endif
    const int lds = lds_bytes_nc<NC>();
    auto kern = stft_kernel<NC, OK, INF, VAR>;
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
            return -1;
        attr_set = true;
    }
    const uint64_t n_tiles = (a.total_frames + Geo<NC>::PASS_FRAMES - 1) / Geo<NC>::PASS_FRAMES;
    if (n_tiles == 0) return 0;
    int grid = grid_for(reinterpret_cast<const void*>(kern), kBlock, lds, n_tiles, a.grid, a.grid_share);
    const uint64_t tpb = (n_tiles + grid - 1) / grid;
    grid = (int)((n_tiles + tpb - 1) / tpb);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, stream, a, tpb);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int NC, int INF>
static int launch_fmt(const StftLaunch& a, hipStream_t s) {
    switch (ok_of(a.out_kind)) {
        case 0: return launch_k<NC, 0, INF>(a, s);
        case 1: return launch_k<NC, 1, INF>(a, s);
        default: return launch_k<NC, 2, INF>(a, s);
    }
}

template <int NC>
static int launch_nc(const StftLaunch& a, hipStream_t s) {
    return a.in_format == IN_S16 ? launch_fmt<NC, IN_S16>(a, s) : launch_fmt<NC, IN_F32>(a, s);
}

int launch_stft(const StftLaunch& a, hipStream_t s) {
    switch (a.n_fft / 2) {
        case 1: return launch_nc<1>(a, s);
        case 2: return launch_nc<2>(a, s);
        case 4: return launch_nc<4>(a, s);
        case 8: return launch_nc<8>(a, s);
        case 16: return launch_nc<16>(a, s);
        case 32: return launch_nc<32>(a, s);
        case 64: return launch_nc<64>(a, s);
        case 128: return launch_nc<128>(a, s);
        case 256: return launch_nc<256>(a, s);
        case 512: return launch_nc<512>(a, s);
        case 1024: return launch_nc<1024>(a, s);
        case 2048: return launch_nc<2048>(a, s);
        default: return -2;
    }
}

int stft_kernel_info(int n_fft, int* lds_bytes, int* tile_frames, int* lanes_per_frame) {
    int lds = 0, tile = 0, L = 0;
    switch (n_fft / 2) {
#define THESIA_INFO(NC) \
        case NC: lds = lds_bytes_nc<NC>(); tile = Geo<NC>::PASS_FRAMES; L = Geo<NC>::L; break;
        THESIA_INFO(1) THESIA_INFO(2) THESIA_INFO(4) THESIA_INFO(8) THESIA_INFO(16)
        THESIA_INFO(32) THESIA_INFO(64) THESIA_INFO(128) THESIA_INFO(256) THESIA_INFO(512)
        THESIA_INFO(1024) THESIA_INFO(2048)
#undef THESIA_INFO
        default: return -2;
    }
    if (lds_bytes) *lds_bytes = lds;
    if (tile_frames) *tile_frames = tile;
    if (lanes_per_frame) *lanes_per_frame = L;
    return 0;
}
#endif  // THESIA_NO_DISPATCH

}  // namespace thesia
