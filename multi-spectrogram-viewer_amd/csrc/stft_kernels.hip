// stft_kernels.hip -- fused frame + window + real FFT + |X| (+ mel MFMA) + dB for gfx950.
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
//  * mel: |X| rows of a 16-frame tile stay in LDS and are projected with
//    v_mfma_f32_16x16x4_f32 over each 16-mel tile's bin band (block-sparse K), dB fused.
// Built with -ffp-contract=off: arithmetic that has a reference order (window product,
// untangle, dB, mel chain) is evaluated exactly in that order; FFT butterflies use
// explicit fmaf (their order is not pinned to rustfft's, parity there is by tolerance).
#include "device_fft.hpp"
#include "kernels.hpp"

#include <algorithm>

namespace thesia {

constexpr int kWaves = 8;
constexpr int kBlock = 64 * kWaves;

typedef float floatx4 __attribute__((ext_vector_type(4)));

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
    static constexpr int XREG = P * (L + 1);     // exchange floats per frame
    static constexpr int RS = round_to_mod32(XREG, L % 32);  // linear-mode region stride
    static constexpr int PASS_FRAMES = kWaves * FPW;
    static constexpr int MEL_TILE = PASS_FRAMES >= 16 ? PASS_FRAMES : 16;
    static constexpr int MEL_PASSES = MEL_TILE / PASS_FRAMES;
    static constexpr int ROW_MIN = (XREG > F + 16) ? XREG : F + 16;
    static constexpr int ROW = round_to_mod32(ROW_MIN, 2);   // mel-mode |X| row stride
    static constexpr int WIN_FLOATS = ((2 * NC) + 3) / 4 * 4; // window table in LDS
    // twiddle bases: W_NC^{j*k1}, k1 = TB*a + b
    static constexpr int TB = P < 8 ? P : 8;
    static constexpr int TA = P / TB;
    static constexpr int MIN_WAVES = P >= 32 ? 2 : 4;         // VGPR cap 256 / 128
    static_assert(P % L == 0, "P must be a multiple of L");
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
__device__ __noinline__ float read_sample_wide(const void* in, uint64_t p, int C) {
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
    // decibel.rs:49-55 with ref = 1 (log_ref = 0) then the separate *factor pass (:65/:75)
    float l = x > amin ? log10f(x) : log_amin;
    return factor * (l - 0.0f);
}

template <int NC, int OK, int INF>
__global__ void __launch_bounds__(kBlock, Geo<NC>::MIN_WAVES)
stft_kernel(StftLaunch a, uint64_t tiles_per_block) {
    using G = Geo<NC>;
    constexpr int L = G::L, P = G::P, FPW = G::FPW, F = G::F;
    constexpr int CPL = P / L;  // stage-2 DFTs per lane
    constexpr bool MEL = (OK == 2);
    constexpr int TILE = MEL ? G::MEL_TILE : G::PASS_FRAMES;
    constexpr int PASSES = MEL ? G::MEL_PASSES : 1;
    constexpr int TB = G::TB, TA = G::TA;
    constexpr int LCH = P < 8 ? P : 8;  // fast-path load chunk (registers pinned per chunk)

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtab = lds;                    // [2*NC] window zero-padded to n_fft
    float* work = lds + G::WIN_FLOATS;    // exchange regions / |X| rows

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int slot = lane / L;
    const int j = lane % L;  // n2 in stage 1, j in stage 2
    const int lane_base = slot * L;
    const int partner = lane_base + ((L - j) % L);

    // window -> LDS once per block
    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) wtab[i] = a.wpad[i];

    // per-lane twiddle bases (loop invariant): W_NC^{j*b}, W_NC^{j*TB*aa}; untangle
    // bases (sin, cos)(pi*(j + c*L)/NC) straight from the reference table (k < P).
    float2 twb[TB], twa[TA];
#pragma unroll
    for (int b = 0; b < TB; ++b) twb[b] = a.tw1[(j * b) % NC];
#pragma unroll
    for (int aa = 0; aa < TA; ++aa) twa[aa] = a.tw1[(j * TB * aa) % NC];
    float2 ub[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) ub[c] = a.sincos[j + c * L];
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t n_tiles = (total + TILE - 1) / TILE;
    const uint64_t t_begin = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t t_end = t_begin + tiles_per_block < n_tiles ? t_begin + tiles_per_block : n_tiles;

    const int half_win = a.win / 2;
    const int C = a.channels;
    const bool fold = a.fold != 0;
    const bool full_win = (a.pad_left == 0 && a.win == 2 * NC);
    int hint = -1;

    for (uint64_t tile = t_begin; tile < t_end; ++tile) {
        for (int pass = 0; pass < PASSES; ++pass) {
            const int f_in_tile = pass * G::PASS_FRAMES + wave * FPW + slot;
            const uint64_t g = tile * TILE + (uint64_t)f_in_tile;
            const bool valid = g < total;
            float* region = MEL ? work + f_in_tile * G::ROW : work + (wave * FPW + slot) * G::RS;

            // ---------------- load + window (lib.rs:367-386, uniform reflect rule) -------
            float2 v[P];
            if (valid) {
                hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
                const uint64_t t = g - a.trk_frame0[hint];
                const int64_t n = (int64_t)a.trk_len[hint];
                const uint64_t base = a.trk_in_off[hint];
                const int64_t start = (int64_t)t * a.hop - half_win - a.pad_left;
                const bool interior = full_win && start >= 0 && start + 2 * NC <= n;
                if (interior && INF == IN_F32 && C == 1 && !fold && ((base + start) & 1) == 0) {
                    const float2* src = reinterpret_cast<const float2*>(
                        static_cast<const float*>(a.in) + base + start) + j;
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
                } else if (interior && INF == IN_F32 && C == 2 && fold && ((base + 2 * start) & 3) == 0) {
                    const float4* src = reinterpret_cast<const float4*>(
                        static_cast<const float*>(a.in) + base + 2 * start) + j;
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
                } else {
                    // edge / unaligned / generic-format frames: a runtime loop writes the
                    // windowed samples of this lane into its frame's LDS region (even then
                    // odd positions), then static reads fill the registers.
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
            } else {
#pragma unroll
                for (int n1 = 0; n1 < P; ++n1) v[n1] = make_float2(0.f, 0.f);
            }

            // ---------------- stage 1: P-point DFT over n1, twiddle W_NC^{n2 k1} --------
            pin(v);
            dif_fft<P, 1, 0, P>(v);
            pin(v);

            // ---------------- LDS transpose (re then im through one region) -------------
            float2 w2r[P];
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

            // ---------------- stage 2: L-point DFTs over n2 ---------------------------
            pin(w2r);
            static_for<0, CPL>([&](auto cc) {
                constexpr int c = decltype(cc)::value;
                dif_fft<L, 1, c * L, P>(w2r);
            });

            pin(w2r);
            // ---------------- realfft untangle + epilogue -----------------------------
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
                    if constexpr (OK == 0) {
                        if (valid) reinterpret_cast<float2*>(a.out)[g * F + k] = make_float2(xr, xi);
                    } else if constexpr (OK == 1) {
                        float val;
                        const int kind = a.out_kind;
                        if (kind == OUT_POWER || kind == OUT_POWER_DB) {
                            val = xr * xr + xi * xi;
                            if (kind == OUT_POWER_DB) val = db_of(val, a.log_amin, 1e-36f, 10.0f);
                        } else {
                            val = __builtin_sqrtf(xr * xr + xi * xi);
                            if (kind == OUT_AMP_DB) val = db_of(val, a.log_amin, 1e-18f, 20.0f);
                        }
                        if (valid) static_cast<float*>(a.out)[g * F + k] = val;
                    } else {
                        region[k] = __builtin_sqrtf(xr * xr + xi * xi);
                    }
                    pin(w2r);
                });
            });
            if (j == 0) {  // Nyquist bin, realfft.rs:157
                const float2 z0 = w2r[0];
                const float xr = z0.x - z0.y;
                if constexpr (OK == 0) {
                    if (valid) reinterpret_cast<float2*>(a.out)[g * F + NC] = make_float2(xr, 0.0f);
                } else if constexpr (OK == 1) {
                    float val;
                    const int kind = a.out_kind;
                    if (kind == OUT_POWER || kind == OUT_POWER_DB) {
                        val = xr * xr + 0.0f * 0.0f;
                        if (kind == OUT_POWER_DB) val = db_of(val, a.log_amin, 1e-36f, 10.0f);
                    } else {
                        val = __builtin_sqrtf(xr * xr + 0.0f * 0.0f);
                        if (kind == OUT_AMP_DB) val = db_of(val, a.log_amin, 1e-18f, 20.0f);
                    }
                    if (valid) static_cast<float*>(a.out)[g * F + NC] = val;
                } else {
                    region[NC] = __builtin_sqrtf(xr * xr + 0.0f * 0.0f);
                }
            }
            if constexpr (MEL) {  // zero the row tail the mel bands may read past F
                for (int col = F + j; col < G::ROW; col += L) region[col] = 0.0f;
            }
        }

        if constexpr (MEL) {
            __syncthreads();
            // ---------------- mel projection: MFMA over each tile's bin band ------------
            constexpr int RB = TILE / 16;
            const int* jobs = a.wave_jobs + wave * a.max_jobs;
            for (int q = 0; q < a.max_jobs; ++q) {
                const int job = jobs[q];
                if (job < 0) break;
                const int mt = job / RB, rb = job % RB;
                const MelTile T = a.mel_tiles[mt];
                floatx4 acc = {0.f, 0.f, 0.f, 0.f};
                const float* xrow = work + (rb * 16 + (lane & 15)) * G::ROW + T.klo + (lane >> 4);
                const float4* wp = a.mel_w + T.w_off + lane;
                for (int kg = 0; kg < T.n_kg; ++kg) {
                    const float4 bw = wp[kg * 64];
                    const float* xk = xrow + kg * 16;
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xk[0], bw.x, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xk[4], bw.y, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xk[8], bw.z, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xk[12], bw.w, acc, 0, 0, 0);
                }
                const int mel = mt * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint64_t gf = tile * TILE + (uint64_t)(rb * 16 + 4 * (lane >> 4) + r);
                    if (gf < total && mel < a.n_mels) {
                        float val = acc[r];
                        if (a.out_kind == OUT_MEL_AMP_DB) val = db_of(val, a.log_amin, 1e-18f, 20.0f);
                        static_cast<float*>(a.out)[gf * (uint64_t)a.n_mels + mel] = val;
                    }
                }
            }
            __syncthreads();
        }
    }
}

#ifndef THESIA_NO_DISPATCH
// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
template <int NC, int OK>
static int lds_bytes_for() {
    using G = Geo<NC>;
    if (OK == 2) return (G::WIN_FLOATS + G::MEL_TILE * G::ROW) * 4;
    return (G::WIN_FLOATS + G::PASS_FRAMES * G::RS) * 4;
}

template <int NC, int OK>
static int tile_frames_for() {
    using G = Geo<NC>;
    return OK == 2 ? G::MEL_TILE : G::PASS_FRAMES;
}

static int ok_of(int out_kind) {
    if (out_kind == OUT_COMPLEX) return 0;
    if (out_kind == OUT_MEL || out_kind == OUT_MEL_AMP_DB) return 2;
    return 1;
}

template <int NC, int OK, int INF>
static int launch_t(const StftLaunch& a, hipStream_t stream) {
    const int lds = lds_bytes_for<NC, OK>();
    const int tile = tile_frames_for<NC, OK>();
    auto kern = stft_kernel<NC, OK, INF>;
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
            return -1;
        attr_set = true;
    }
    const uint64_t n_tiles = (a.total_frames + tile - 1) / tile;
    if (n_tiles == 0) return 0;
    int grid = a.grid;
    if (grid <= 0) {
        int dev = 0, cus = 256, per_cu = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, lds) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        grid = cus * per_cu;
    }
    if ((uint64_t)grid > n_tiles) grid = (int)n_tiles;
    const uint64_t tpb = (n_tiles + grid - 1) / grid;
    grid = (int)((n_tiles + tpb - 1) / tpb);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, stream, a, tpb);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int NC>
static int launch_nc(const StftLaunch& a, hipStream_t s) {
    const int ok = ok_of(a.out_kind);
    if (a.in_format == IN_S16) {
        if (ok == 0) return launch_t<NC, 0, IN_S16>(a, s);
        if (ok == 1) return launch_t<NC, 1, IN_S16>(a, s);
        return launch_t<NC, 2, IN_S16>(a, s);
    }
    if (ok == 0) return launch_t<NC, 0, IN_F32>(a, s);
    if (ok == 1) return launch_t<NC, 1, IN_F32>(a, s);
    return launch_t<NC, 2, IN_F32>(a, s);
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

template <int NC>
static void info_nc(int ok, int* lds, int* tile) {
    if (ok == 0) { *lds = lds_bytes_for<NC, 0>(); *tile = tile_frames_for<NC, 0>(); }
    else if (ok == 1) { *lds = lds_bytes_for<NC, 1>(); *tile = tile_frames_for<NC, 1>(); }
    else { *lds = lds_bytes_for<NC, 2>(); *tile = tile_frames_for<NC, 2>(); }
}

int stft_kernel_info(int n_fft, int out_kind, int in_format, int* lds_bytes, int* tile_frames,
                     int* blocks_per_cu) {
    (void)in_format;
    const int ok = ok_of(out_kind);
    int lds = 0, tile = 0;
    switch (n_fft / 2) {
        case 1: info_nc<1>(ok, &lds, &tile); break;
        case 2: info_nc<2>(ok, &lds, &tile); break;
        case 4: info_nc<4>(ok, &lds, &tile); break;
        case 8: info_nc<8>(ok, &lds, &tile); break;
        case 16: info_nc<16>(ok, &lds, &tile); break;
        case 32: info_nc<32>(ok, &lds, &tile); break;
        case 64: info_nc<64>(ok, &lds, &tile); break;
        case 128: info_nc<128>(ok, &lds, &tile); break;
        case 256: info_nc<256>(ok, &lds, &tile); break;
        case 512: info_nc<512>(ok, &lds, &tile); break;
        case 1024: info_nc<1024>(ok, &lds, &tile); break;
        case 2048: info_nc<2048>(ok, &lds, &tile); break;
        default: return -2;
    }
    if (lds_bytes) *lds_bytes = lds;
    if (tile_frames) *tile_frames = tile;
    if (blocks_per_cu) *blocks_per_cu = lds > 0 ? (160 * 1024) / lds : 8;
    return 0;
}

int stft_mel_row_stride(int n_fft) {
    switch (n_fft / 2) {
        case 1: return Geo<1>::ROW;
        case 2: return Geo<2>::ROW;
        case 4: return Geo<4>::ROW;
        case 8: return Geo<8>::ROW;
        case 16: return Geo<16>::ROW;
        case 32: return Geo<32>::ROW;
        case 64: return Geo<64>::ROW;
        case 128: return Geo<128>::ROW;
        case 256: return Geo<256>::ROW;
        case 512: return Geo<512>::ROW;
        case 1024: return Geo<1024>::ROW;
        case 2048: return Geo<2048>::ROW;
        default: return 0;
    }
}

#endif  // THESIA_NO_DISPATCH

}  // namespace thesia
