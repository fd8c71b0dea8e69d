// stft2_core.hpp -- building blocks of the 4-waves/SIMD and streaming STFT kernels
// (stft2_kernels.hip, stft3_kernels.hip): geometry, in-place two-stage FFT with the b64
// transpose, paired realfft untangle, float4 mel projection. Design notes: stft2_kernels.hip.
#pragma once

#include "stft_common.hpp"

namespace thesia {

constexpr int round_up_mod64(int v, int r) {
    while (v % 64 != r) ++v;
    return v;
}

template <int NC>
struct Geo2 {
    static constexpr int L = geo_L(NC);
    static constexpr int P = NC / L;
    static constexpr int CPL = P / L;
    static constexpr int FPW = 64 / L;
    static constexpr int F = NC + 1;
    static constexpr int F4 = (F + 3) / 4 * 4;
    static constexpr int S = L + 2;  // transpose row stride
    static constexpr int XREG = P * S;
    // frames of one 32-lane group sit 2L floats apart mod 64: their b64 reads interleave
    static constexpr int RS = round_up_mod64(XREG, L >= 32 ? 0 : (2 * L) % 64);
    static constexpr int PASS_FRAMES = kWaves * FPW;
    static constexpr int WIN_FLOATS = 2 * NC;
    static constexpr int TB = Geo<NC>::TB, TA = Geo<NC>::TA;
    static constexpr int LDS_BYTES = (WIN_FLOATS + PASS_FRAMES * RS) * 4;
    static_assert(P % L == 0 && L >= 8, "stft2 geometry");
    static_assert(XREG >= F4 && XREG >= NC, "the |X| row and the load staging must fit a region");
    static_assert(RS % 4 == 0, "16-byte aligned regions");
    static_assert(2 * LDS_BYTES <= 163840, "two blocks per CU");
};

// One point's worth of input per lane (2 samples x C interleaved channels) and its downmix:
// f32 as is, s16 as value / 2^15 (audio.rs:16-19, exact), channels summed (lib.rs:42).
template <int C, int INF>
struct Chunk;
template <>
struct Chunk<1, IN_F32> {
    using T = float2;
    __device__ static float2 mix(T x) { return x; }
};
template <>
struct Chunk<2, IN_F32> {
    using T = float4;
    __device__ static float2 mix(T x) { return make_float2(x.x + x.y, x.z + x.w); }
};
template <>
struct Chunk<1, IN_S16> {
    using T = short2;
    __device__ static float2 mix(T x) { return make_float2((float)x.x / 32768.0f, (float)x.y / 32768.0f); }
};
template <>
struct Chunk<2, IN_S16> {
    using T = short4;
    __device__ static float2 mix(T x) {
        return make_float2((float)x.x / 32768.0f + (float)x.y / 32768.0f,
                           (float)x.z / 32768.0f + (float)x.w / 32768.0f);
    }
};

// Interior frames of f32 mono / stereo input straight from HBM (8 / 16 B per lane); the
// stereo sum is x[ch0] + x[ch1] (lib.rs:42; the fold's leading 0.0 + only differs for -0).
template <int NC, int INF>
__device__ __forceinline__ bool load_direct2(const StftLaunch& a, int j, int64_t start, int64_t n,
                                             uint64_t base, int C, bool fold, const float* wtab,
                                             float2 (&v)[Geo2<NC>::P]) {
    constexpr int L = Geo2<NC>::L, P = Geo2<NC>::P;
    if constexpr (INF != IN_F32) {
        return false;
    } else {
        if (!(a.pad_left == 0 && a.win == 2 * NC && start >= 0 && start + 2 * NC <= n)) return false;
        if (C == 1 && !fold && ((base + start) & 1) == 0) {
            const float2* src = reinterpret_cast<const float2*>(static_cast<const float*>(a.in) + base + start) + j;
            const float2* wp = reinterpret_cast<const float2*>(wtab) + j;
            static_for<0, P / 8>([&](auto gc) {  // 8 loads in flight per chunk (VGPR budget)
                constexpr int g8 = decltype(gc)::value;
                static_for<0, 8>([&](auto ic) {
                    constexpr int n1 = 8 * g8 + decltype(ic)::value;
                    const float2 x = src[L * n1];
                    const float2 w = wp[L * n1];
                    v[n1] = make_float2(x.x * w.x, x.y * w.y);
                });
                pin_range<8 * g8, 8 * g8 + 8>(v);
            });
            return true;
        }
        if (C == 2 && fold && ((base + 2 * start) & 3) == 0) {
            const float4* src = reinterpret_cast<const float4*>(static_cast<const float*>(a.in) + base + 2 * start) + j;
            const float2* wp = reinterpret_cast<const float2*>(wtab) + j;
            static_for<0, P / 8>([&](auto gc) {
                constexpr int g8 = decltype(gc)::value;
                static_for<0, 8>([&](auto ic) {
                    constexpr int n1 = 8 * g8 + decltype(ic)::value;
                    const float4 x = src[L * n1];
                    const float2 w = wp[L * n1];
                    v[n1] = make_float2((x.x + x.y) * w.x, (x.z + x.w) * w.y);
                });
                pin_range<8 * g8, 8 * g8 + 8>(v);
            });
            return true;
        }
        return false;
    }
}

// Stage-1 DFT_P + twiddles W_NC^{j k1}, LDS transpose (re then im), stage-2 DFT_L, in place.
// On return v[c*L + ce_pos(L, k2)] = Z[k1 + P*k2] / 2 with k1 = j + c*L.
// twf(k1c, x): applies the stage-1 twiddle W_NC^{j*k1} to x (k1c an integral_constant).
// WIDE: transpose rows of stride L + 4 floats read back as ds_read_b128 (4 LDS cycles per KiB,
// conflict-free for L = 32: the 16-lane groups of a b128 read start on 16 distinct 4-bank
// slots) instead of stride L + 2 read as float2 pairs, which the compiler merges into
// ds_read2_b64 (8 cycles per KiB; MI355X_MICROARCH.md LDS table). Regions must then hold
// P * (L + 4) floats and be 16-byte aligned.
template <int NC>
constexpr int fft2_stride(bool wide) { return Geo2<NC>::L + (wide ? 4 : 2); }

// TPRIO > 0: the twiddle reads and the LDS transpose run at wave priority TPRIO, the register
// DFT stages at 0 (stft3 priority phases).
template <int NC, class TwF, bool WIDE = false, int TPRIO = 0>
__device__ __forceinline__ void fft2(float2 (&v)[Geo2<NC>::P], float* region, int j, const TwF& twf,
                                     int jw = -1) {
    // jw: the transpose column this lane's stage-1 outputs go to (default j; stft3's viewer
    // geometries write the frame's column and read row j)
    if (jw < 0) jw = j;
    using G = Geo2<NC>;
    constexpr int L = G::L, P = G::P, S = fft2_stride<NC>(WIDE), CPL = G::CPL;
    pin(v);
    dif_fft<P, 1, 0, P>(v);
    pin(v);
    if constexpr (TPRIO > 0) __builtin_amdgcn_s_setprio(TPRIO);
    if constexpr (TwF::kPairs) {
        // two twiddles per ds_read_b128: all reads of the table issued before the products
        float4 tw[P / 2];
        static_for<0, P / 2>([&](auto qc) { tw[decltype(qc)::value] = twf.pair(decltype(qc)::value); });
        static_for<1, P>([&](auto kc) {
            constexpr int k1 = decltype(kc)::value;
            constexpr int pk = ce_pos(P, k1);
            const float4 t = tw[k1 / 2];
            v[pk] = cmul(v[pk], (k1 & 1) ? make_float2(t.z, t.w) : make_float2(t.x, t.y));
        });
    } else {
        static_for<1, P>([&](auto kc) {
            constexpr int pk = ce_pos(P, decltype(kc)::value);
            v[pk] = twf(kc, v[pk]);
        });
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        wave_lds_sync();
        static_for<0, P>([&](auto kc) {
            constexpr int k1 = decltype(kc)::value;
            constexpr int pk = ce_pos(P, k1);
            region[k1 * S + jw] = e == 0 ? v[pk].x : v[pk].y;
        });
        wave_lds_sync();
        static_for<0, CPL>([&](auto cc) {
            constexpr int c = decltype(cc)::value;
            if constexpr (WIDE) {
                const float4* row = static_cast<const float4*>(
                    __builtin_assume_aligned(region + (j + c * L) * S, 16));
                static_for<0, L / 4>([&](auto qc) {
                    constexpr int q = 4 * decltype(qc)::value;
                    const float4 t = row[q / 4];
                    if (e == 0) {
                        v[c * L + q].x = t.x; v[c * L + q + 1].x = t.y;
                        v[c * L + q + 2].x = t.z; v[c * L + q + 3].x = t.w;
                    } else {
                        v[c * L + q].y = t.x; v[c * L + q + 1].y = t.y;
                        v[c * L + q + 2].y = t.z; v[c * L + q + 3].y = t.w;
                    }
                });
            } else {
                const float2* row = reinterpret_cast<const float2*>(region + (j + c * L) * S);
                static_for<0, L / 2>([&](auto qc) {
                    constexpr int q = 2 * decltype(qc)::value;
                    const float2 t = row[q / 2];
                    if (e == 0) { v[c * L + q].x = t.x; v[c * L + q + 1].x = t.y; }
                    else        { v[c * L + q].y = t.x; v[c * L + q + 1].y = t.y; }
                });
            }
        });
    }
    wave_lds_sync();
    pin(v);
    if constexpr (TPRIO > 0) __builtin_amdgcn_s_setprio(0);
    static_for<0, CPL>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        dif_fft<L, 1, c * L, P>(v);
    });
    pin(v);
}

// W_NC^{j*b}, W_NC^{j*TB*aa} from the lane-major table a.tw2 ([TB + TA][L]: one base and
// immediate offsets).
template <int NC>
__device__ __forceinline__ void load_tw2(const StftLaunch& a, int j, float2 (&twb)[Geo2<NC>::TB],
                                         float2 (&twa)[Geo2<NC>::TA]) {
    constexpr int L = Geo2<NC>::L, TB = Geo2<NC>::TB, TA = Geo2<NC>::TA;
    const float2* twp = a.tw2 + j;
#pragma unroll
    for (int b = 0; b < TB; ++b) twb[b] = twp[b * L];
#pragma unroll
    for (int aa = 0; aa < TA; ++aa) twa[aa] = twp[(TB + aa) * L];
}

// Stage-1 twiddles as two products W_NC^{j*b} * W_NC^{j*TB*aa} (k1 = TB*aa + b) from bases in
// registers.
template <int NC>
struct TwBases {
    static constexpr bool kPairs = false;
    float2 b[Geo2<NC>::TB], a[Geo2<NC>::TA];
    template <class K>
    __device__ __forceinline__ float2 operator()(K, float2 x) const {
        constexpr int TB = Geo2<NC>::TB;
        constexpr int k1 = K::value, bb = k1 % TB, aa = k1 / TB;
        if constexpr (bb != 0) x = cmul(x, b[bb]);
        if constexpr (aa != 0) x = cmul(x, a[aa]);
        return x;
    }
};

// Stage-1 twiddles as one product with W_NC^{j*k1} from a lane-major [P][L] table (LDS):
// conflict-free ds_read_b64 (consecutive lanes, consecutive entries).
struct TwTable {
    static constexpr bool kPairs = false;
    const float2* row;  // table + j
    int L;
    template <class K>
    __device__ __forceinline__ float2 operator()(K, float2 x) const {
        return cmul(x, row[K::value * L]);
    }
};
// The same table with k1 pairs interleaved: [P/2][L] float4 {W^{j*2q}, W^{j*(2q+1)}}
// (conflict-free ds_read_b128: consecutive lanes, consecutive 16-byte entries).
struct TwTable4 {
    static constexpr bool kPairs = true;
    const float4* row;  // table + j
    int L;
    __device__ __forceinline__ float4 pair(int q) const { return row[q * L]; }
};

// Calls epi(k, re, im, slot) when the epilogue takes the bin's compile-time slot (2i: bin
// k = j + c*L + P*t with i = c*(L/2) + t, 2i + 1: bin NC - k, 2*CPL*(L/2): lane 0's NC/2),
// else epi(k, re, im).
template <int S, class Epi>
__device__ __forceinline__ void call_epi(Epi& epi, int k, float re, float im) {
    if constexpr (std::is_invocable_v<Epi&, int, float, float, std::integral_constant<int, S>>)
        epi(k, re, im, std::integral_constant<int, S>{});
    else
        epi(k, re, im);
}

// realfft untangle on bin pairs; calls epi(k, re, im) for every bin this lane produces
// (k = j + c*L + P*t and NC - k for t < L/2; lane 0 also the self-paired bin NC/2).
template <int NC, bool BATCH = false, class Epi>
__device__ __forceinline__ void untangle2(const float2 (&v)[Geo2<NC>::P], int j, int partner,
                                          const float2 (&ub)[Geo2<NC>::CPL], Epi&& epi) {
    using G = Geo2<NC>;
    constexpr int L = G::L, P = G::P, CPL = G::CPL;
    const bool lane0 = j == 0;
    auto pair = [&](float2 b, float2 r, float s, float co, int k, auto slotc) {
        constexpr int slot = decltype(slotc)::value;
        constexpr bool both = slot < 2 * CPL * (L / 2);
        const float ar = b.x + r.x, ai = b.y - r.y;  // A = Z_k + conj Z_{NC-k}
        const float br = b.x - r.x, bi = b.y + r.y;  // B = Z_k - conj Z_{NC-k}
        const float p = __builtin_fmaf(co, br, s * bi);     // (p, q) = (co - i s) B
        const float q = __builtin_fmaf(co, bi, -(s * br));
        call_epi<slot>(epi, k, ar + q, ai - p);
        if constexpr (both) call_epi<slot + 1>(epi, NC - k, ar - q, -ai - p);
    };
    // BATCH: every partner value is requested before the first pair is formed (one LDS
    // latency per frame instead of one per pair; costs CPL*L registers)
    float2 recv[BATCH ? CPL * (L / 2) : 1];
    if constexpr (BATCH) {
        static_for<0, CPL>([&](auto cc) {
            constexpr int c = decltype(cc)::value;
            static_for<0, L / 2>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                constexpr int ps = (CPL - 1 - c) * L + ce_pos(L, L - 1 - t);
                recv[c * (L / 2) + t].x = __shfl(v[ps].x, partner, 64);
                recv[c * (L / 2) + t].y = __shfl(v[ps].y, partner, 64);
            });
        });
        // keep the batch a batch: without this the scheduler sinks each ds_bpermute next to
        // its use and the untangle becomes CPL*L/4 dependent LDS round trips
        pin(recv);
    }
    static_for<0, CPL>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        static_for<0, L / 2>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            constexpr int pb = c * L + ce_pos(L, t);
            constexpr int ps = (CPL - 1 - c) * L + ce_pos(L, L - 1 - t);
            const float2 b = v[pb];
            float2 r;
            if constexpr (BATCH) {
                r = recv[c * (L / 2) + t];
            } else {
                const float2 send = v[ps];
                r.x = __shfl(send.x, partner, 64);
                r.y = __shfl(send.y, partner, 64);
            }
            // lane 0 pairs inside its own registers: Z[(CPL-c) % CPL][c ? L-1-t : (L-t) % L]
            constexpr int c0 = (CPL - c) % CPL;
            constexpr int k20 = c == 0 ? (L - t) % L : L - 1 - t;
            constexpr int po = c0 * L + ce_pos(L, k20);
            const float2 own = v[po];
            r.x = lane0 ? own.x : r.x;
            r.y = lane0 ? own.y : r.y;
            // (sin, cos)(pi k / NC) = base(j + cL) rotated by pi t / L
            float s, co;
            if constexpr (t == 0) {
                s = ub[c].x;
                co = ub[c].y;
            } else {
                constexpr float cb = ce_tw_re(t, 2 * L);
                constexpr float sb = -ce_tw_im(t, 2 * L);
                s = __builtin_fmaf(ub[c].x, cb, ub[c].y * sb);
                co = __builtin_fmaf(ub[c].y, cb, -(ub[c].x * sb));
            }
            pair(b, r, s, co, j + c * L + P * t, std::integral_constant<int, 2 * (c * (L / 2) + t)>{});
        });
    });
    if (lane0) {  // k = NC/2 pairs with itself: (sin, cos)(pi/2) from the base sin_cos[0]
        constexpr int ph = ce_pos(L, L / 2);
        const float2 b = v[ph];
        constexpr float cb = ce_tw_re(L / 2, 2 * L);
        constexpr float sb = -ce_tw_im(L / 2, 2 * L);
        const float s = __builtin_fmaf(ub[0].x, cb, ub[0].y * sb);
        const float co = __builtin_fmaf(ub[0].y, cb, -(ub[0].x * sb));
        pair(b, b, s, co, NC / 2, std::integral_constant<int, 2 * CPL * (L / 2)>{});
    }
}

// lib.rs:131-132 on the |X| row in `region`: round r gives lane j mel r*L + j.
// wt / rounds / k0: the float4 weight rows, the per-round {row, steps} and the per-lane start
// bins (a.mel4_* in HBM, or their copies in LDS).
template <int NC, int U = 4, int NACC = 1>
__device__ __forceinline__ void mel4(const StftLaunch& a, const float* region, const float4* wt,
                                     const int2* rounds, const int* k0, int j, uint64_t g,
                                     bool valid) {
    constexpr int L = Geo2<NC>::L;
    constexpr int PR = 4;  // rounds whose {row, steps} and start bins are fetched up front
    const int n_mels = a.n_mels;
    const int R = a.mel4_rounds;
    const bool db = a.out_kind == OUT_MEL_AMP_DB;
    float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
    auto round = [&](int2 rd, int k0m) {
        // {first float4 row, float4 steps} are wave-uniform: scalar loop control
        rd.x = __builtin_amdgcn_readfirstlane(rd.x);
        rd.y = __builtin_amdgcn_readfirstlane(rd.y);
        const float4* xp = reinterpret_cast<const float4*>(region + (k0m & 0xFFFF));
        const float4* wp = wt + (size_t)rd.x * L + j;
        // NACC = 4: one accumulator per float4 component (four independent fma chains, summed
        // (a0 + a1) + (a2 + a3) at the end) instead of one k-ascending chain: a quarter of the
        // dependent-fma latency; reassociation within fp32 rounding (tolerance parity)
        float acc = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
        int it = 0;
        // every LDS read of a batch is issued before its fma chain: one LDS round trip per
        // batch (the host pads each round to a multiple of 4 steps with zero weights, so a
        // round is U-batches plus at most one 4-batch; the 1-step loop is a safety net)
        auto batch = [&](auto uc) {
            constexpr int B = decltype(uc)::value;
            float4 w[B], x[B];
#pragma unroll
            for (int u = 0; u < B; ++u) w[u] = wp[(it + u) * L];
#pragma unroll
            for (int u = 0; u < B; ++u) x[u] = xp[it + u];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                if constexpr (NACC == 4) {
                    acc = __builtin_fmaf(x[u].x, w[u].x, acc);
                    a1 = __builtin_fmaf(x[u].y, w[u].y, a1);
                    a2 = __builtin_fmaf(x[u].z, w[u].z, a2);
                    a3 = __builtin_fmaf(x[u].w, w[u].w, a3);
                } else {
                    acc = __builtin_fmaf(x[u].x, w[u].x, acc);
                    acc = __builtin_fmaf(x[u].y, w[u].y, acc);
                    acc = __builtin_fmaf(x[u].z, w[u].z, acc);
                    acc = __builtin_fmaf(x[u].w, w[u].w, acc);
                }
            }
            it += B;
        };
        while (it + U <= rd.y) batch(std::integral_constant<int, U>{});
        if constexpr (U > 4) {
            if (it + 4 <= rd.y) batch(std::integral_constant<int, 4>{});
        }
        for (; it < rd.y; ++it) {
            const float4 w = wp[it * L], x = xp[it];
            acc = __builtin_fmaf(x.x, w.x, acc);
            acc = __builtin_fmaf(x.y, w.y, acc);
            acc = __builtin_fmaf(x.z, w.z, acc);
            acc = __builtin_fmaf(x.w, w.w, acc);
        }
        if constexpr (NACC == 4) acc = (acc + a1) + (a2 + a3);
        const int m = (int)((unsigned)k0m >> 16);  // start bin | mel << 16 (build_mel4)
        if (valid && m < n_mels) st_out(out + m, db ? db_of(acc, a.log_amin, 1e-18f, 20.0f) : acc);
    };
    // the first PR rounds' setup in one LDS round trip (not one dependent read per round)
    int2 rdp[PR];
    int k0p[PR];
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        rdp[r] = r < R ? rounds[r] : int2{0, 0};
        k0p[r] = r < R ? k0[r * L + j] : 0;
    }
#pragma unroll
    for (int r = 0; r < PR; ++r)
        if (r < R) round(rdp[r], k0p[r]);
    for (int r = PR; r < R; ++r) round(rounds[r], k0[r * L + j]);
}

// mel4 as a software pipeline (a.mel_chunks = CMAX = 4 or 8: the rounds as a stream of 4-step chunks,
// engine.cpp build_mel4): the 8 LDS reads of chunk c + 1 are issued before the fma chain of
// chunk c, so a chunk's LDS latency hides under the previous chunk's chain instead of stalling
// the wave once per batch (stamps: the mel phase spent 2/3 of its cycles waiting). Chunk c reads
// weight rows 4c..4c+3 (immediate offsets) and the |X| floats at xo[c] & 0xFFFF; the per-lane
// chunk words come from one LDS round trip up front. Same k-ascending chain per mel as mel4
// (bit-exact with it).
template <int NC, int CMAX>
__device__ __forceinline__ void mel4p(const StftLaunch& a, const float* region, const float4* wt,
                                      const int* xo_tab, int j, uint64_t g, bool valid) {
    constexpr int L = Geo2<NC>::L;
    const int n_mels = a.n_mels;
    const bool db = a.out_kind == OUT_MEL_AMP_DB;
    float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
    // a.mel_chunks == CMAX (the host pads the stream to 4 or 8 chunks)
    int xo[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) xo[c] = xo_tab[c * L + j];
    const float4* wp = wt + j;
    auto load = [&](auto cc, float4 (&w)[4], float4 (&x)[4]) {
        constexpr int c = decltype(cc)::value;
        const float4* xp = reinterpret_cast<const float4*>(region + (xo[c] & 0xFFFF));
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = wp[(4 * c + u) * L];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = xp[u];
    };
    float acc = 0.0f;
    auto chain = [&](auto cc, const float4 (&w)[4], const float4 (&x)[4]) {
        constexpr int c = decltype(cc)::value;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc = __builtin_fmaf(x[u].x, w[u].x, acc);
            acc = __builtin_fmaf(x[u].y, w[u].y, acc);
            acc = __builtin_fmaf(x[u].z, w[u].z, acc);
            acc = __builtin_fmaf(x[u].w, w[u].w, acc);
        }
        if (xo[c] < 0) {  // the round's last chunk: this lane's mel is done
            const int m = (xo[c] >> 16) & 0x7FFF;
            if (valid && m < n_mels) st_out(out + m, db ? db_of(acc, a.log_amin, 1e-18f, 20.0f) : acc);
            acc = 0.0f;
        }
    };
    float4 w0[4], x0[4], w1[4], x1[4];
    load(std::integral_constant<int, 0>{}, w0, x0);
    static_for<0, CMAX>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if constexpr (c + 1 < CMAX) {
            if constexpr ((c & 1) == 0) load(std::integral_constant<int, c + 1>{}, w1, x1);
            else load(std::integral_constant<int, c + 1>{}, w0, x0);
        }
        // keep the next chunk's reads ahead of this chunk's chain (the scheduler would sink
        // them next to their use and the pipeline would collapse)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr ((c & 1) == 0) chain(cc, w0, x0);
        else chain(cc, w1, x1);
    });
}

// previous mel4 (per-round dependent setup reads), kept for in-process A/B (stft3 VAR bit6)
template <int NC, int U = 4>
__device__ __forceinline__ void mel4_v1(const StftLaunch& a, const float* region, const float4* wt,
                                     const int2* rounds, const int* k0, int j, uint64_t g,
                                     bool valid) {
    constexpr int L = Geo2<NC>::L;
    const int n_mels = a.n_mels;
    const bool db = a.out_kind == OUT_MEL_AMP_DB;
    float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
    for (int r = 0; r < a.mel4_rounds; ++r) {
        const int2 rd = rounds[r];  // {first float4 row, float4 steps}: wave-uniform
        const int k0m = k0[r * L + j];  // start bin | mel index << 16 (engine.cpp build_mel4)
        const float4* xp = reinterpret_cast<const float4*>(region + (k0m & 0xFFFF));
        const float4* wp = wt + (size_t)rd.x * L + j;
        float acc = 0.0f;
        int it = 0;
        // every LDS read of a batch is issued before its fma chain: one LDS round trip per
        // batch (the host pads each round to a multiple of 4 steps with zero weights, so a
        // round is U-batches plus at most one 4-batch; the 1-step loop is a safety net)
        auto batch = [&](auto uc) {
            constexpr int B = decltype(uc)::value;
            float4 w[B], x[B];
#pragma unroll
            for (int u = 0; u < B; ++u) w[u] = wp[(it + u) * L];
#pragma unroll
            for (int u = 0; u < B; ++u) x[u] = xp[it + u];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                acc = __builtin_fmaf(x[u].x, w[u].x, acc);
                acc = __builtin_fmaf(x[u].y, w[u].y, acc);
                acc = __builtin_fmaf(x[u].z, w[u].z, acc);
                acc = __builtin_fmaf(x[u].w, w[u].w, acc);
            }
            it += B;
        };
        while (it + U <= rd.y) batch(std::integral_constant<int, U>{});
        if constexpr (U > 4) {
            if (it + 4 <= rd.y) batch(std::integral_constant<int, 4>{});
        }
        for (; it < rd.y; ++it) {
            const float4 w = wp[it * L], x = xp[it];
            acc = __builtin_fmaf(x.x, w.x, acc);
            acc = __builtin_fmaf(x.y, w.y, acc);
            acc = __builtin_fmaf(x.z, w.z, acc);
            acc = __builtin_fmaf(x.w, w.w, acc);
        }
        const int m = (int)((unsigned)k0m >> 16);
        if (valid && m < n_mels) st_out(out + m, db ? db_of(acc, a.log_amin, 1e-18f, 20.0f) : acc);
    }
}

}  // namespace thesia
