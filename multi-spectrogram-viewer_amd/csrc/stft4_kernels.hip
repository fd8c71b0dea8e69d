// stft4_kernels.hip -- the streaming STFT kernel with ONE frame stream per wave, for the
// headline geometry n_fft = 2048 (NC = 1024 complex points), win = n_fft, hop = n_fft/4.
//
// Same contract and the same streaming idea as stft3_kernel (each wave walks consecutive
// frames; the downmixed samples stay in a register ring that shifts by a hop; only the hop of
// new samples is loaded, one frame ahead), but a frame spans all 64 lanes instead of 32:
// lane l holds the points m = l + 64 q, q < 16 (samples 2m, 2m+1 from the frame start). That
// halves the registers per lane (ring 32, frame 32, prefetch <= 16 VGPRs) and the LDS per
// frame stream, so four waves fit on a SIMD (128 VGPRs, two 8-wave blocks per CU) instead of
// two: twice the waves to hide the LDS round trips and the HBM prefetch behind.
//
// FFT: NC = 1024 = 16 x 64 with the 64 split as 16 x 4.
//   stage A  Y[l][k1] = sum_q z[l + 64q] W16^{q k1} in registers, times W1024^{l k1} (LDS table)
//   transpose (re, then im) through the wave's LDS region: lane (la, k1) = la + 4 k1 receives
//            Y[la + 4 lb][k1], lb < 16 (row k1, sub-row la: four conflict-free ds_read_b128)
//   stage B  U[kb] = sum_lb Y W16^{lb kb} in registers, times W64^{la kb}
//   stage C  DFT-4 over la ACROSS the lane quad with DPP (quad_perm) butterflies:
//            lane la ends with ka = bitrev2(la), i.e. Z[k1 + 16 kb + 256 ka] in register kb.
// The realfft untangle then pairs bin k with NC - k: for k1 != 0 that is lane
// (3 - la) + 4 (16 - k1), register 15 - kb; the k1 = 0 quad pairs inside itself (register
// 16 - kb of lane 3 - la; kb = 0 and kb = 8 are special, see untangle4).
//
// Mel (lib.rs:131): each lane runs up to two whole filters per round (LPT-paired so every
// lane's step count is about equal); the switch from the first to the second is a per-lane
// select, the chain per filter is the same k-ascending fma chain as stft3 (bit-exact for
// equal |X|).
#include "stft2_core.hpp"

#include <cstdlib>
#include <type_traits>

namespace thesia {

struct Geo4 {
    static constexpr int NC = 1024, P = 16, SH = 4, F = NC + 1, F4 = 1028;
    static constexpr int WAVES = 8, BLOCK = 64 * WAVES;
    static constexpr int TS = 68;                   // transpose row: 4 sub-rows of 16 + 4 pad
    static constexpr int RS = 16 * TS;              // 1088 floats per wave (>= XROW, >= NC)
    // The |X| row in LDS is skewed: bin k at k + 8 (k >> 8) (8 unused floats after every 256
    // bins), so the bins k + 256 ka that the four lanes of a quad write at once fall on distinct
    // banks (unskewed they are a 4-way conflict on every ds_write_b32). XROW = skew(F4 - 1) + 1.
    static constexpr int XROW = 1060;
    static constexpr int WL_STRIDE = 2 * P + 4;     // window row per lane (float4 reads)
    static constexpr int WL_FLOATS = 64 * WL_STRIDE;
    static constexpr int TWA_FLOATS = 2 * P * 64;   // [k1][lane] W1024^{lane k1}
    static constexpr int TWB_STRIDE = 17;           // [la][kb] W64^{la kb}, padded row
    static constexpr int TWB_FLOATS = 2 * 4 * TWB_STRIDE;
    static constexpr int TAB_FLOATS = WL_FLOATS + TWA_FLOATS + TWB_FLOATS;
    static constexpr int BASE_FLOATS = TAB_FLOATS + WAVES * RS;
    static_assert(TAB_FLOATS % 4 == 0 && RS % 4 == 0, "16-byte aligned regions");
    static_assert(RS >= XROW && RS >= NC, "the |X| row and the load staging fit a region");
};

__host__ __device__ constexpr int skew4(int k) { return k + ((k >> 8) << 3); }
static_assert(skew4(Geo4::F4 - 1) + 1 == Geo4::XROW, "skewed row length");

// DPP quad permutations (dpp_ctrl quad_perm encodings)
constexpr int kQuadSwap2 = 0x4E;  // [2,3,0,1]
constexpr int kQuadSwap1 = 0xB1;  // [1,0,3,2]
constexpr int kQuadRev = 0x1B;    // [3,2,1,0]

template <int CTRL>
__device__ __forceinline__ float quad_dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL,
                                                              0xF, 0xF, false));
}

// Reflect-padded, downmixed samples of a frame (the uniform rule of load_frame_generic,
// stft_common.hpp, for win = n_fft); staged through LDS because the loop is a runtime one.
template <int INF>
__device__ __forceinline__ void load_raw_generic4(const StftLaunch& a, float* region, int lane,
                                                  int64_t start, int64_t n, uint64_t base, int C,
                                                  bool fold, float2 (&raw)[Geo4::P]) {
    constexpr int P = Geo4::P;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        wave_lds_sync();
        for (int q = 0; q < P; ++q) {
            const int m = 64 * q + lane;
            int64_t i = start + 2 * m + e;
            if (i < 0) i = -i;
            if (i > n - 1) i = 2 * (n - 1) - i;
            i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
            region[m] = read_sample<INF>(a.in, base, i, C, fold);
        }
        wave_lds_sync();
        static_for<0, P>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const float r = region[64 * q + lane];
            if (e == 0) raw[q].x = r; else raw[q].y = r;
        });
    }
}

// The frame's FFT in place (stages A, B, C of the header). On return
// v[ce_pos(16, kb)] = Z[k1 + 16 kb + 256 bitrev2(la)] / 2 for lane = la + 4 k1.
__device__ __forceinline__ void fft4(float2 (&v)[Geo4::P], float* region, int lane, int la, int kq,
                                     const float2* twa, const float2* twb, float sg1, float sg2,
                                     bool rot3) {
    constexpr int P = Geo4::P, TS = Geo4::TS;
    pin(v);
    dif_fft<P, 1, 0, P>(v);
    pin(v);
    // table offsets made opaque here: the twiddle reads cannot be hoisted above the DFT (they
    // would hold 30 VGPRs across it)
    int ta = lane;
    asm volatile("" : "+v"(ta));
    static_for<1, P>([&](auto kc) {
        constexpr int k1 = decltype(kc)::value;
        constexpr int pk = ce_pos(P, k1);
        v[pk] = cmul(v[pk], twa[k1 * 64 + ta]);
    });
    const int wofs = (lane & 3) * 16 + (lane >> 2);  // writer l = la_w + 4 lb_w -> [k1][la_w][lb_w]
    const float4* rrow = reinterpret_cast<const float4*>(region + kq * TS + la * 16);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        wave_lds_sync();
        static_for<0, P>([&](auto kc) {
            constexpr int k1 = decltype(kc)::value;
            constexpr int pk = ce_pos(P, k1);
            region[k1 * TS + wofs] = e == 0 ? v[pk].x : v[pk].y;
        });
        wave_lds_sync();
        static_for<0, 4>([&](auto cc) {
            constexpr int c = decltype(cc)::value;
            const float4 t = rrow[c];
            if (e == 0) {
                v[4 * c].x = t.x; v[4 * c + 1].x = t.y; v[4 * c + 2].x = t.z; v[4 * c + 3].x = t.w;
            } else {
                v[4 * c].y = t.x; v[4 * c + 1].y = t.y; v[4 * c + 2].y = t.z; v[4 * c + 3].y = t.w;
            }
        });
    }
    wave_lds_sync();
    pin(v);
    dif_fft<P, 1, 0, P>(v);
    pin(v);
    int tb = la * Geo4::TWB_STRIDE;
    asm volatile("" : "+v"(tb));
    static_for<1, P>([&](auto kc) {
        constexpr int kb = decltype(kc)::value;
        constexpr int pk = ce_pos(P, kb);
        v[pk] = cmul(v[pk], twb[tb + kb]);
    });
    // DFT-4 over the quad (DIF, radix 2 x 2): distance 2 (lanes la < 2 add, la >= 2 take the
    // difference, lane 3 of the quad then times -i), distance 1 (even add, odd difference).
    // fmaf(+-1, a, b) is exactly b +- a.
    // (groups of four registers between pins bound the temporaries)
    static_for<0, P / 4>([&](auto gc) {
        constexpr int g4 = 4 * decltype(gc)::value;
        static_for<g4, g4 + 4>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const float bx = quad_dpp<kQuadSwap2>(v[i].x), by = quad_dpp<kQuadSwap2>(v[i].y);
            const float rx = __builtin_fmaf(sg1, v[i].x, bx), ry = __builtin_fmaf(sg1, v[i].y, by);
            const float tx = rot3 ? ry : rx, ty = rot3 ? -rx : ry;
            const float cx = quad_dpp<kQuadSwap1>(tx), cy = quad_dpp<kQuadSwap1>(ty);
            v[i] = make_float2(__builtin_fmaf(sg2, tx, cx), __builtin_fmaf(sg2, ty, cy));
        });
        pin_range<g4, g4 + 4>(v);
    });
    pin(v);
}

// realfft untangle (realfft.rs:140-157) on the stage-C layout; calls epi(k, skew4(k), re, im)
// once for every bin 0..NC. Lane (la, k1) forms the pairs of its registers kb < 8 (bins k and NC - k);
// in the k1 = 0 quad, kb = 0 holds the bins 0 (with NC), 512 (self-paired) and 256 / 768,
// and the kb = 8 pairs (128 / 896, 640 / 384) are formed by lanes 0 and 1.
template <bool BATCH, class Epi>
__device__ __forceinline__ void untangle4(const float2 (&v)[Geo4::P], int la, int kq, int pl0,
                                          int pl1, float2 ub, Epi&& epi) {
    constexpr int NC = Geo4::NC, P = Geo4::P;
    const int ka = ((la & 1) << 1) | (la >> 1);
    const int kbase = kq + 256 * ka;
    // skewed addresses: k = kbase + 16 t stays in block ka, NC - k in block 3 - ka (t, k1 not
    // both 0; that pair computes its own)
    const int sk1 = kbase + 8 * ka, sk2 = NC - kbase + 8 * (3 - ka);
    auto pair = [&](float2 b, float2 r, float s, float co, int k, int a1, int a2, bool first,
                    bool second) {
        const float ar = b.x + r.x, ai = b.y - r.y;  // A = Z_k + conj Z_{NC-k}
        const float br = b.x - r.x, bi = b.y + r.y;  // B = Z_k - conj Z_{NC-k}
        const float p = __builtin_fmaf(co, br, s * bi);  // (p, q) = (co - i s) B
        const float q = __builtin_fmaf(co, bi, -(s * br));
        if (first) epi(k, a1, ar + q, ai - p);
        if (second) epi(NC - k, a2, ar - q, -ai - p);
    };
    // (sin, cos)(pi (kbase + 16 t) / NC) = the base rotated by 2 pi t / 128
    auto rot = [&](auto tc, float& s, float& co) {
        constexpr int t = decltype(tc)::value;
        if constexpr (t == 0) {
            s = ub.x;
            co = ub.y;
        } else {
            constexpr float cb = ce_tw_re(t, 128);
            constexpr float sb = -ce_tw_im(t, 128);
            s = __builtin_fmaf(ub.x, cb, ub.y * sb);
            co = __builtin_fmaf(ub.y, cb, -(ub.x * sb));
        }
    };
    const bool q0 = kq == 0;
    auto fetch = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        constexpr int pn = ce_pos(P, P - 1 - t), ps = ce_pos(P, (P - t) % P);
        const float sx = q0 ? v[ps].x : v[pn].x, sy = q0 ? v[ps].y : v[pn].y;
        const int src = t == 0 ? pl0 : pl1;
        float2 r;
        r.x = __shfl(sx, src, 64);
        r.y = __shfl(sy, src, 64);
        return r;
    };
    // BATCH: every partner value requested before the first pair (16 more VGPRs)
    float2 recv[BATCH ? P / 2 : 1];
    if constexpr (BATCH) static_for<0, P / 2>([&](auto tc) { recv[decltype(tc)::value] = fetch(tc); });
    static_for<0, P / 2>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        float2 r;
        if constexpr (BATCH) r = recv[t]; else r = fetch(tc);
        constexpr int pb = ce_pos(P, t);  // (constexpr: a runtime ce_pos is a call + scratch)
        float s, co;
        rot(tc, s, co);
        if constexpr (t == 0) {
            const bool first = !(q0 && la == 3);           // 768 comes from lane 2
            const bool second = first && !(q0 && la == 1);  // 512 pairs with itself
            pair(v[pb], r, s, co, kbase, sk1, skew4(NC - kbase), first, second);
        } else {
            pair(v[pb], r, s, co, kbase + 16 * t, sk1 + 16 * t, sk2 - 16 * t, true, true);
        }
    });
    {
        constexpr int p8 = ce_pos(P, P / 2);
        float2 r;
        r.x = quad_dpp<kQuadRev>(v[p8].x);
        r.y = quad_dpp<kQuadRev>(v[p8].y);
        if (q0 && la < 2) {
            float s, co;
            rot(std::integral_constant<int, P / 2>{}, s, co);
            pair(v[p8], r, s, co, kbase + 16 * (P / 2), sk1 + 16 * (P / 2), sk2 - 16 * (P / 2), true,
                 true);
        }
    }
}

// lib.rs:131 on the (skewed) |X| row in `region`. Round u: lane runs sA steps of filter A from kA
// (float4 steps, row positions), then filter B for the rest of the round's S steps from kB; weights
// wt[(row + s) * 64 + lane] (zero outside the filters and on the skew gaps). meta = {kA, kB - 4 sA, sA, mA | mB << 16}
// (0xffff = no filter).
template <int U>
__device__ __forceinline__ void mel5(const StftLaunch& a, const float* region, const float4* wt,
                                     const int4* meta, const int2* rounds, int lane, uint64_t g) {
    const int n_mels = a.n_mels;
    const bool db = a.out_kind == OUT_MEL_AMP_DB;
    float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
    for (int u = 0; u < a.mel5_rounds; ++u) {
        const int2 rd = rounds[u];
        const int4 mt = meta[u * 64 + lane];
        const float4* wp = wt + (size_t)rd.x * 64 + lane;
        const float4* xa = reinterpret_cast<const float4*>(region + mt.x);
        const float4* xb = reinterpret_cast<const float4*>(region + mt.y);
        float accA = 0.0f, acc = 0.0f;
        auto step = [&](int s, float4 x, float4 w) {
            const bool sw = s == mt.z;
            accA = sw ? acc : accA;
            acc = sw ? 0.0f : acc;
            acc = __builtin_fmaf(x.x, w.x, acc);
            acc = __builtin_fmaf(x.y, w.y, acc);
            acc = __builtin_fmaf(x.z, w.z, acc);
            acc = __builtin_fmaf(x.w, w.w, acc);
        };
        int s = 0;
        for (; s + U <= rd.y; s += U) {
            float4 w[U], x[U];
#pragma unroll
            for (int i = 0; i < U; ++i) w[i] = wp[(s + i) * 64];
#pragma unroll
            for (int i = 0; i < U; ++i) x[i] = (s + i < mt.z ? xa : xb)[s + i];
#pragma unroll
            for (int i = 0; i < U; ++i) step(s + i, x[i], w[i]);
        }
        for (; s < rd.y; ++s) step(s, (s < mt.z ? xa : xb)[s], wp[s * 64]);
        const unsigned mA = (unsigned)mt.w & 0xffffu, mB = (unsigned)mt.w >> 16;
        if (mA != 0xffffu) out[mA] = db ? db_of(accA, a.log_amin, 1e-18f, 20.0f) : accA;
        if (mB != 0xffffu) out[mB] = db ? db_of(acc, a.log_amin, 1e-18f, 20.0f) : acc;
    }
}

// OK: 0 complex, 1 linear kinds, 2 mel kinds. C: 1 mono, 2 stereo (interleaved); INF: f32 / s16.
// VAR (experiments, THESIA_STFT_VARIANT): bit0 = per-pair partner exchange instead of the
// batched one; bit1 / bit2 = next-frame prefetch issued after the FFT / after the untangle
// instead of before the FFT; ablations (outputs wrong, timing only): bit3 = no mel, bit4 = no
// FFT, bit5 = no untangle / |X| / mel; bit6 = LDS padded to one block (2 waves/SIMD) per CU.
template <int OK, int C, int INF, int VAR = 0>
__global__ void __launch_bounds__(Geo4::BLOCK, 4)
stft4_kernel(StftLaunch a, uint64_t fps) {
    using G = Geo4;
    using CK = Chunk<C, INF>;
    using CT = typename CK::T;
    using ET = typename std::conditional<INF == IN_S16, int16_t, float>::type;
    constexpr int NC = G::NC, P = G::P, SH = G::SH, F = G::F;

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtl = lds;
    float2* twa = reinterpret_cast<float2*>(lds + G::WL_FLOATS);
    float2* twb = reinterpret_cast<float2*>(lds + G::WL_FLOATS + G::TWA_FLOATS);
    float* work = lds + G::TAB_FLOATS;
    float4* mel_w = reinterpret_cast<float4*>(lds + G::BASE_FLOATS);
    int4* mel_meta = reinterpret_cast<int4*>(mel_w + (OK == 2 ? a.mel5_rows * 64 : 0));
    int2* mel_rd = reinterpret_cast<int2*>(mel_meta + (OK == 2 ? a.mel5_rounds * 64 : 0));

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int la = lane & 3, kq = lane >> 2;
    const int ka = ((la & 1) << 1) | (la >> 1);

    for (int i = threadIdx.x; i < 2 * NC; i += G::BLOCK) {  // w/2 is exact (realfft's 1/2)
        const int m = i >> 1, l = m & 63, q = m >> 6;
        wtl[l * G::WL_STRIDE + 2 * q + (i & 1)] = a.wpad[i] * 0.5f;
    }
    for (int i = threadIdx.x; i < P * 64; i += G::BLOCK) twa[i] = a.tw4a[i];
    for (int i = threadIdx.x; i < 4 * G::TWB_STRIDE; i += G::BLOCK) twb[i] = a.tw4b[i];
    if constexpr (OK == 2) {
        for (int i = threadIdx.x; i < a.mel5_rows * 64; i += G::BLOCK) mel_w[i] = a.mel5_wt[i];
        for (int i = threadIdx.x; i < a.mel5_rounds * 64; i += G::BLOCK) mel_meta[i] = a.mel5_meta[i];
        for (int i = threadIdx.x; i < a.mel5_rounds; i += G::BLOCK) mel_rd[i] = a.mel5_round[i];
    }
    float2 ub = a.sincos[kq + 256 * ka];
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t stream = (uint64_t)blockIdx.x * G::WAVES + wave;
    const uint64_t g0 = stream * fps;
    const uint64_t g1 = g0 + fps < total ? g0 + fps : total;
    const int hop = a.hop;
    float* region = work + wave * G::RS;
    const ET* in = static_cast<const ET*>(a.in);
    // untangle partners: t > 0 and t == 0 (untangle4)
    const int pl1 = kq ? (3 - la) + 4 * (16 - kq) : 3 - la;
    const int pl0 = kq ? pl1 : (la < 2 ? la : 5 - la);
    const float sg1 = la < 2 ? 1.0f : -1.0f, sg2 = (la & 1) ? -1.0f : 1.0f;
    const bool rot3 = la == 3;

    float2 raw[P];
    CT pre[SH];
    bool pre_ok = false;
    int hint = -1;
    // the stream's current track (wave-uniform), looked up again only past its end
    uint64_t g_beg = 1, g_end = 0, base = 0;
    int64_t n = 0;
    for (uint64_t g = g0; g < g1; ++g) {
        asm volatile("" : "+v"(ub.x), "+v"(ub.y));
        int wl = lane;
        asm volatile("" : "+v"(wl));
        const float4* wrow = reinterpret_cast<const float4*>(wtl + wl * G::WL_STRIDE);
        if (g >= g_end || g < g_beg) {
            hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
            g_beg = a.trk_frame0[hint];
            g_end = a.trk_frame0[hint + 1];
            n = (int64_t)a.trk_len[hint];
            base = a.trk_in_off[hint];
        }
        const int64_t start = (int64_t)(g - g_beg) * hop - NC;  // half_win = NC, pad_left = 0
        if (pre_ok) {
#pragma unroll
            for (int q = 0; q < P - SH; ++q) raw[q] = raw[q + SH];
#pragma unroll
            for (int q = 0; q < SH; ++q) raw[P - SH + q] = CK::mix(pre[q]);
        } else if (start >= 0 && start + 2 * NC <= n && ((base + (uint64_t)start * C) % (2 * C)) == 0) {
            const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)start * C) + lane;
            static_for<0, P>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                raw[q] = CK::mix(src[64 * q]);
            });
        } else {
            load_raw_generic4<INF>(a, region, lane, start, n, base, C, a.fold != 0, raw);
        }
        // prefetch the next frame's new points P-SH .. P-1 (VAR bit1: after the FFT)
        auto prefetch = [&]() {
            const int64_t nstart = start + hop;
            const int64_t off = nstart + 2 * 64 * (P - SH);
            const bool nxt = g + 1 < g1 && g + 1 < g_end && nstart + 2 * NC <= n && off >= 0 &&
                             ((base + (uint64_t)off * C) % (2 * C)) == 0;
            if (nxt) {
                const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)off * C) + lane;
#pragma unroll
                for (int q = 0; q < SH; ++q) pre[q] = src[64 * q];
            }
            pre_ok = nxt;
        };
        // window (lib.rs:379, with the 1/2 of realfft.rs:148-154 folded in)
        float2 v[P];
        static_for<0, P / 2>([&](auto hc) {
            constexpr int h = decltype(hc)::value;
            const float4 w = wrow[h];
            v[2 * h] = make_float2(raw[2 * h].x * w.x, raw[2 * h].y * w.y);
            v[2 * h + 1] = make_float2(raw[2 * h + 1].x * w.z, raw[2 * h + 1].y * w.w);
        });
        if constexpr ((VAR & 6) == 0) prefetch();
        if constexpr ((VAR & 16) == 0) fft4(v, region, lane, la, kq, twa, twb, sg1, sg2, rot3);
        else pin(v);
        if constexpr ((VAR & 6) == 2) prefetch();
        if constexpr (OK == 2 && (VAR & 32) != 0) {  // ablation: no untangle / |X| / mel
            pin(v);
            if constexpr ((VAR & 4) != 0) prefetch();
        } else if constexpr (OK == 2) {
            untangle4<(VAR & 1) == 0>(v, la, kq, pl0, pl1, ub, [&](int, int ad, float xr, float xi) {
                region[ad] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xr, xr, xi * xi));  // |X| (lib.rs:124)
            });
            // zero the skew gaps (4 x 8 floats) and the row tail (bins F..F4-1): the filters give
            // them weight 0, and 0 * leftover could be NaN
            if (lane < 35) region[lane < 32 ? 256 + 264 * (lane >> 3) + (lane & 7) : skew4(F) + lane - 32] = 0.0f;
            if constexpr ((VAR & 4) != 0) prefetch();
            wave_lds_sync();
            if constexpr ((VAR & 8) == 0) mel5<4>(a, region, mel_w, mel_meta, mel_rd, lane, g);
        } else if constexpr (OK == 0) {
            float2* crow = reinterpret_cast<float2*>(a.out) + g * F;
            untangle4<(VAR & 1) == 0>(v, la, kq, pl0, pl1, ub, [&](int k, int, float xr, float xi) {
                crow[k] = make_float2(xr, xi);
            });
        } else {
            const int kind = a.out_kind;
            const bool power = kind == OUT_POWER || kind == OUT_POWER_DB;
            const bool db = kind == OUT_AMP_DB || kind == OUT_POWER_DB;
            untangle4<(VAR & 1) == 0>(v, la, kq, pl0, pl1, ub, [&](int, int ad, float xr, float xi) {
                const float p2 = __builtin_fmaf(xr, xr, xi * xi);
                region[ad] = power ? p2 : __builtin_amdgcn_sqrtf(p2);
            });
            wave_lds_sync();
            float* frow = static_cast<float*>(a.out) + g * F;
            for (int k = lane; k < F; k += 64) {
                float val = region[skew4(k)];
                if (db) val = power ? db_of(val, a.log_amin, 1e-36f, 10.0f)
                                    : db_of(val, a.log_amin, 1e-18f, 20.0f);
                frow[k] = val;
            }
        }
    }
}

// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
int stft4_lds_bytes(const StftLaunch& a, bool mel) {
    return (Geo4::BASE_FLOATS +
            (mel ? a.mel5_rows * 256 + a.mel5_rounds * 256 + 2 * a.mel5_rounds : 0)) * 4;
}

template <int OK, int C, int INF, int VAR = 0>
static int launch4_k(const StftLaunch& a, hipStream_t stream) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (VAR == 0 && OK == 2 && C == 2 && INF == IN_F32) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        switch (e ? atoi(e) : 0) {
            case 1: return launch4_k<OK, C, INF, 1>(a, stream);
            case 2: return launch4_k<OK, C, INF, 2>(a, stream);
            case 3: return launch4_k<OK, C, INF, 3>(a, stream);
            case 4: return launch4_k<OK, C, INF, 4>(a, stream);
            case 5: return launch4_k<OK, C, INF, 5>(a, stream);
            case 8: return launch4_k<OK, C, INF, 8>(a, stream);
            case 16: return launch4_k<OK, C, INF, 16>(a, stream);
            case 48: return launch4_k<OK, C, INF, 48>(a, stream);
            case 64: return launch4_k<OK, C, INF, 64>(a, stream);
            default: break;
        }
    }
#endif
    int lds = stft4_lds_bytes(a, OK == 2);
    if (lds > 163840) return -2;
    if constexpr ((VAR & 64) != 0) lds = lds > 90000 ? lds : 90000;  // experiment: 1 block / CU
    auto kern = stft4_kernel<OK, C, INF, VAR>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    constexpr uint64_t per_block = Geo4::WAVES;
    int grid = grid_for(reinterpret_cast<const void*>(kern), Geo4::BLOCK, lds,
                        (a.total_frames + per_block - 1) / per_block, a.grid);
    const uint64_t streams = (uint64_t)grid * per_block;
    const uint64_t fps = (a.total_frames + streams - 1) / streams;
    grid = (int)((a.total_frames + fps * per_block - 1) / (fps * per_block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(Geo4::BLOCK), lds, stream, a, fps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int C, int INF>
static int launch4_c(const StftLaunch& a, hipStream_t s) {
    if (a.out_kind == OUT_COMPLEX) return launch4_k<0, C, INF>(a, s);
    if (a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB) {
        if (!a.mel5_wt || a.mel5_rounds <= 0) return -2;
        return launch4_k<2, C, INF>(a, s);
    }
    return launch4_k<1, C, INF>(a, s);
}

bool stft4_supports(int n_fft, int win, int hop, int in_format, int channels) {
    return n_fft == 2048 && win == n_fft && hop * 4 == n_fft &&
           (in_format == IN_F32 || in_format == IN_S16) && (channels == 1 || channels == 2);
}

int launch_stft4(const StftLaunch& a, hipStream_t s) {
    if (!stft4_supports(a.n_fft, a.win, a.hop, a.in_format, a.channels) || !a.tw4a || !a.tw4b)
        return -2;
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch4_c<2, IN_S16>(a, s) : launch4_c<1, IN_S16>(a, s);
    return a.channels == 2 ? launch4_c<2, IN_F32>(a, s) : launch4_c<1, IN_F32>(a, s);
}

}  // namespace thesia
