// stft6_kernels.hip -- the streaming STFT kernel with ONE frame per 64-lane wave, for the
// headline geometry n_fft 2048 (NC = 1024 complex points), win = n_fft, hop = n_fft/4, mel kinds.
//
// Why: stft5 (two 32-lane frames per wave) holds 32 ring points + 32 frame points per lane,
// 253 VGPRs, so two waves per SIMD, and at two waves its instruction stream stalls ~40 % of the
// time. Spreading a frame over 64 lanes halves every per-lane array (ring 16
// points, frame 16, prefetched hop 4), which fits three waves per SIMD (<= 168 VGPRs; 12-wave
// blocks, one per CU), while keeping stft5's property that the realfft untangle
// (realfft.rs:140-157) needs no cross-lane exchange.
//
// FFT: NC = 1024 = 16 (n1) x 64 (j), and the 64 = 16 (a) x 4 (b) with j = 4 a + b:
//   stage 1   lane j: Y[j][k1] = DFT-16 over n1 of z[64 n1 + j] (the window fused into its
//             first radix-4 level), times W_1024^{j k1} (LDS table);
//   transpose 1: lane t = 4 k1 + b receives Y[4 a + b][k1], a < 16 (one ds_write_b64 per k1,
//             eight ds_read_b128; segments b >= 2 store their halves swapped: conflict-free);
//   stage 2a  Z[c] = DFT-16 over a, times W_64^{b c} (LDS table);
//   transpose 2: row k1, segment b holds Z[c], c < 16 (eight ds_write_b128), and row 16 holds
//             row 0 shifted by one (position p: c = p + 1 mod 16; written by the four k1 = 0
//             lanes);
//   stage 2b  lane t = 4 k1 + x reads, for every b, its own row's c in [4x, 4x + 4) and the
//             partner row 16 - k1 at positions 15 - c, and runs the DFT-4 over b on both:
//             X[k1 + 16 c + 256 d] for d = 0, 1 from its own row, and for d' = 3, 2 from the
//             partner's, which are exactly the untangle partners NC - k of its own bins
//             ((k1, c, d) pairs with (16 - k1, 15 - c, 3 - d); for k1 = 0 with (0, 16 - c, 3 - d),
//             hence the shifted row 16). Every bin is formed once, 8 pairs per lane.
//   Lane 0 (k1 = 0, c = 0) pairs differently: bin 0 with NC (from Z[0]), 256 with 768, 512 with
//   itself; per-slot selects cover it, as in stft5.
// The index map is modelled in numpy by scripts/model_stft6.py (reproduces np.fft.rfft and
// counts the LDS bank slots of every transpose access).
//
// Mel (lib.rs:131): stft5's packed stream (engine.cpp build_melp) for 64 lanes. With 64 lanes
// the widest filters (not the lane count) would set the chunk count, so a filter wider than the
// plan's cap runs as two pieces on two lanes, each a k-ascending fma chain, summed at the
// output (A + B; unsplit mels add the zero at region[F]).
#include "stft3_core.hpp"

#include <type_traits>

namespace thesia {

struct Geo6 {
    static constexpr int NC = 1024, L = 64, P = 16, SH = P / 4, F = NC + 1, F4 = 1028;
    static constexpr int WV = 12;  // waves per block, one block per CU: 3 per SIMD
    static constexpr int BLOCK = 64 * WV;
    static constexpr int SEG = 32;          // transpose segment: 16 complex
    static constexpr int TS = 4 * SEG + 4;  // transpose row: 4 segments (+4 floats: bank spread)
    static constexpr int ROWS = 17;         // 16 rows + row 0 shifted (the k1 = 0 partners)
    static constexpr int RS = ROWS * TS;    // region per wave (floats)
    static constexpr int WL_STRIDE = 2 * P + 4, WL_FLOATS = L * WL_STRIDE;  // window rows
    static constexpr int TA_STRIDE = 2 * P + 4, TA_FLOATS = L * TA_STRIDE;  // W_1024^{j k1} rows
    static constexpr int TB_STRIDE = 36, TB_FLOATS = 4 * TB_STRIDE;         // W_64^{b c} rows
    static constexpr int TAB_FLOATS = WL_FLOATS + TA_FLOATS + TB_FLOATS;
    static_assert(RS % 4 == 0 && TAB_FLOATS % 4 == 0, "16-byte aligned regions");
    static_assert(RS >= F4 + 2 * 128 + 16, "the |X| row and two mel slots per mel fit a region");
};
static_assert(Geo6::F4 == kMelpOut && Geo6::RS == kStft6Region, "melp region layout");

// The packed mel stream for 64 lanes (melp5 of stft5_kernels.hip; engine.cpp build_melp):
// chunks pipelined one ahead, a chunk's running sum stored at woff(c) and ANDed with keep(c).
// The frame's mels then leave as dB rows: mel m = A[m] + B[m] (bo: B's float offset per mel).
template <int S>
__device__ __forceinline__ void melp6(const StftLaunch& a, float* region, const int4* meta,
                                      const float4* wt, const int* bo, int j, uint64_t g, bool valid) {
    constexpr int L = Geo6::L;
    const int C = a.melp_chunks;
    char* rb = reinterpret_cast<char*>(region);
    int lj = j;
    asm volatile("" : "+v"(lj));
    const int4* mp = meta + lj;
    const float4* wp = wt + lj;
    struct Buf {
        float4 w[S], x[S];
        int4 m;
    };
    auto issue = [&](int c, int xoff, Buf& b) {
        b.m = mp[(c + 1) * L];
#pragma unroll
        for (int u = 0; u < S; ++u) b.w[u] = wp[(c * S + u) * L];
        const float4* xp = reinterpret_cast<const float4*>(rb + xoff);
#pragma unroll
        for (int u = 0; u < S; ++u) b.x[u] = xp[u];
        __builtin_amdgcn_sched_barrier(0);
    };
    float acc = 0.0f;
    auto chain = [&](const Buf& b) {
#pragma unroll
        for (int u = 0; u < S; ++u) {
            acc = __builtin_fmaf(b.x[u].x, b.w[u].x, acc);
            acc = __builtin_fmaf(b.x[u].y, b.w[u].y, acc);
            acc = __builtin_fmaf(b.x[u].z, b.w[u].z, acc);
            acc = __builtin_fmaf(b.x[u].w, b.w[u].w, acc);
        }
        *reinterpret_cast<float*>(rb + b.m.x) = acc;
        acc = __builtin_bit_cast(float, __builtin_bit_cast(int, acc) & b.m.y);
    };
    Buf A, B;
    int c = 0;
    const int x0 = mp[0].z;
    if (C & 1) {
        issue(0, x0, B);
        issue(1, B.m.z, A);
        chain(B);
        c = 1;
    } else {
        issue(0, x0, A);
    }
    for (; c < C; c += 2) {
        issue(c + 1, A.m.z, B);
        chain(A);
        issue(c + 2, B.m.z, A);
        chain(B);
    }
    wave_lds_sync();
    const int n_mels = a.n_mels;
    const bool db = a.out_kind == OUT_MEL_AMP_DB;
    float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
    const float* mo = region + kMelpOut;
    if (a.melp_v4) {  // n_mels % 4 == 0, <= 128, aligned rows: one 8-byte store per lane
        if (2 * lj < n_mels) {
            float2 r = *reinterpret_cast<const float2*>(mo + 2 * lj);
            const int2 b2 = *reinterpret_cast<const int2*>(bo + 2 * lj);
            r.x += region[b2.x];
            r.y += region[b2.y];
            if (db) {
                r.x = db_of(r.x, a.log_amin, 1e-18f, 20.0f);
                r.y = db_of(r.y, a.log_amin, 1e-18f, 20.0f);
            }
            if (valid) st_out(reinterpret_cast<float2*>(out + 2 * lj), r);
        }
    } else {
        for (int m = lj; m < n_mels; m += L) {
            const float v = mo[m] + region[bo[m]];
            if (valid) st_out(out + m, db ? db_of(v, a.log_amin, 1e-18f, 20.0f) : v);
        }
    }
}

// C: 1 mono, 2 stereo (interleaved); INF: f32 / s16. Mel kinds only (OUT_MEL, OUT_MEL_AMP_DB).
template <int C, int INF>
__global__ void __launch_bounds__(Geo6::BLOCK, Geo6::WV / 4)
stft6_kernel(StftLaunch a, uint64_t fps) {
    using G = Geo6;
    using CK = Chunk<C, INF>;
    using CT = typename CK::T;
    using ET = typename std::conditional<INF == IN_S16, int16_t, float>::type;
    constexpr int NC = G::NC, P = G::P, L = G::L, F = G::F, SH = G::SH, TS = G::TS, SEG = G::SEG;

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtl = lds;
    float* tal = lds + G::WL_FLOATS;
    float* tbl = tal + G::TA_FLOATS;
    float* work = lds + G::TAB_FLOATS;
    int4* pm_lds = reinterpret_cast<int4*>(work + G::WV * G::RS);
    float4* pw_lds = reinterpret_cast<float4*>(pm_lds + (a.melp_chunks + 2) * L);
    int* bo_lds = reinterpret_cast<int*>(pw_lds + (a.melp_chunks + 1) * a.melp_steps * L);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int hi4 = lane >> 2, lo4 = lane & 3;  // (k1, b) in stage 2a, (k1, x) in stage 2b
    const bool z0 = lane == 0;

    for (int i = threadIdx.x; i < 2 * NC; i += G::BLOCK) {  // w/2 is exact (realfft's 1/2)
        const int m = i >> 1, jj = m % L, n1 = m / L;
        wtl[jj * G::WL_STRIDE + 2 * n1 + (i & 1)] = a.wpad[i] * 0.5f;
    }
    for (int i = threadIdx.x; i < L * P; i += G::BLOCK) {  // [j][k1] W_1024^{j k1}
        const int jj = i / P, k1 = i % P;
        *reinterpret_cast<float2*>(tal + jj * G::TA_STRIDE + 2 * k1) = a.tw6[i];
    }
    for (int i = threadIdx.x; i < 4 * 16; i += G::BLOCK) {  // [b][c] W_64^{b c}
        *reinterpret_cast<float2*>(tbl + (i >> 4) * G::TB_STRIDE + 2 * (i & 15)) = a.tw6[L * P + i];
    }
    for (int i = threadIdx.x; i < (a.melp_chunks + 2) * L; i += G::BLOCK) pm_lds[i] = a.melp_meta[i];
    for (int i = threadIdx.x; i < (a.melp_chunks + 1) * a.melp_steps * L; i += G::BLOCK) pw_lds[i] = a.melp_wt[i];
    for (int i = threadIdx.x; i < a.n_mels; i += G::BLOCK) bo_lds[i] = a.melp_bo[i];
    // untangle rotations (realfft's sin_cos table) of the lane's 8 pairs: slot 2 i + d is bin
    // k1 + 16 (4 x + i) + 256 d; lane 0's slots 0 / 1 are bins 256 / 512
    float2 rot[8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            const int k = (z0 && i == 0) ? 256 + 256 * d : hi4 + 64 * lo4 + 16 * i + 256 * d;
            rot[2 * i + d] = a.sincos[k];
        }
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t stream = (uint64_t)blockIdx.x * G::WV + wave;
    const uint64_t g0 = stream * fps;
    const uint64_t g1 = g0 + fps < total ? g0 + fps : total;
    const int hop = a.hop;
    float* region = work + wave * G::RS;
    const ET* in = static_cast<const ET*>(a.in);

    float2 raw[P];
    CT pre[SH];
    bool pre_ok = false;
    int hint = -1;
    uint64_t g_beg = 1, g_end = 0, base = 0;
    int64_t n = 0;
    for (uint64_t it = 0; it < fps; ++it) {  // wave-uniform trip count
        __builtin_amdgcn_s_setprio(0);
        const uint64_t g = g0 + it;
        const bool valid = g < g1;
        // opaque per frame: the per-lane offsets stay inside the loop (not hoisted into VGPRs)
        int wj = lane, wq = hi4, wx = lo4;
        asm volatile("" : "+v"(wj), "+v"(wq), "+v"(wx));
        int64_t start = 0;
        if (valid) {
            if (g >= g_end || g < g_beg) {
                hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
                g_beg = a.trk_frame0[hint];
                g_end = a.trk_frame0[hint + 1];
                n = (int64_t)a.trk_len[hint];
                base = a.trk_in_off[hint];
            }
            start = (int64_t)(g - g_beg) * hop - NC;  // half_win = NC, pad_left = 0
        }
        // ---- the frame's raw samples: shift by SH points + the prefetched hop ----
        if (pre_ok) {
#pragma unroll
            for (int n1 = 0; n1 < P - SH; ++n1) raw[n1] = raw[n1 + SH];
#pragma unroll
            for (int q = 0; q < SH; ++q) raw[P - SH + q] = CK::mix(pre[q]);
        } else if (valid && start >= 0 && start + 2 * NC <= n && ((base + (uint64_t)start * C) % (2 * C)) == 0) {
            const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)start * C) + wj;
            static_for<0, P>([&](auto qc) {
                constexpr int n1 = decltype(qc)::value;
                raw[n1] = CK::mix(src[L * n1]);
            });
        } else if (valid) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                wave_lds_sync();
                fill_raw_half<L, P, INF>(a.in, region, lane, start, n, base, C, a.fold != 0, e);
                wave_lds_sync();
                static_for<0, P>([&](auto qc) {
                    constexpr int n1 = decltype(qc)::value;
                    const float r = region[L * n1 + lane];
                    if (e == 0) raw[n1].x = r; else raw[n1].y = r;
                });
            }
        } else {
#pragma unroll
            for (int n1 = 0; n1 < P; ++n1) raw[n1] = make_float2(0.f, 0.f);
        }
        // ---- prefetch the next frame's new points P-SH .. P-1 ----
        {
            const int64_t nstart = start + hop;
            const int64_t off = nstart + 2 * L * (P - SH);
            const bool nxt = valid && g + 1 < g1 && g + 1 < g_end && nstart + 2 * NC <= n && off >= 0 &&
                             ((base + (uint64_t)off * C) % (2 * C)) == 0;
            if (nxt) {
                const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)off * C) + wj;
#pragma unroll
                for (int q = 0; q < SH; ++q) pre[q] = src[L * q];
            }
            pre_ok = nxt;
        }
        // ---- stage 1: window inside the first radix-4 level of the DFT-16 (as stft5) ----
        float2 v[P];
        {
            const float4* wrow = reinterpret_cast<const float4*>(wtl + wj * G::WL_STRIDE);
            static_for<0, 2>([&](auto jc) {
                constexpr int jp = decltype(jc)::value;
                const float4 wq4[4] = {wrow[jp], wrow[jp + 2], wrow[jp + 4], wrow[jp + 6]};
                static_for<0, 2>([&](auto hc) {
                    constexpr int h = decltype(hc)::value, jj = 2 * jp + h;
                    auto wv = [&](int t) {
                        return h == 0 ? make_float2(wq4[t].x, wq4[t].y) : make_float2(wq4[t].z, wq4[t].w);
                    };
                    const float2 w0 = wv(0), w1 = wv(1), w2 = wv(2), w3 = wv(3);
                    const float2 a0 = raw[jj], a1 = raw[jj + 4], a2 = raw[jj + 8], a3 = raw[jj + 12];
                    const float2 m2 = make_float2(a2.x * w2.x, a2.y * w2.y);
                    const float2 m3 = make_float2(a3.x * w3.x, a3.y * w3.y);
                    const float2 t0 = make_float2(__builtin_fmaf(a0.x, w0.x, m2.x), __builtin_fmaf(a0.y, w0.y, m2.y));
                    const float2 t1 = make_float2(__builtin_fmaf(a0.x, w0.x, -m2.x), __builtin_fmaf(a0.y, w0.y, -m2.y));
                    const float2 t2 = make_float2(__builtin_fmaf(a1.x, w1.x, m3.x), __builtin_fmaf(a1.y, w1.y, m3.y));
                    const float2 t3 = mul_negi(make_float2(__builtin_fmaf(a1.x, w1.x, -m3.x), __builtin_fmaf(a1.y, w1.y, -m3.y)));
                    v[jj] = cadd(t0, t2);
                    v[jj + 4] = twc<16, jj>(cadd(t1, t3));
                    v[jj + 8] = twc<16, 2 * jj>(csub(t0, t2));
                    v[jj + 12] = twc<16, 3 * jj>(csub(t1, t3));
                });
            });
        }
        pin(v);
        dif_fft<4, 1, 0, P>(v);
        dif_fft<4, 1, 4, P>(v);
        dif_fft<4, 1, 8, P>(v);
        dif_fft<4, 1, 12, P>(v);
        pin(v);
        {  // W_1024^{j k1}: row j, float4 u = (k1 = 2u, 2u + 1)
            const float4* tp = reinterpret_cast<const float4*>(tal + wj * G::TA_STRIDE);
            float4 tw[8];
            static_for<0, 8>([&](auto uc) { tw[decltype(uc)::value] = tp[decltype(uc)::value]; });
            static_for<0, 8>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                if constexpr (u > 0) {
                    constexpr int pk0 = ce_pos(P, 2 * u);
                    v[pk0] = cmul(v[pk0], make_float2(tw[u].x, tw[u].y));
                }
                constexpr int pk1 = ce_pos(P, 2 * u + 1);
                v[pk1] = cmul(v[pk1], make_float2(tw[u].z, tw[u].w));
            });
        }
        // ---- transpose 1: row k1, segment b = j % 4, complex a = j / 4 (halves swapped for
        // b >= 2) ----
        wave_lds_sync();
        {
            const int b = wj & 3, sw = b >= 2 ? 8 : 0;
            float* wp = region + b * SEG + 2 * ((wj >> 2) ^ sw);
            static_for<0, P>([&](auto kc) {
                constexpr int k1 = decltype(kc)::value;
                constexpr int pk = ce_pos(P, k1);  // (constexpr: a runtime ce_pos is a call)
                *reinterpret_cast<float2*>(wp + k1 * TS) = v[pk];
            });
        }
        wave_lds_sync();
        {
            const int s16 = wx >= 2 ? 16 : 0;
            const float* rowb = region + wq * TS + wx * SEG;
            const float4* pa = reinterpret_cast<const float4*>(rowb + s16);  // u < 4 (logical)
            const float4* pb = reinterpret_cast<const float4*>(rowb - s16);  // u >= 4
            static_for<0, 8>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                const float4 t = u < 4 ? pa[u] : pb[u];
                v[2 * u] = make_float2(t.x, t.y);
                v[2 * u + 1] = make_float2(t.z, t.w);
            });
        }
        // ---- stage 2a: DFT-16 over a, W_64^{b c} ----
        pin(v);
        dif_fft<P, 1, 0, P>(v);
        pin(v);
        {
            const float4* tp = reinterpret_cast<const float4*>(tbl + wx * G::TB_STRIDE);
            float4 tw[8];
            static_for<0, 8>([&](auto uc) { tw[decltype(uc)::value] = tp[decltype(uc)::value]; });
            static_for<0, 8>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                if constexpr (u > 0) {
                    constexpr int pk0 = ce_pos(P, 2 * u);
                    v[pk0] = cmul(v[pk0], make_float2(tw[u].x, tw[u].y));
                }
                constexpr int pk1 = ce_pos(P, 2 * u + 1);
                v[pk1] = cmul(v[pk1], make_float2(tw[u].z, tw[u].w));
            });
        }
        // ---- transpose 2: row k1, segment b, complex c; row 16 = row 0 shifted by one ----
        wave_lds_sync();
        {
            float4* wp = reinterpret_cast<float4*>(region + wq * TS + wx * SEG);
            static_for<0, 8>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                constexpr int p0 = ce_pos(P, 2 * u), p1 = ce_pos(P, 2 * u + 1);
                const float2 e0 = v[p0], e1 = v[p1];
                wp[u] = make_float4(e0.x, e0.y, e1.x, e1.y);
            });
            if (wq == 0) {
                float4* wz = reinterpret_cast<float4*>(region + 16 * TS + wx * SEG);
                static_for<0, 8>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    constexpr int p0 = ce_pos(P, (2 * u + 1) & 15), p1 = ce_pos(P, (2 * u + 2) & 15);
                    const float2 e0 = v[p0], e1 = v[p1];
                    wz[u] = make_float4(e0.x, e0.y, e1.x, e1.y);
                });
            }
        }
        wave_lds_sync();
        // own[b][i] = T[k1][b][4x + i]; par[b][i] = partner row at position 15 - 4x - i
        float2 own[4][4], par[4][4];
        {
            const float4* po = reinterpret_cast<const float4*>(region + wq * TS + 8 * wx);
            const float4* pp = reinterpret_cast<const float4*>(region + (16 - wq) * TS + 24 - 8 * wx);
            static_for<0, 4>([&](auto bc) {
                constexpr int b = decltype(bc)::value;
                const float4 o0 = po[b * SEG / 4], o1 = po[b * SEG / 4 + 1];
                const float4 p0 = pp[b * SEG / 4], p1 = pp[b * SEG / 4 + 1];
                own[b][0] = make_float2(o0.x, o0.y);
                own[b][1] = make_float2(o0.z, o0.w);
                own[b][2] = make_float2(o1.x, o1.y);
                own[b][3] = make_float2(o1.z, o1.w);
                par[b][3] = make_float2(p0.x, p0.y);
                par[b][2] = make_float2(p0.z, p0.w);
                par[b][1] = make_float2(p1.x, p1.y);
                par[b][0] = make_float2(p1.z, p1.w);
            });
        }
        wave_lds_sync();  // the |X| row overwrites the transpose
        __builtin_amdgcn_s_setprio(2);
        // ---- stage 2b (DFT-4 over b), untangle, |X| (lib.rs:124) ----
        float mag[16];
        float2 e0 = make_float2(0.f, 0.f);
        static_for<0, 4>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const float2 o0 = own[0][i], o1 = own[1][i], o2 = own[2][i], o3 = own[3][i];
            const float2 A = cadd(o0, o2), B = cadd(o1, o3), Cc = csub(o0, o2), D = csub(o1, o3);
            const float2 d0 = cadd(A, B);
            const float2 d1 = make_float2(Cc.x + D.y, Cc.y - D.x);  // C - i D
            const float2 q0 = par[0][i], q1 = par[1][i], q2 = par[2][i], q3 = par[3][i];
            const float2 Ap = cadd(q0, q2), Bp = cadd(q1, q3), Cp = csub(q0, q2), Dp = csub(q1, q3);
            const float2 p3 = make_float2(Cp.x - Dp.y, Cp.y + Dp.x);  // C' + i D'
            const float2 p2 = csub(Ap, Bp);
            float2 b0 = d0, r0 = p3, b1 = d1, r1 = p2;
            if constexpr (i == 0) {  // lane 0: (256, 768), (512, 512); bins 0 / NC from d0
                e0 = d0;
                b0.x = z0 ? d1.x : b0.x;
                b0.y = z0 ? d1.y : b0.y;
                b1.x = z0 ? p2.x : b1.x;
                b1.y = z0 ? p2.y : b1.y;
            }
            auto pair = [&](float2 bb, float2 rr, float2 sc, float& m1, float& m2, bool self) {
                // realfft.rs:148-154 on the pair (Z_k, Z_{NC-k}); the 1/2 is in the window
                const float ar = bb.x + rr.x, ai = bb.y - rr.y;
                const float br = bb.x - rr.x, bi = bb.y + rr.y;
                const float p = __builtin_fmaf(sc.y, br, sc.x * bi);
                const float q = __builtin_fmaf(sc.y, bi, -(sc.x * br));
                const float x1r = ar + q, x1i = ai - p;
                float x2r = ar - q, x2i = -ai - p;
                x2r = self ? x1r : x2r;
                x2i = self ? x1i : x2i;
                m1 = __builtin_fmaf(x1r, x1r, x1i * x1i);
                m2 = __builtin_fmaf(x2r, x2r, x2i * x2i);
            };
            pair(b0, r0, rot[2 * i], mag[4 * i], mag[4 * i + 1], false);
            pair(b1, r1, rot[2 * i + 1], mag[4 * i + 2], mag[4 * i + 3], i == 0 && z0);
        });
        pin_f(mag);
#pragma unroll
        for (int i = 0; i < 16; ++i) mag[i] = __builtin_amdgcn_sqrtf(mag[i]);
        pin_f(mag);
        {
            const int kb = wq + 64 * wx;
            const int k00 = z0 ? 256 : kb, k01 = z0 ? 512 : kb + 256;
            region[k00] = mag[0];
            region[NC - k00] = mag[1];
            region[k01] = mag[2];
            region[NC - k01] = mag[3];
            float* lo = region + kb;
            float* hi = region + NC - kb;
            static_for<1, 4>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                lo[16 * i] = mag[4 * i];
                hi[-16 * i] = mag[4 * i + 1];
                lo[16 * i + 256] = mag[4 * i + 2];
                hi[-16 * i - 256] = mag[4 * i + 3];
            });
            if (z0) {  // Z[0] with itself: bins 0 and NC (s = 0, co = 1)
                const float ar = e0.x + e0.x, bi = e0.y + e0.y, x0 = ar + bi, xn = ar - bi;
                region[0] = __builtin_amdgcn_sqrtf(__builtin_fmaf(x0, x0, 0.0f));
                region[NC] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xn, xn, 0.0f));
#pragma unroll
                for (int k = F; k < G::F4; ++k) region[k] = 0.0f;
            }
        }
        wave_lds_sync();
        if (a.melp_steps == 2) melp6<2>(a, region, pm_lds, pw_lds, bo_lds, lane, g, valid);
        else melp6<3>(a, region, pm_lds, pw_lds, bo_lds, lane, g, valid);
    }
}

// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
int stft6_lds_bytes(const StftLaunch& a) {
    const int mel = ((a.melp_chunks + 2) + (a.melp_chunks + 1) * a.melp_steps) * Geo6::L * 4 + a.n_mels;
    return (Geo6::TAB_FLOATS + Geo6::WV * Geo6::RS + mel) * 4;
}

template <int C, int INF>
static int launch6_k(const StftLaunch& a, hipStream_t stream) {
    if (a.melp_chunks <= 0 || !a.melp_bo || !a.tw6 || (a.melp_steps != 2 && a.melp_steps != 3)) return -2;
    const int lds = stft6_lds_bytes(a);
    if (lds > 163840) return -2;
    auto kern = stft6_kernel<C, INF>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    constexpr uint64_t per_block = Geo6::WV;
    int grid = grid_for(reinterpret_cast<const void*>(kern), Geo6::BLOCK, lds,
                        (a.total_frames + per_block - 1) / per_block, a.grid);
    const uint64_t streams = (uint64_t)grid * per_block;
    const uint64_t fps = (a.total_frames + streams - 1) / streams;
    grid = (int)((a.total_frames + fps * per_block - 1) / (fps * per_block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(Geo6::BLOCK), lds, stream, a, fps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

bool stft6_supports(int n_fft, int win, int hop, int in_format, int channels, int out_kind) {
    return n_fft == 2048 && win == n_fft && hop * 4 == n_fft &&
           (in_format == IN_F32 || in_format == IN_S16) && (channels == 1 || channels == 2) &&
           (out_kind == OUT_MEL || out_kind == OUT_MEL_AMP_DB);
}

int launch_stft6(const StftLaunch& a, hipStream_t s) {
    if (!stft6_supports(a.n_fft, a.win, a.hop, a.in_format, a.channels, a.out_kind)) return -2;
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch6_k<2, IN_S16>(a, s) : launch6_k<1, IN_S16>(a, s);
    return a.channels == 2 ? launch6_k<2, IN_F32>(a, s) : launch6_k<1, IN_F32>(a, s);
}

}  // namespace thesia
