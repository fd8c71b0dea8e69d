// stftr_kernels.hip -- the reference-order STREAMING STFT (batch kernel 7): every f32 operation of
// the reference path in the reference's order, as stftx_kernel (stftx_kernels.hip), so the rows
// equal the oracle's bit for bit, with the streaming data movement of the fast kernels
// (stft3/stft5): a wave walks consecutive frames of a stream, the downmixed samples stay in a
// register ring and a hop loads only its new samples.
//
// n_fft 2048 (NC = 1024 complex points), win = n_fft, hop = n_fft / 4: the C2-C4 geometry of
// BASELINE.json. One frame per 64-lane wave, 16 points per lane.
//
// rustfft 4.0 Radix4 for NC = 1024 (oracle cfft_tab, realfft.rs:126-138): input point m sits at
// position p = digit-reverse4(m) (prepare_radix4); level 0 is butterfly_4 over base-4 digit 0 of
// p, levels 1..4 are butterfly_4 over digit l with the table twiddles tw[j t NC / 4^(l+1)], j = p
// mod 4^l. Bit-exactness needs only that every butterfly sees the same operands in the same
// operation order -- which lane holds which point does not matter. So:
//   ring layout   lane l holds m = l + 64 n (n < 16): the hop (256 points) keeps a point in its
//                 lane (the ring shifts by 4 registers). m's base-4 digits (i0 .. i4) are p's
//                 digits reversed: lane l = d4 + 4 d3 + 16 d2, register n = d1 + 4 d0.
//   levels 0, 1   in registers (digits d0, d1); level-1 twiddles are wave-uniform (tw[64 d0 t]).
//   swap          lane bits 4, 5 (d2) <-> register bits 2, 3 (d0): v_permlane16_swap /
//                 v_permlane32_swap, one VALU per dword (no LDS): lane = d4 + 4 d3 + 16 d0,
//                 register = d1 + 4 d2.
//   level 2       in registers (d2; twiddles per lane from the LDS table).
//   transpose     LDS, one row of 64 complex per p >> 6: lane l writes its 16 points into row
//                 d3 + 4 d4 (columns d0 + 4 n), lane reads column c = p mod 64 (row stride 130
//                 floats: conflict-free stores and contiguous row reads).
//   levels 3, 4   in registers (d3, d4): register r holds Z[c + 64 r] (natural order).
//   untangle      realfft.rs:142-157 on the pairs (k, NC - k): the partner of column c is 64 - c,
//                 and lanes are numbered so that it is lane +- 32 (c <= 32: lane c; c > 32: lane
//                 96 - c), so one v_permlane32_swap per dword brings the partner's Z[8 .. 15];
//                 lanes 0 (c = 0) and 32 (c = 32) pair inside their own column.
//   |X|           hypotf as glibc (double, one rounding; exact_math.hpp), |X|^2 as num-complex
//                 norm_sqr, mel as the k-ascending fma chain (a packed stream for 64 lanes,
//                 engine.cpp build_melp), dB with glibc's log10f (exact_math.hpp).
// No fused multiply-add anywhere but the mel chain (the oracle's dot is an fma chain):
// -ffp-contract=off, products as num-complex Mul.
#include "stft3_core.hpp"
#include "stftr_core.hpp"

#include <type_traits>
#include <cstdlib>

namespace thesia {

struct GeoR {
    static constexpr int NC = 1024, L = 64, P = 16, F = NC + 1, SH = 4, KEEP = P - SH;
    // transpose row stride (floats): 128 + 2. A ds_write_b64 serves 16 contiguous lanes per LDS
    // cycle with banks (a/4) mod 32; those lanes write one column of 16 different rows, so rows
    // 2 dwords apart mod 32 put the 16 lanes on all 32 banks once. The reads (ds_read_b64, 32
    // lanes, banks mod 64) take 64 contiguous dwords of a row.
    static constexpr int RS = 130;
    static constexpr int REGION = 16 * RS;     // per-wave LDS region (floats): 2080
    static constexpr int WL_STRIDE = 2 * P + 4;  // window row of a lane (floats)
    static constexpr int WL_FLOATS = L * WL_STRIDE;
    static constexpr int TW_FLOATS = 2 * NC + 4;   // rustfft twiddles tw[0 .. NC)
    static constexpr int SC_FLOATS = 2 * NC + 4;   // realfft sin_cos, entry NC = padding
    static constexpr int LOGT_FLOATS = 64;        // logf's table (exact_math.hpp kLogfT), LDS copy
    static constexpr int TAB_FLOATS = WL_FLOATS + TW_FLOATS + SC_FLOATS + LOGT_FLOATS;
    static_assert(REGION >= 2 * F + 3 && REGION >= kMelpOut + 16 && REGION == stftr_region_floats(), "region");
};

namespace {

// The packed mel stream for 64 lanes per frame (engine.cpp build_melp with L = 64): lane j runs
// its filters' chunks back to back, each a k-ascending fma chain over S float4 steps of the |X|
// row (region), its running sum stored at woff and ANDed with keep after the chunk; chunk c + 1's
// meta, weights and |X| are read before chunk c's chain.
template <int S>
__device__ __forceinline__ void melr_stream(const int4* meta, const float4* wt, float* region, int lj, int C) {
    constexpr int L = GeoR::L;
    char* rb = reinterpret_cast<char*>(region);
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
}

}  // namespace

// KIND: the output kind (kernels.hpp OUT_*), a template parameter so every path is straight-line
// code. C: 1 mono, 2 stereo (interleaved); INF: f32 / s16. WV waves per block (one block per CU):
// 12 (3 waves per SIMD) or 8 (when the mel tables leave no room for 12 regions). VAR: ablations
// of the experiment library only (wrong output by design): 1 |X| by the f32 sqrt, 2 no mel
// stream, 4 no untangle / |X| / mel (the FFT alone).
// DIR (round 6): any other geometry with n_fft 2048 -- the viewer's win 1764 / 1920 and hops 441 /
// 480 (lib.rs:43-46, 44.1 / 48 kHz) -- as stftq_kernel's DIR: every frame loads its samples itself
// (no ring; an odd start sample by sample) and the window step keeps x * w inside the window and
// +0 in the centring pads, whatever the sample there (a mask: the reference pads the windowed
// frame with +0 and reads no sample there, lib.rs:377-385).
// RG (round 6, amp dB): the per-track range of the rows folded into the epilogue (Batch::range,
// as stftq_kernel's RG) instead of the separate pass over the rows.
template <int KIND, int C, int INF, int WV, int VAR = 0, bool DIR = false, bool RG = false>
__global__ void __launch_bounds__(64 * WV)
stftr_kernel(StftLaunch a, uint64_t fps) {
    using G = GeoR;
    using CK = Chunk<C, INF>;
    using CT = typename CK::T;
    using ET = typename std::conditional<INF == IN_S16, int16_t, float>::type;
    constexpr int NC = G::NC, P = G::P, L = G::L, F = G::F, SH = G::SH, KEEP = G::KEEP, RS = G::RS;
    constexpr bool MEL = KIND == OUT_MEL || KIND == OUT_MEL_AMP_DB;
    constexpr bool CPLX = KIND == OUT_COMPLEX;

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtl = lds;
    float2* twl = reinterpret_cast<float2*>(lds + G::WL_FLOATS);
    float2* scl = reinterpret_cast<float2*>(lds + G::WL_FLOATS + G::TW_FLOATS);
    float* wcl = lds + G::TAB_FLOATS;  // DIR: the window step's pad mask (same layout)
    float* work = lds + G::TAB_FLOATS + (DIR ? G::WL_FLOATS : 0);
    const exact::LogfEntry* logt = logf_tab_to_lds(lds + G::WL_FLOATS + G::TW_FLOATS + G::SC_FLOATS);
    int4* pm_lds = reinterpret_cast<int4*>(work + WV * G::REGION);
    float4* pw_lds = reinterpret_cast<float4*>(pm_lds + (MEL ? (a.melr_chunks + 2) * L : 0));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kBlock = 64 * WV;

    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) {  // window: lane row (w[2m], w[2m+1])
        const int m = i >> 1, l = m % L, n = m / L;
        wtl[l * G::WL_STRIDE + 2 * n + (i & 1)] = a.wpad[i];
        if constexpr (DIR)  // the window step's mask: all ones inside the window, 0 in the pads
            wcl[l * G::WL_STRIDE + 2 * n + (i & 1)] = __uint_as_float(i >= a.pad_left && i < a.pad_left + a.win ? ~0u : 0u);
    }
    for (int i = threadIdx.x; i < NC; i += kBlock) {
        twl[i] = a.tw1[i];
        scl[i] = a.sincos[i];
    }
    if (threadIdx.x == 0) scl[NC] = make_float2(0.f, 0.f);
    if constexpr (MEL) {
        for (int i = threadIdx.x; i < (a.melr_chunks + 2) * L; i += kBlock) pm_lds[i] = a.melr_meta[i];
        const int nw = (a.melr_chunks + 1) * a.melr_steps * L;
        for (int i = threadIdx.x; i < nw; i += kBlock) pw_lds[i] = a.melr_wt[i];
    }
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t stream = (uint64_t)blockIdx.x * WV + wave;
    const uint64_t g0 = stream * fps;
    const uint64_t g1 = g0 + fps < total ? g0 + fps : total;
    const int hop = a.hop;
    float* region = work + wave * G::REGION;
    const ET* in = static_cast<const ET*>(a.in);

    float2 raw[P];
    CT pre[SH];
    bool pre_ok = false;
    int hint = -1;
    uint64_t g_beg = 1, g_end = 0, base = 0;
    int64_t n = 0;
    // RG: the range of the rows this wave writes for its current track (r_trk)
    float r_max = -INFINITY, r_min = INFINITY;
    int r_nan = 0, r_trk = -1;
    auto r_flush = [&]() {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            r_max = fmaxf(r_max, __shfl_xor(r_max, m));
            r_min = fminf(r_min, __shfl_xor(r_min, m));
            r_nan |= __shfl_xor(r_nan, m);
        }
        if (lane == 0) {
            int* rp = a.trk_range + 3 * r_trk;
            atomicMax(rp, range_ord(r_max));
            atomicMin(rp + 1, range_ord(r_min));
            if (r_nan) atomicOr(rp + 2, 1);
        }
        r_max = -INFINITY;
        r_min = INFINITY;
        r_nan = 0;
    };
    for (uint64_t it = 0; it < fps; ++it) {  // wave-uniform trip count
        const uint64_t g = g0 + it;
        const bool valid = g < g1;
        // the lane index opaque per frame: the per-lane table addresses are formed in the loop
        // instead of held across it in registers
        int lj = lane;
        asm volatile("" : "+v"(lj));
        int64_t start = 0;
        if (valid) {
            if (g >= g_end || g < g_beg) {
                hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
                g_beg = a.trk_frame0[hint];
                g_end = a.trk_frame0[hint + 1];
                n = (int64_t)a.trk_len[hint];
                base = a.trk_in_off[hint];
            }
            start = (int64_t)(g - g_beg) * hop - NC;  // t hop - win / 2 (pad_left = 0)
        }
        // ---- the frame's downmixed samples: ring shift by SH rows + the prefetched hop ----
        if (DIR && valid && start >= 0 && start + 2 * NC <= n && ((base + (uint64_t)start * C) % (2 * C)) != 0) {
            // (DIR) an interior frame at an odd start: sample by sample
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const int64_t i0 = start + 2 * (lj + L * q);
                raw[q] = make_float2(read_sample<INF>(a.in, base, i0, C, a.fold != 0),
                                     read_sample<INF>(a.in, base, i0 + 1, C, a.fold != 0));
            }
        } else if (pre_ok) {
#pragma unroll
            for (int q = 0; q < KEEP; ++q) raw[q] = raw[q + SH];
#pragma unroll
            for (int q = 0; q < SH; ++q) raw[KEEP + q] = CK::mix(pre[q]);
        } else if (valid && start >= 0 && start + 2 * NC <= n && ((base + (uint64_t)start * C) % (2 * C)) == 0) {
            const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)start * C) + lj;
#pragma unroll
            for (int q = 0; q < P; ++q) raw[q] = CK::mix(src[L * q]);
        } else if (valid) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                wave_lds_sync();
                fill_raw_half<L, P, INF>(a.in, region, lj, start, n, base, C, a.fold != 0, e);
                wave_lds_sync();
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    const float r = region[L * q + lj];
                    if (e == 0) raw[q].x = r; else raw[q].y = r;
                }
            }
            wave_lds_sync();
        } else {
#pragma unroll
            for (int q = 0; q < P; ++q) raw[q] = make_float2(0.f, 0.f);
        }
        // ---- prefetch the next frame's new points (rows KEEP .. P - 1) ----
        {
            const int64_t nstart = start + hop;
            const bool nxt = !DIR && valid && g + 1 < g1 && g + 1 < g_end && nstart + 2 * NC <= n &&
                             nstart + 2 * L * KEEP >= 0 &&
                             ((base + (uint64_t)(nstart + 2 * L * KEEP) * C) % (2 * C)) == 0;
            if (nxt) {
                const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)(nstart + 2 * L * KEEP) * C) + lj;
#pragma unroll
                for (int q = 0; q < SH; ++q) pre[q] = src[L * q];
            }
            pre_ok = nxt;
        }
        // ---- window (lib.rs:379: x * w) ----
        float2 v[P];
        {
            const float4* wr = reinterpret_cast<const float4*>(wtl + lj * G::WL_STRIDE);
#pragma unroll
            for (int q = 0; q < P / 2; ++q) {
                const float4 w = wr[q];
                v[2 * q] = make_float2(raw[2 * q].x * w.x, raw[2 * q].y * w.y);
                v[2 * q + 1] = make_float2(raw[2 * q + 1].x * w.z, raw[2 * q + 1].y * w.w);
            }
            if constexpr (DIR) {  // x * w inside the window (bits unchanged), +0 in the pads, whatever x
                const uint4* cr = reinterpret_cast<const uint4*>(wcl + lj * G::WL_STRIDE);
                auto msk = [](float x, unsigned m) { return __uint_as_float(__float_as_uint(x) & m); };
#pragma unroll
                for (int q = 0; q < P / 2; ++q) {
                    const uint4 c = cr[q];
                    v[2 * q] = make_float2(msk(v[2 * q].x, c.x), msk(v[2 * q].y, c.y));
                    v[2 * q + 1] = make_float2(msk(v[2 * q + 1].x, c.z), msk(v[2 * q + 1].y, c.w));
                }
            }
        }
        // ---- level 0: Butterfly4 over d0 (registers d1 + 4 d0) ----
#pragma unroll
        for (int d1 = 0; d1 < 4; ++d1) rbfly4(v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12]);
        // ---- level 1: butterfly_4 over d1, j = d0, twiddles tw[64 j t] (wave-uniform) ----
#pragma unroll
        for (int j = 0; j < 4; ++j)
            rbfly(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3], twl[64 * j], twl[128 * j], twl[192 * j]);
        // ---- swap lane bits 4, 5 with register bits 2, 3 ----
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if ((q & 4) == 0) pl16(v[q], v[q + 4]);
#pragma unroll
        for (int q = 0; q < 8; ++q) pl32(v[q], v[q + 8]);
        // ---- level 2: butterfly_4 over d2 (registers d1 + 4 d2), j = d0 + 4 d1 ----
        {
            const int d0s = lj >> 4;  // d0 after the swap
#pragma unroll
            for (int d1 = 0; d1 < 4; ++d1) {
                const int j = d0s + 4 * d1;
                rbfly(v[d1], v[d1 + 4], v[d1 + 8], v[d1 + 12], twl[16 * j], twl[32 * j], twl[48 * j]);
            }
            // ---- LDS transpose: row d3 + 4 d4, column d0 + 4 n'; read column col ----
            wave_lds_sync();
            const int wrow = ((lj >> 2) & 3) + 4 * (lj & 3);
            float2* wb = reinterpret_cast<float2*>(region + wrow * RS) + d0s;
#pragma unroll
            for (int q = 0; q < P; ++q) wb[4 * q] = v[q];
        }
        // the lane's column after the transpose: its partner column 64 - col is lane +- 32
        const int col = lj <= 32 ? lj : 96 - lj;
        wave_lds_sync();
        {
            const float2* rb = reinterpret_cast<const float2*>(region) + col;
#pragma unroll
            for (int r = 0; r < P; ++r) v[r] = rb[r * (RS / 2)];
        }
        // ---- level 3: butterfly_4 over d3 (registers d3 + 4 d4), j = col ----
        {
            const float2 w3a = twl[col * 4], w3b = twl[col * 8], w3c = twl[col * 12];
#pragma unroll
            for (int d4 = 0; d4 < 4; ++d4)
                rbfly(v[4 * d4], v[4 * d4 + 1], v[4 * d4 + 2], v[4 * d4 + 3], w3a, w3b, w3c);
        }
        // ---- level 4: butterfly_4 over d4, j = col + 64 d3 ----
#pragma unroll
        for (int d3 = 0; d3 < 4; ++d3) {
            const int j = col + 64 * d3;
            rbfly(v[d3], v[d3 + 4], v[d3 + 8], v[d3 + 12], twl[j], twl[2 * j], twl[3 * j]);
        }
        // v[r] = Z[col + 64 r]. ---- untangle (realfft.rs:142-157) on pairs (k, NC - k) ----
        // the partner column's Z[8 .. 15] by one v_permlane32_swap per dword (lanes < 32 receive
        // into the second operand, lanes >= 32 into the first); lanes 0 and 32 pair inside their
        // own column. Partner of own register r < 8: general and lane 32: Z_partner[15 - r]
        // (= pr[7 - r]); lane 0: Z[(16 - r) & 15] = r == 0 ? v[0] : pr[8 - r]
        const unsigned m_lo = lj < 32 ? ~0u : 0u, m_sp = (lj & 31) == 0 ? ~0u : 0u, m_l0 = lj == 0 ? ~0u : 0u;
        float2 pr[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float2 x = v[8 + i], y = v[8 + i];
            pl32(x, y);
            pr[i] = bsel2(m_sp, v[8 + i], bsel2(m_lo, y, x));
        }
        wave_lds_sync();  // the transpose's reads are done: the region takes the output row
        auto pair = [&](float2 b, float2 rr, float2 sck, float2 sckp, float2& xk, float2& xkp) {
            const float sre = b.x + rr.x, sim = b.y + rr.y;
            const float dre = b.x - rr.x, dim = b.y - rr.y;
            xk.x = 0.5f * ((sre + sck.y * sim) - sck.x * dre);
            xk.y = 0.5f * ((dim - sck.x * sim) - sck.y * dre);
            // partner: b' = rr, r' = b: (rr.re + b.re) = sre (sums commute bit for bit); the
            // differences formed again (rr.re - b.re is -dre except for a zero: +0 either way,
            // where -dre would be -0 -- round 6, test_negative_zero_samples_and_silence)
            const float pdre = rr.x - b.x, pdim = rr.y - b.y;
            xkp.x = 0.5f * ((sre + sckp.y * sim) - sckp.x * pdre);
            xkp.y = 0.5f * ((pdim - sckp.x * sim) - sckp.y * pdre);
        };
        float* row = region;
        constexpr bool FOLD = RG && !CPLX && !MEL;
        float f_max = -INFINITY, f_min = INFINITY;  // (FOLD) this frame's values in this lane
        int f_nan = 0;
        const int sh = MEL ? 0
                     : (int)((reinterpret_cast<uintptr_t>(static_cast<float*>(a.out) + g * (uint64_t)(CPLX ? 2 * F : F)) >> 2) & 3);
        auto emit = [&](int k, float2 x) {
            if constexpr (CPLX) {
                *reinterpret_cast<float2*>(row + sh + 2 * k) = x;
            } else {
                float val;
                if constexpr (KIND == OUT_POWER || KIND == OUT_POWER_DB) {
                    val = x.x * x.x + x.y * x.y;  // num-complex norm_sqr
                    if constexpr (KIND == OUT_POWER_DB) val = rdb(val, a.log_amin, 1e-36f, 10.0f, logt);
                } else {
                    if constexpr ((VAR & 1) != 0) val = __builtin_amdgcn_sqrtf(x.x * x.x + x.y * x.y);
                    else val = exact::hypotf_cr(x.x, x.y);  // num-complex norm (lib.rs:124)
                    if constexpr (KIND == OUT_AMP_DB) val = rdb(val, a.log_amin, 1e-18f, 20.0f, logt);
                }
                row[sh + k] = val;
                if constexpr (FOLD) {
                    f_max = fmaxf(f_max, val);
                    f_min = fminf(f_min, val);
                    f_nan |= val != val;
                }
            }
        };
        const float2* scc = scl + col;              // sin_cos of bins col + 64 r
        const float2* scp = scl + (NC - 448 - col);  // ... of NC - col - 64 r = scp[64 (7 - r)]
#pragma unroll
        for (int r = 0; r < ((VAR & 4) != 0 ? 0 : 8); ++r) {
            const int k = col + 64 * r;
            const float2 rr = bsel2(m_l0, r == 0 ? v[0] : pr[8 - r], pr[7 - r]);
            float2 xk, xkp;
            pair(v[r], rr, scc[64 * r], scp[64 * (7 - r)], xk, xkp);
            if (r == 0) xkp = bsel2(m_l0, make_float2(v[0].x - v[0].y, 0.0f), xkp);  // realfft.rs:157
            emit(k, xk);
            emit(NC - k, xkp);  // (lane 0, r = 0: bin NC)
        }
        {  // lane 0: bin NC / 2 pairs with itself (realfft.rs:142-156 with b = r = Z[NC/2])
            float2 xk, xkp;
            pair(v[8], v[8], scl[NC / 2], scl[NC / 2], xk, xkp);
            if (lj == 0) emit(NC / 2, xk);
        }
        wave_lds_sync();
        if constexpr (MEL) {
            // lib.rs:131 (the packed stream) then amp dB (decibel.rs:79-88)
            if (lj == 0) {
#pragma unroll
                for (int k = F; k < kMelpOut; ++k) row[k] = 0.0f;
            }
            wave_lds_sync();
            if constexpr ((VAR & 6) == 0) {
                if (a.melr_steps == 2) melr_stream<2>(pm_lds, pw_lds, region, lj, a.melr_chunks);
                else melr_stream<3>(pm_lds, pw_lds, region, lj, a.melr_chunks);
            }
            wave_lds_sync();
            const int n_mels = a.n_mels;
            float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
            for (int m = lj; m < n_mels; m += L) {
                const float x = region[kMelpOut + m];
                if (valid) out[m] = KIND == OUT_MEL_AMP_DB ? rdb(x, a.log_amin, 1e-18f, 20.0f, logt) : x;
            }
        } else {
            constexpr int nfl = CPLX ? 2 * F : F;
            float* frow = static_cast<float*>(a.out) + g * (uint64_t)nfl;
            if (valid) store_row_b128<L>(frow, sh, region, nfl, lj);
            if constexpr (FOLD) {  // the wave's track changed: commit the previous one's
                const int t = valid ? hint : -1;
                if (t != r_trk) {  // wave-uniform
                    if (r_trk >= 0) r_flush();
                    r_trk = t;
                }
                if (valid) {
                    r_max = fmaxf(r_max, f_max);
                    r_min = fminf(r_min, f_min);
                    r_nan |= f_nan;
                }
            }
        }
    }
    if constexpr (RG && !CPLX && !MEL)
        if (r_trk >= 0) r_flush();  // the wave's last track
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// the canonical geometry streams (win = n_fft, hop = n_fft / 4); any other (DIR) loads per frame
static bool r_canon(const StftLaunch& a) { return a.win == a.n_fft && a.hop * 4 == a.n_fft; }

static int ldsr_bytes(const StftLaunch& a, int wv) {
    const bool mel = a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB;
    const int meltab = mel ? ((a.melr_chunks + 2) + (a.melr_chunks + 1) * a.melr_steps) * GeoR::L * 16 : 0;
    return (GeoR::TAB_FLOATS + (r_canon(a) ? 0 : GeoR::WL_FLOATS) + wv * GeoR::REGION) * 4 + meltab;
}

template <int KIND, int C, int INF, int WV, int VAR = 0, bool DIR = false, bool RG = false>
static int launchr_k(const StftLaunch& a, hipStream_t s) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (VAR == 0 && KIND == OUT_MEL_AMP_DB && C == 2 && INF == IN_F32 && WV == 12) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        const int v = e ? atoi(e) : 0;
        if (v == 1) return launchr_k<KIND, C, INF, WV, 1>(a, s);
        if (v == 2) return launchr_k<KIND, C, INF, WV, 2>(a, s);
        if (v == 4) return launchr_k<KIND, C, INF, WV, 4>(a, s);
        if (v == 3) return launchr_k<KIND, C, INF, WV, 3>(a, s);
    }
#endif
    const int lds = ldsr_bytes(a, WV);
    if (lds > 163840) return -2;
    auto kern = stftr_kernel<KIND, C, INF, WV, VAR, DIR, RG>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    int grid = grid_for(reinterpret_cast<const void*>(kern), 64 * WV, lds, (a.total_frames + WV - 1) / WV, a.grid,
                        a.grid_share);
    const uint64_t streams = (uint64_t)grid * WV;
    const uint64_t fps = (a.total_frames + streams - 1) / streams;
    grid = (int)((a.total_frames + fps * WV - 1) / (fps * WV));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WV), lds, s, a, fps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the spectrum kinds always fit 12 regions (125 KiB); the mel kinds fall back to 8 when their
// tables leave no room
template <int KIND, int C, int INF, bool DIR = false>
static int launchr_w(const StftLaunch& a, hipStream_t s) {
    if constexpr (KIND == OUT_MEL || KIND == OUT_MEL_AMP_DB) {
        if (a.melr_chunks <= 0) return -2;
        if (ldsr_bytes(a, 12) > 163840) return launchr_k<KIND, C, INF, 8, 0, DIR>(a, s);
    }
    return launchr_k<KIND, C, INF, 12, 0, DIR>(a, s);
}

template <int C, int INF, bool DIR = false>
static int launchr_c(const StftLaunch& a, hipStream_t s) {
    switch (a.out_kind) {
        case OUT_COMPLEX: return launchr_w<OUT_COMPLEX, C, INF, DIR>(a, s);
        case OUT_MAG: return launchr_w<OUT_MAG, C, INF, DIR>(a, s);
        case OUT_POWER: return launchr_w<OUT_POWER, C, INF, DIR>(a, s);
        case OUT_AMP_DB:  // (the range folded in when the batch asks for it: the C5 / viewer kind)
            // (16-wave blocks -- 4 waves per SIMD -- where the fold fits 128 VGPRs without spills
            // and the LDS: mono int16 at the canonical geometry, the C5 rows; 12 elsewhere)
            return a.trk_range ? launchr_k<OUT_AMP_DB, C, INF, (C == 1 && INF == IN_S16 && !DIR) ? 16 : 12, 0, DIR, true>(a, s)
                               : launchr_w<OUT_AMP_DB, C, INF, DIR>(a, s);
        case OUT_POWER_DB: return launchr_w<OUT_POWER_DB, C, INF, DIR>(a, s);
        case OUT_MEL: return launchr_w<OUT_MEL, C, INF, DIR>(a, s);
        case OUT_MEL_AMP_DB: return launchr_w<OUT_MEL_AMP_DB, C, INF, DIR>(a, s);
        default: return -2;
    }
}

bool stftr_supports(int n_fft, int win, int hop, int in_format, int channels) {
    if (n_fft != 2048 || !(channels == 1 || channels == 2)) return false;
    if (win == n_fft && hop * 4 == n_fft) return in_format == IN_F32 || in_format == IN_S16;
    // any other geometry (DIR): even win <= n_fft (the frame start t hop - n_fft / 2 is the
    // reference's t hop - win / 2 - pad_left, lib.rs:400-401), f32
    return in_format == IN_F32 && hop >= 1 && win >= 2 && win <= n_fft && win % 2 == 0;
}

int stftr_lds_bytes(const StftLaunch& a) { return ldsr_bytes(a, 8); }

int launch_stftr(const StftLaunch& a, hipStream_t s) {
    if (!stftr_supports(a.n_fft, a.win, a.hop, a.in_format, a.channels)) return -2;
    if (!r_canon(a))  // the viewer's geometries: f32 mono / stereo (MultiTrack's mono pool)
        return a.channels == 2 ? launchr_c<2, IN_F32, true>(a, s) : launchr_c<1, IN_F32, true>(a, s);
    if (a.in_format == IN_S16) return a.channels == 2 ? launchr_c<2, IN_S16>(a, s) : launchr_c<1, IN_S16>(a, s);
    return a.channels == 2 ? launchr_c<2, IN_F32>(a, s) : launchr_c<1, IN_F32>(a, s);
}

}  // namespace thesia
