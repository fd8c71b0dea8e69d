// stft5_kernels.hip -- the streaming STFT kernel for n_fft 2048 (NC = 1024 complex points),
// win = n_fft, hop = n_fft/4: the headline geometry of BASELINE.json (configs C2-C5).
//
// Same contract and the same streaming register ring as stft3_kernel (stft3_kernels.hip: each
// wave runs two frame streams on its 32-lane halves; a stream's downmixed samples stay in
// registers and a hop loads only its new samples). What changes is the second FFT stage, so
// that the realfft untangle (realfft.rs:140-157) needs no cross-lane exchange:
//
//   NC = 32 x 32. Stage 1 (lane j = n2): Y[j][k1] = DFT-32 over n1 of z[32 n1 + j], times
//   W_1024^{j k1}; LDS transpose. In stft3, lane j then runs the DFT-32 of column k1 = j and
//   holds the bins k = j + 32 k2, whose untangle partners NC - k = (32 - j) + 32 (31 - k2) live
//   in lane 32 - j (one ds_bpermute per value). Here lane j reads TWO transpose rows, its own
//   column A = j and the partner column B = (32 - j) mod 32, and splits both DFT-32s by their
//   first radix-2 step: the even outputs of A (a DFT-16 of A[n] + A[n+16]) and the odd outputs
//   of B (a DFT-16 of (B[n] - B[n+16]) W_32^n). Bin A + 64 i = E[i] then pairs with
//   NC - A - 64 i = B + 32 (31 - 2 i) = O[15 - i] in the same lane. The arithmetic is that of
//   one DFT-32 per lane, as before; the exchange becomes 8 more ds_read_b128 per transpose pass.
//   Lane 0 (A = B = 0) pairs its own outputs differently (O with O, E with E, E[0] and E[8]
//   with themselves: bins 0, NC and NC/2); per-slot selects cover it, as in stft3.
//
// Occupancy: two waves per SIMD (8-wave blocks, 253 VGPRs: the ring, the frame's points, the
// prefetched hop and the per-lane untangle rotations). Three waves (12-wave blocks, <= 168
// VGPRs) compiled without spills only with the hop prefetched by LDS-DMA, the rotations in LDS
// and 32-bit frame words, and measured slower; those compile-time variants (and
// the unfused window / split partner-row reads) were removed from this file in round 3 and live
// in git history (commit 490a8f5, THESIA_WV5 / DMA5 / SC5 / S32 / WF5 / BH5 / TWC5 / PF5). The
// two frames of a wave keep their LDS regions on opposite halves of the 64 banks.
#include "stft3_core.hpp"

#include <cstdlib>
#include <type_traits>

namespace thesia {

#ifdef THESIA_MARKS
#define MARK5(x, i) asm volatile("; MARK " #x)
#elif defined(THESIA_STAMPS)
// diagnostic build (scripts/stamps.py): the cycles since the previous mark go to phase i
#define MARK5(x, i)                                                                        \
    do {                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        unsigned long long t_;                                                             \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        st_acc[i] += t_ - st_last;                                                         \
        st_last = t_;                                                                      \
    } while (0)
#else
#define MARK5(x, i)
#endif

struct Geo5 {
    static constexpr int NC = 1024, L = 32, P = 32, FPW = 2, F = NC + 1, SH = P / 4;
    static constexpr int S = L + 4;       // transpose row stride (16 lanes of a b128 read: distinct banks)
    static constexpr int WV = 8;          // waves per block: 2 per SIMD
    static constexpr int BLOCK = 64 * WV;
    static constexpr int STREAMS = WV * FPW;
    // region per stream: the transpose (P * S = 1152 floats), the |X| row (1028) or a staged
    // linear row (F + 6); RS = 1184 = 32 mod 64 puts the wave's two frames on opposite bank
    // halves (RS_MIN when the mel weights leave no room for it)
    static constexpr int RS = 1184, RS_MIN = 1152;
    static constexpr int WL_STRIDE = 2 * P + 4, WL_FLOATS = L * WL_STRIDE;
    static constexpr int TW_FLOATS = 2 * P * L;
    static constexpr int TAB_FLOATS = WL_FLOATS + TW_FLOATS;
    static constexpr int TWC = 8;  // stage-1 twiddle float4 reads per batch
    static_assert(RS_MIN >= P * S && RS_MIN >= F + 6 && RS_MIN % 4 == 0 && RS % 4 == 0, "region");
};

// (sin, cos)(pi (kb + 64 i) / NC) from the lane's base (sin, cos)(pi kb / NC): rotation by
// pi i / 16, compile-time constants (f64-rounded), as stft3's untangle does per 32 bins.
template <int I>
__device__ __forceinline__ void rot16(float2 ub, float& s, float& co) {
    if constexpr (I == 0) {
        s = ub.x;
        co = ub.y;
    } else {
        constexpr float cb = ce_tw_re(I, 32);
        constexpr float sb = -ce_tw_im(I, 32);
        s = __builtin_fmaf(ub.x, cb, ub.y * sb);
        co = __builtin_fmaf(ub.y, cb, -(ub.x * sb));
    }
}

// The realfft untangle of slots I0 <= i < I1 (see the header): calls
// epi(k, re, im, integral_constant<2 (i - I0) + h>) for bin k (h = 0) and NC - k (h = 1).
// v[ce_pos(16, i)] = E[i], v[16 + ce_pos(16, i)] = O[i].
// The (sin, cos) of slot i come from a per-lane table computed once from the lane's two bases
// (32 VGPRs held for 64 VALU per frame pair).
struct RotTable {
    const float2 (&t)[16];
    template <int I>
    __device__ __forceinline__ void get(float& s, float& co) const { s = t[I].x; co = t[I].y; }
};

template <int I0, int I1, class Rot, class Epi>
__device__ __forceinline__ void untangle5(const float2 (&v)[32], bool lane0, const Rot& rot,
                                          int kb_lo, int j, Epi&& epi) {
    constexpr int NC = Geo5::NC;
    static_for<I0, I1>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        // (constexpr positions: ce_pos is recursive, a runtime call would index v dynamically)
        constexpr int pe = ce_pos(16, i), po = 16 + ce_pos(16, 15 - i), pob = 16 + ce_pos(16, i);
        constexpr int per = ce_pos(16, (16 - i) & 15);
        float2 b = v[pe];
        float2 r = v[po];
        if constexpr (i < 8) {  // lane 0: O[i] with O[15 - i] (bins 32 + 64 i, NC - 32 - 64 i)
            const float2 o = v[pob];
            b.x = lane0 ? o.x : b.x;
            b.y = lane0 ? o.y : b.y;
        } else if constexpr (i == 8) {  // lane 0: E[8] with itself (bin NC/2)
            r.x = lane0 ? b.x : r.x;
            r.y = lane0 ? b.y : r.y;
        } else {  // lane 0: E[i] with E[16 - i] (bins 64 i, NC - 64 i)
            const float2 e = v[per];
            r.x = lane0 ? e.x : r.x;
            r.y = lane0 ? e.y : r.y;
        }
        float s, co;
        rot.template get<i>(s, co);
        const int k = (i < 8 ? kb_lo : j) + 64 * i;
        // realfft.rs:148-154 on the pair (Z_k, Z_{NC-k}); the 1/2 is in the window
        const float ar = b.x + r.x, ai = b.y - r.y;
        const float br = b.x - r.x, bi = b.y + r.y;
        const float p = __builtin_fmaf(co, br, s * bi);
        const float q = __builtin_fmaf(co, bi, -(s * br));
        const float x1r = ar + q, x1i = ai - p;
        float x2r = ar - q, x2i = -ai - p;
        if constexpr (i == 8) {  // lane 0's self pair: bin NC/2 is the first output only
            x2r = lane0 ? x1r : x2r;
            x2i = lane0 ? x1i : x2i;
        }
        epi(k, x1r, x1i, std::integral_constant<int, 2 * (i - I0)>{});
        epi(NC - k, x2r, x2i, std::integral_constant<int, 2 * (i - I0) + 1>{});
    });
}

// The packed mel stream (engine.cpp build_melp, kernels.hpp melp_*): the chunks of the lane's
// filters back to back, software-pipelined one chunk ahead (chunk c + 1's meta, weight and |X|
// reads are issued before chunk c's fma chain; chunk c + 1's |X| offset came with chunk c's
// meta). A chunk ends by storing its running sum at woff(c) of the region (the mel's slot, or a
// dummy slot while the filter continues) and ANDing it with keep(c): +0 after a filter's last
// chunk. The chain of each mel is mel4's k-ascending fma chain (identical bits). The frame's
// mels then leave as dB rows: one 16-byte store per lane for n_mels % 4 == 0.
static_assert(Geo5::RS == kStft5Region && Geo2<Geo5::NC>::F4 == kMelpOut, "melp region layout");
template <int S>
__device__ __forceinline__ void melp5(const StftLaunch& a, float* region, const int4* meta,
                                      const float4* wt, int j, uint64_t g, bool valid) {
    constexpr int L = Geo5::L;
    const int C = a.melp_chunks;
    char* rb = reinterpret_cast<char*>(region);
    // opaque lane index: the table addresses are formed per frame, not hoisted out of the
    // frame loop into registers held across it
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
        // keep the reads ahead of the previous chunk's chain
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
    for (; c < C; c += 2) {  // C - c even; chunk C is the tables' zero padding (read, not used)
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
    if (a.melp_v4) {
        if (4 * lj < n_mels) {
            float4 r = *reinterpret_cast<const float4*>(mo + 4 * lj);
            if (db) {
                r.x = db_of(r.x, a.log_amin, 1e-18f, 20.0f);
                r.y = db_of(r.y, a.log_amin, 1e-18f, 20.0f);
                r.z = db_of(r.z, a.log_amin, 1e-18f, 20.0f);
                r.w = db_of(r.w, a.log_amin, 1e-18f, 20.0f);
            }
            if (valid) *reinterpret_cast<float4*>(out + 4 * lj) = r;
        }
    } else {
        for (int m = lj; m < n_mels; m += L) {
            const float v = mo[m];
            if (valid) st_out(out + m, db ? db_of(v, a.log_amin, 1e-18f, 20.0f) : v);
        }
    }
}

// OK: 0 complex, 1 linear kinds, 2 mel kinds. C: 1 mono, 2 stereo (interleaved); INF: f32 / s16.
// VAR bits 18-20: the linear kind fixed at compile time (as stft3_kernel.hpp: no per-bin uniform
// branches on the kind; amp dB, the default kind, is instantiated so).
// VAR bit 0 (experiment): the register ring rotates instead of shifting -- logical point group t
// (points 8 t .. 8 t + 7 of the lane's 32) lives in physical group (t + ph) & 3, the hop's new
// samples overwrite the oldest group and ph advances (no 48 v_mov per frame pair); the first
// radix-4 level, the only reader, is compiled once per phase behind a uniform branch.
// HQ > 0: a viewer geometry with an even hop (lib.rs:43-46: 48 kHz, win 1920 / hop 480 /
// n_fft 2048: hop / 2 = 240 points = HQ 7 rows of 32 + rem 16), stft3's column rule
// (stft3_kernel.hpp): lane j keeps the points of one residue mod L of the track's point grid, so
// frame t finds them in its column jc = (j - t rem) mod L; a new frame shifts the ring by HQ rows
// where the previous column was >= rem and by HQ + 1 where it was < rem (a select per row) and
// takes HQ + 1 prefetched rows; the window row, the stage-1 twiddles and the transpose's write
// column are jc's, and from the transpose's reads on (rows A = j, B = 32 - j) the lane is j.
template <int OK, int C, int INF, int VAR = 0, int HQ = 0>
__global__ void __launch_bounds__(Geo5::BLOCK, Geo5::WV / 4)
stft5_kernel(StftLaunch a, uint64_t fps, int rs) {
    constexpr bool kRot = (VAR & 1) != 0;
    constexpr bool VIEW = HQ > 0;
    static_assert(!(VIEW && kRot), "the phase ring is for the canonical hop");
    using G = Geo5;
    using CK = Chunk<C, INF>;
    using CT = typename CK::T;
    using ET = typename std::conditional<INF == IN_S16, int16_t, float>::type;
    constexpr int NC = G::NC, P = G::P, L = G::L, FPW = G::FPW, F = G::F, SH = G::SH, S = G::S;
    constexpr int kBlock = G::BLOCK;
    constexpr bool kStage = OK == 1;  // linear kinds: LDS-staged 16-byte row stores
    constexpr int NPRE = VIEW ? HQ + 1 : SH;  // rows prefetched per frame
    constexpr int KEEP = P - NPRE;            // ring rows carried into the next frame
    static_assert(KEEP > 0, "hop shorter than the frame");

    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int kTab = G::TAB_FLOATS + (kRot ? 3 * G::TW_FLOATS : 0);
    float* wtl = lds;
    float2* twtab = reinterpret_cast<float2*>(lds + G::WL_FLOATS);
    float* work = lds + kTab;
    // mel tables: the packed stream (meta rows, then weight rows) or the rounds' chunk stream
    const bool packed = OK == 2 && a.melp_chunks > 0;
    float4* mel_lds = reinterpret_cast<float4*>(lds + kTab + G::STREAMS * rs);
    int4* pm_lds = reinterpret_cast<int4*>(mel_lds);
    float4* pw_lds = mel_lds + (packed ? (a.melp_chunks + 2) * L : 0);
    int* k0_lds = reinterpret_cast<int*>(mel_lds + (OK == 2 && !packed ? a.mel4_rows * L : 0));
    int2* rd_lds = reinterpret_cast<int2*>(k0_lds + (OK == 2 && !packed ? a.mel4_rounds * L : 0));
    int* xo_lds = reinterpret_cast<int*>(rd_lds + (OK == 2 && !packed ? a.mel4_rounds : 0));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slot = lane / L, j = lane % L;
    const bool lane0 = j == 0;
    const int jb = (L - j) & (L - 1);  // the partner column B

    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) {  // w/2 is exact (realfft's 1/2)
        const int m = i >> 1, jj = m % L, n1 = m / L;
        wtl[jj * G::WL_STRIDE + 2 * n1 + (i & 1)] = a.wpad[i] * 0.5f;
    }
    if (packed) {
        for (int i = threadIdx.x; i < (a.melp_chunks + 2) * L; i += kBlock) pm_lds[i] = a.melp_meta[i];
        const int nw = (a.melp_chunks + 1) * a.melp_steps * L;
        for (int i = threadIdx.x; i < nw; i += kBlock) pw_lds[i] = a.melp_wt[i];
    } else if constexpr (OK == 2) {
        const int nw = a.mel4_rows * L;
        for (int i = threadIdx.x; i < nw; i += kBlock) mel_lds[i] = a.mel4_wt[i];
        for (int i = threadIdx.x; i < a.mel4_rounds * L; i += kBlock) k0_lds[i] = a.mel4_k0[i];
        for (int i = threadIdx.x; i < a.mel4_rounds; i += kBlock) rd_lds[i] = a.mel4_round[i];
        for (int i = threadIdx.x; i < a.mel_chunks * L; i += kBlock) xo_lds[i] = a.mel_xo[i];
    }
    // stage-1 twiddles with k1 pairs interleaved: [k1/2][j][k1&1]; kRot: one table per ring
    // phase ph, the entries times i^(ph k1) (exact: a swap and negations)
    for (int i = threadIdx.x; i < (kRot ? 4 : 1) * P * L; i += kBlock) {
        const int phi = i / (P * L), ii = i % (P * L), k1 = ii / L, jj = ii % L;
        float2 t = a.tw3[ii];
        const int r = (phi * k1) & 3;
        if (r == 1) t = make_float2(-t.y, t.x);
        else if (r == 2) t = make_float2(-t.x, -t.y);
        else if (r == 3) t = make_float2(t.y, -t.x);
        twtab[phi * P * L + ((k1 >> 1) * L + jj) * 2 + (k1 & 1)] = t;
    }
    // untangle bases: slots 0..7 start at bin kb_lo (lane 0: 32), slots 8..15 at bin j
    float2 ub_lo = a.sincos[lane0 ? 32 : j], ub_hi = a.sincos[j];
    float2 sct[16];
    static_for<0, 16>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        rot16<i>(i < 8 ? ub_lo : ub_hi, sct[i].x, sct[i].y);
    });
    const RotTable rot{sct};
    const int kb_lo = lane0 ? 32 : j;
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t stream = ((uint64_t)blockIdx.x * G::WV + wave) * FPW + slot;
    using FI = uint64_t;
    using SI = int64_t;
    const FI g0 = (FI)(stream * fps);
    const FI g1 = (FI)(stream * fps + fps < total ? stream * fps + fps : total);
    const int hop = a.hop;
    float* region = work + (wave * FPW + slot) * rs;
    const ET* in = static_cast<const ET*>(a.in);

    float2 raw[P];
    CT pre[NPRE];
    const int rem = VIEW ? (hop >> 1) & (L - 1) : 0;
    bool pre_ok = false;
    int ph = 0;  // kRot: physical group of logical group 0 (wave-uniform)
    int hint = -1;
    FI g_beg = 1, g_end = 0;
    uint64_t base = 0;
    SI n = 0;
#ifdef THESIA_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
    for (uint64_t it = 0; it < fps; ++it) {  // wave-uniform trip count
        // wave priority phases (stft3): loads / window / FFT at 0, untangle / |X|
        // / mel / stores at 2
        __builtin_amdgcn_s_setprio(0);
        MARK5(top, 7);
        const FI g = g0 + (FI)it;
        const bool valid = g < g1;
        // opaque per frame: keeps the per-lane offsets (window row, transpose rows, untangle
        // bins) inside the loop instead of hoisted as loop invariants into dozens of VGPRs
        int wj = j, wjb = jb, wkb = kb_lo;
        asm volatile("" : "+v"(wj), "+v"(wjb), "+v"(wkb));
        SI start = 0;
        if (valid) {
            if (g >= g_end || g < g_beg) {
                hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
                g_beg = (FI)a.trk_frame0[hint];
                g_end = (FI)a.trk_frame0[hint + 1];
                n = (SI)a.trk_len[hint];
                base = a.trk_in_off[hint];
            }
            start = (SI)(g - g_beg) * hop - NC;  // half_win = NC, pad_left = 0
        }
        // the frame's column (HQ > 0): (j - frame start in points) mod L; window, twiddles and
        // the transpose's write column follow it
        int jc = j, wc = wj;  // (canonical geometry: the opaque wj, no further register)
        if constexpr (VIEW) {
            if (valid) jc = (j - (int)((start >> 1) & (L - 1))) & (L - 1);
            wc = jc;
            asm volatile("" : "+v"(wc));
        }
        // ---- the frame's raw samples: shift by SH points + the prefetched hop ----
        if (pre_ok && kRot) {
            // the oldest group takes the new hop; the ring's origin moves one group on
            static_assert(!kRot || P == 4 * SH, "phase ring: four groups of one hop");
            const int p0 = __builtin_amdgcn_readfirstlane(ph);
            auto ins = [&](auto gc) {
                constexpr int gi = decltype(gc)::value;
#pragma unroll
                for (int q = 0; q < SH; ++q) raw[gi * SH + q] = CK::mix(pre[q]);
            };
            if (p0 == 0) ins(std::integral_constant<int, 0>{});
            else if (p0 == 1) ins(std::integral_constant<int, 1>{});
            else if (p0 == 2) ins(std::integral_constant<int, 2>{});
            else ins(std::integral_constant<int, 3>{});
            ph = (p0 + 1) & 3;
        } else if (pre_ok) {
            if constexpr (VIEW) {
                const bool up = ((jc + rem) & (L - 1)) < rem;  // the previous column < rem
#pragma unroll
                for (int n1 = 0; n1 < KEEP; ++n1) {
                    raw[n1].x = up ? raw[n1 + HQ + 1].x : raw[n1 + HQ].x;
                    raw[n1].y = up ? raw[n1 + HQ + 1].y : raw[n1 + HQ].y;
                }
            } else {
#pragma unroll
                for (int n1 = 0; n1 < KEEP; ++n1) raw[n1] = raw[n1 + SH];
            }
#pragma unroll
            for (int q = 0; q < NPRE; ++q) raw[KEEP + q] = CK::mix(pre[q]);
        } else if (valid && start >= 0 && start + 2 * NC <= n && ((base + (uint64_t)start * C) % (2 * C)) == 0) {
            const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)start * C) + jc;
            static_for<0, P / 8>([&](auto gc) {
                constexpr int g8 = decltype(gc)::value;
                static_for<0, 8>([&](auto ic) {
                    constexpr int n1 = 8 * g8 + decltype(ic)::value;
                    raw[n1] = CK::mix(src[L * n1]);
                });
                pin_range<8 * g8, 8 * g8 + 8>(raw);
            });
        } else if (valid) {
            load_raw_generic_ool<NC, INF>(a, region, jc, start, n, base, C, a.fold != 0, raw);
        } else {
#pragma unroll
            for (int n1 = 0; n1 < P; ++n1) raw[n1] = make_float2(0.f, 0.f);
        }
        if (!(pre_ok && kRot)) ph = 0;  // a reloaded ring is in logical order
        MARK5(loaded, 0);
        const float4* wrow = reinterpret_cast<const float4*>(wtl + wc * G::WL_STRIDE);
        // ---- prefetch the next frame's hop of new samples (its points P-SH .. P-1) right
        // away: a whole frame to land, as stft3 ----
        auto prefetch = [&]() {
            const SI nstart = start + hop;
            const bool nxt = valid && g + 1 < g1 && g + 1 < g_end && nstart + 2 * NC <= n &&
                             nstart + 2 * L * KEEP >= 0 &&
                             ((base + (uint64_t)(nstart + 2 * L * KEEP) * C) % (2 * C)) == 0;
            if (nxt) {
                const int jn = (jc - rem) & (L - 1);  // the next frame's column (= j unless HQ > 0)
                const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)(nstart + 2 * L * KEEP) * C) + jn;
#pragma unroll
                for (int q = 0; q < NPRE; ++q) pre[q] = src[L * q];
            }
            pre_ok = nxt;
        };
        prefetch();
        // ---- stage 1: DFT-32 over n1, twiddles W_NC^{j k1} ----
        // window (lib.rs:379, with the 1/2 of realfft.rs:148-154 folded in) inside the first
        // radix-4 level of the DFT-32 (dif_fft's N = 32 level): the products of inputs 2 and 3
        // are formed once and the ones of inputs 0 and 1 ride in the butterfly fmas (12 VALU per
        // butterfly instead of 16)
        float2 v[P];
        // kRot: the DFT-32 runs over the ring in PHYSICAL order, the window of each physical
        // group read from its logical row ((g - ph) & 3); the result is the DFT of the frame
        // rotated by 8 ph points, i.e. Y[k1] (-i)^(ph k1), undone exactly by the stage-1
        // twiddle table of phase ph (W^{j k1} i^(ph k1): a swap / negation of the entries)
        const int phs = kRot ? __builtin_amdgcn_readfirstlane(ph) : 0;
        const float4* wg[4] = {wrow + 4 * ((0 - phs) & 3), wrow + 4 * ((1 - phs) & 3),
                               wrow + 4 * ((2 - phs) & 3), wrow + 4 * ((3 - phs) & 3)};
        {
        static_for<0, 4>([&](auto jc) {
            constexpr int jp = decltype(jc)::value;
            const float4 wq[4] = {wg[0][jp], wg[1][jp], wg[2][jp], wg[3][jp]};
            static_for<0, 2>([&](auto hc) {
                constexpr int h = decltype(hc)::value, jj = 2 * jp + h;
                auto wv = [&](int t) {
                    return h == 0 ? make_float2(wq[t].x, wq[t].y) : make_float2(wq[t].z, wq[t].w);
                };
                const float2 w0 = wv(0), w1 = wv(1), w2 = wv(2), w3 = wv(3);
                const float2 a0 = raw[jj], a1 = raw[jj + 8], a2 = raw[jj + 16], a3 = raw[jj + 24];
                const float2 m2 = make_float2(a2.x * w2.x, a2.y * w2.y);
                const float2 m3 = make_float2(a3.x * w3.x, a3.y * w3.y);
                const float2 t0 = make_float2(__builtin_fmaf(a0.x, w0.x, m2.x), __builtin_fmaf(a0.y, w0.y, m2.y));
                const float2 t1 = make_float2(__builtin_fmaf(a0.x, w0.x, -m2.x), __builtin_fmaf(a0.y, w0.y, -m2.y));
                const float2 t2 = make_float2(__builtin_fmaf(a1.x, w1.x, m3.x), __builtin_fmaf(a1.y, w1.y, m3.y));
                const float2 t3 = mul_negi(make_float2(__builtin_fmaf(a1.x, w1.x, -m3.x), __builtin_fmaf(a1.y, w1.y, -m3.y)));
                v[jj] = cadd(t0, t2);
                v[jj + 8] = twc<32, jj>(cadd(t1, t3));
                v[jj + 16] = twc<32, 2 * jj>(csub(t0, t2));
                v[jj + 24] = twc<32, 3 * jj>(csub(t1, t3));
            });
        });
        }
        pin(v);
        dif_fft<8, 1, 0, P>(v);
        dif_fft<8, 1, 8, P>(v);
        dif_fft<8, 1, 16, P>(v);
        dif_fft<8, 1, 24, P>(v);
        pin(v);
        MARK5(stage1, 1);
        {
            const float4* tp = reinterpret_cast<const float4*>(twtab) + wc + phs * (P / 2 * L);
            static_for<0, P / 2 / G::TWC>([&](auto cc) {
                constexpr int c0 = decltype(cc)::value * G::TWC;
                __builtin_amdgcn_sched_barrier(0);
                float4 tw[G::TWC];
                static_for<0, G::TWC>([&](auto uc) { tw[decltype(uc)::value] = tp[(c0 + decltype(uc)::value) * L]; });
                static_for<0, G::TWC>([&](auto uc) {
                    constexpr int q = c0 + decltype(uc)::value;
                    if constexpr (q > 0) {
                        constexpr int pk0 = ce_pos(P, 2 * q);
                        v[pk0] = cmul(v[pk0], make_float2(tw[decltype(uc)::value].x, tw[decltype(uc)::value].y));
                    }
                    constexpr int pk1 = ce_pos(P, 2 * q + 1);
                    v[pk1] = cmul(v[pk1], make_float2(tw[decltype(uc)::value].z, tw[decltype(uc)::value].w));
                });
            });
        }
        MARK5(twiddled, 2);
        // ---- transpose (re, then im): rows A = j and B = 32 - j, first radix-2 step ----
        // v[n] <- A[n] + A[n + 16]; v[16 + n] <- B[n] - B[n + 16] (n < 16)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            wave_lds_sync();
            static_for<0, P>([&](auto kc) {
                constexpr int k1 = decltype(kc)::value;
                constexpr int pk = ce_pos(P, k1);
                region[k1 * S + wc] = e == 0 ? v[pk].x : v[pk].y;
            });
            wave_lds_sync();
            // row A lands in the component just written out: A[n] into v[n].e (e = re / im;
            // explicit branches on the unrolled e: a reference select would put v in scratch)
            const float4* ra = static_cast<const float4*>(__builtin_assume_aligned(region + wj * S, 16));
            const float4* rb = static_cast<const float4*>(__builtin_assume_aligned(region + wjb * S, 16));
            auto put = [&](float2& x, float val) {
                if (e == 0) x.x = val; else x.y = val;
            };
            auto get = [&](const float2& x) { return e == 0 ? x.x : x.y; };
            static_for<0, 8>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const float4 t = ra[q];
                put(v[4 * q], t.x); put(v[4 * q + 1], t.y); put(v[4 * q + 2], t.z); put(v[4 * q + 3], t.w);
            });
            static_for<0, 16>([&](auto nc) {  // even outputs of A: A[n] + A[n + 16]
                constexpr int nn = decltype(nc)::value;
                put(v[nn], get(v[nn]) + get(v[nn + 16]));
            });
            // row B: v[16 + n].e = B[n] - B[n + 16]
            {
                float4 xb[8];
                static_for<0, 4>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    xb[q] = rb[q];
                    xb[4 + q] = rb[q + 4];
                });
                static_for<0, 4>([&](auto uc) {
                    constexpr int u = decltype(uc)::value, n0 = 4 * u;
                    put(v[16 + n0], xb[u].x - xb[u + 4].x);
                    put(v[17 + n0], xb[u].y - xb[u + 4].y);
                    put(v[18 + n0], xb[u].z - xb[u + 4].z);
                    put(v[19 + n0], xb[u].w - xb[u + 4].w);
                });
            }
        }
        wave_lds_sync();
        MARK5(transposed, 3);
        MARK5(prefetched, 4);
        // ---- stage 2: W_32^n on B's differences, then the two DFT-16s ----
        static_for<1, 16>([&](auto nc) {
            constexpr int nn = decltype(nc)::value;
            v[16 + nn] = twc<32, nn>(v[16 + nn]);
        });
        pin(v);
        dif_fft<16, 1, 0, P>(v);
        dif_fft<16, 1, 16, P>(v);
        pin(v);
        __builtin_amdgcn_s_setprio(2);
        MARK5(stage2, 5);
        if constexpr (OK == 2) {
            // |X| (lib.rs:124) per half frame: the |X|^2 of 16 bins, their v_sqrt, the row writes
            auto half = [&](auto h0) {
                constexpr int I0 = decltype(h0)::value;
                float mag[16];
                untangle5<I0, I0 + 8>(v, lane0, rot, wkb, wj, [&](int, float xr, float xi, auto sc) {
                    mag[decltype(sc)::value] = __builtin_fmaf(xr, xr, xi * xi);
                });
                pin_f(mag);
#pragma unroll
                for (int i = 0; i < 16; ++i) mag[i] = __builtin_amdgcn_sqrtf(mag[i]);
                pin_f(mag);
                float* lo = region + wkb;      // bins kb + 64 i (slots < 8; wkb = j for j > 0)
                float* hi = region + (NC - wj); // bins NC - j - 64 i
                float* lo0 = region + NC - wkb;
                static_for<0, 8>([&](auto ic) {
                    constexpr int i = I0 + decltype(ic)::value;
                    if constexpr (i < 8) {
                        lo[64 * i] = mag[2 * (i - I0)];
                        lo0[-64 * i] = mag[2 * (i - I0) + 1];
                    } else {
                        region[wj + 64 * i] = mag[2 * (i - I0)];
                        hi[-64 * i] = mag[2 * (i - I0) + 1];
                    }
                });
            };
            half(std::integral_constant<int, 0>{});
            half(std::integral_constant<int, 8>{});
            if (lane0) {  // E[0] with itself: bins 0 and NC (s = 0, co = 1)
                const float2 e0 = v[0];
                const float ar = e0.x + e0.x, bi = e0.y + e0.y, x0 = ar + bi, xn = ar - bi;
                region[0] = __builtin_amdgcn_sqrtf(__builtin_fmaf(x0, x0, 0.0f));
                region[NC] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xn, xn, 0.0f));
#pragma unroll
                for (int k = F; k < Geo2<NC>::F4; ++k) region[k] = 0.0f;
            }
            wave_lds_sync();
            MARK5(untangled, 6);
            if (packed) {
                if (a.melp_steps == 2) melp5<2>(a, region, pm_lds, pw_lds, j, g, valid);
                else melp5<3>(a, region, pm_lds, pw_lds, j, g, valid);
            }
#ifndef THESIA_MELP_ONLY
            else if (a.mel_chunks == 8) mel4p<NC, 8>(a, region, mel_lds, xo_lds, j, g, valid);
            else if (a.mel_chunks == 4) mel4p<NC, 4>(a, region, mel_lds, xo_lds, j, g, valid);
            else mel4<NC, 8, 1>(a, region, mel_lds, rd_lds, k0_lds, j, g, valid);
#endif
        } else if constexpr (OK == 0) {  // lane-wise 8-byte stores
            float2* crow = reinterpret_cast<float2*>(a.out) + g * F;
            auto st = [&](int k, float xr, float xi, auto) {
                if (valid) st_out(crow + k, make_float2(xr, xi));
            };
            untangle5<0, 16>(v, lane0, rot, wkb, wj, st);
            if (lane0 && valid) {
                const float2 e0 = v[0];
                const float ar = e0.x + e0.x, bi = e0.y + e0.y;
                st_out(crow, make_float2(ar + bi, 0.0f));
                st_out(crow + NC, make_float2(ar - bi, 0.0f));
            }
        } else {
            static_assert(kStage, "linear kinds stage their rows");
            constexpr int KD = (VAR >> 18) & 7;  // the kind fixed at compile time (0: run time)
            float* frow = static_cast<float*>(a.out) + g * F;
            const int sh = (int)((reinterpret_cast<uintptr_t>(frow) >> 2) & 3);
            float* stg = region + sh;
            // the row for kind K (compile time: no per-bin branches); the run-time kind switches
            // once per frame
            auto rows = [&](auto kc) {
                constexpr int K = decltype(kc)::value;
                constexpr bool power = K == OUT_POWER || K == OUT_POWER_DB;
                constexpr bool db = K == OUT_AMP_DB || K == OUT_POWER_DB;
                auto val_of = [&](float xr, float xi) {
                    const float p2 = __builtin_fmaf(xr, xr, xi * xi);
                    // amp dB from |X|^2 (amp_db_of: no v_sqrt); amp / power as is
                    return db ? (power ? db_of(p2, a.log_amin, 1e-36f, 10.0f) : amp_db_of(p2, a.log_amin))
                              : (power ? p2 : __builtin_amdgcn_sqrtf(p2));
                };
                untangle5<0, 16>(v, lane0, rot, wkb, wj, [&](int k, float xr, float xi, auto) {
                    stg[k] = val_of(xr, xi);
                });
                if (lane0) {
                    const float2 e0 = v[0];
                    const float ar = e0.x + e0.x, bi = e0.y + e0.y;
                    stg[0] = val_of(ar + bi, 0.0f);
                    stg[NC] = val_of(ar - bi, 0.0f);
                }
            };
            if constexpr (KD != 0) {
                rows(std::integral_constant<int, KD>{});
            } else {
                switch (a.out_kind) {
                    case OUT_MAG: rows(std::integral_constant<int, OUT_MAG>{}); break;
                    case OUT_POWER: rows(std::integral_constant<int, OUT_POWER>{}); break;
                    case OUT_AMP_DB: rows(std::integral_constant<int, OUT_AMP_DB>{}); break;
                    default: rows(std::integral_constant<int, OUT_POWER_DB>{}); break;
                }
            }
            wave_lds_sync();
            if (valid) store_row_b128<L>(frow, sh, region, F, j);
        }
    }
#ifdef THESIA_STAMPS
    MARK5(end, 7);
    if (a.stamps && lane == 0) {  // vector stores (lane-indexed address)
        unsigned long long* o = a.stamps + ((uint64_t)blockIdx.x * G::WV + wave) * 9 + lane;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = st_acc[i];
        o[8] = fps;
    }
#endif
}

// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
template <int OK, int VAR = 0>
static int lds5_bytes(const StftLaunch& a, int rs) {
    const int mel = OK != 2 ? 0
                    : a.melp_chunks > 0 ? ((a.melp_chunks + 2) + (a.melp_chunks + 1) * a.melp_steps) * Geo5::L * 4
                    : (a.mel4_rows * 4 + a.mel4_rounds + a.mel_chunks) * Geo5::L + 2 * a.mel4_rounds;
    const int tab = Geo5::TAB_FLOATS + ((VAR & 1) ? 3 * Geo5::TW_FLOATS : 0);
    return (tab + Geo5::STREAMS * rs + mel) * 4;
}
template <int OK, int VAR = 0>
static int region_stride5(const StftLaunch& a) {
    // the packed mel stream stages the frame's mels behind the |X| row: full regions only
    if (OK == 2 && a.melp_chunks > 0) return Geo5::RS;
    return lds5_bytes<OK, VAR>(a, Geo5::RS) <= 163840 ? Geo5::RS : Geo5::RS_MIN;
}

template <int OK, int C, int INF, int VAR = 0, int HQ = 0>
static int launch5_k(const StftLaunch& a, hipStream_t stream) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (VAR == 0 && C == 2 && INF == IN_F32) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        if (e && atoi(e) == 1) return launch5_k<OK, C, INF, 1>(a, stream);  // phase ring
    }
#endif
    const int rs = region_stride5<OK, VAR>(a);
    const int lds = lds5_bytes<OK, VAR>(a, rs);
    if (lds > 163840) return -2;
    auto kern = stft5_kernel<OK, C, INF, VAR, HQ>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    constexpr uint64_t per_block = Geo5::STREAMS;
    int grid = grid_for(reinterpret_cast<const void*>(kern), Geo5::BLOCK, lds,
                        (a.total_frames + per_block - 1) / per_block, a.grid, a.grid_share);
    const uint64_t streams = (uint64_t)grid * per_block;
    const uint64_t fps = (a.total_frames + streams - 1) / streams;
    grid = (int)((a.total_frames + fps * per_block - 1) / (fps * per_block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(Geo5::BLOCK), lds, stream, a, fps, rs);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the viewer geometry (HQ 7: hop 480, win <= 2048) for the mel and linear kinds (complex rows
// stay on stft3, which is faster for them)
static bool view5(const StftLaunch& a) { return !(a.win == 2048 && a.hop * 4 == 2048); }
template <int C, int INF>
static int launch5_c(const StftLaunch& a, hipStream_t s) {
    const bool mel = a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB;
    bool fixed = a.out_kind == OUT_AMP_DB;  // amp dB rows: the kind at compile time
#ifdef THESIA_EXPERIMENTS
    if (getenv("THESIA_STFT3_RTKIND")) fixed = false;  // A/B: the run-time kind
#endif
    constexpr int KDB = OUT_AMP_DB << 18;
    if (view5(a)) {
        if (a.out_kind == OUT_COMPLEX) return -2;
        if (mel) return launch5_k<2, C, INF, 0, 7>(a, s);
        return fixed ? launch5_k<1, C, INF, KDB, 7>(a, s) : launch5_k<1, C, INF, 0, 7>(a, s);
    }
    if (a.out_kind == OUT_COMPLEX) return launch5_k<0, C, INF>(a, s);
    if (mel) return launch5_k<2, C, INF>(a, s);
    return fixed ? launch5_k<1, C, INF, KDB>(a, s) : launch5_k<1, C, INF>(a, s);
}

int stft5_lds_bytes(const StftLaunch& a) {
    const bool mel = a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB;
    return a.out_kind == OUT_COMPLEX ? lds5_bytes<0>(a, region_stride5<0>(a))
           : mel ? lds5_bytes<2>(a, region_stride5<2>(a)) : lds5_bytes<1>(a, region_stride5<1>(a));
}

bool stft5_supports(int n_fft, int win, int hop, int in_format, int channels) {
    // the canonical geometry, or the 48 kHz viewer one (hop / 2 = 7 rows of 32 + 16; an even win
    // <= n_fft, as the streaming start rule needs, stft3v_kernels.hip)
    const bool canon = win == n_fft && hop * 4 == n_fft;
    const bool view = hop % 2 == 0 && (hop / 2) / 32 == 7 && win <= n_fft && win % 2 == 0 && win >= 2;
    return n_fft == 2048 && (canon || view) && (in_format == IN_F32 || in_format == IN_S16) &&
           (channels == 1 || channels == 2);
}

int launch_stft5(const StftLaunch& a, hipStream_t s) {
    if (a.n_fft != 2048) return -2;
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch5_c<2, IN_S16>(a, s) : launch5_c<1, IN_S16>(a, s);
    return a.channels == 2 ? launch5_c<2, IN_F32>(a, s) : launch5_c<1, IN_F32>(a, s);
}

}  // namespace thesia
