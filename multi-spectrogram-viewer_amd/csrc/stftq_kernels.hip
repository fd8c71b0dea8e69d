// stftq_kernels.hip -- the reference-order STREAMING STFT for n_fft 256 / 512 / 1024 (batch kernel
// 7 with stftr_kernels.hip's n_fft 2048): every f32 operation of the reference path in the
// reference's order, as stftx_kernel, so the rows equal the oracle's bit for bit, with the
// streaming data movement of the fast kernels (win = n_fft, hop = n_fft / 4: the C5 geometry).
//
// A frame is held by L lanes x P registers: lane l, register n hold the complex point m = l + L n
// (the ring layout: a hop moves P / 4 registers and loads only its new samples). rustfft 4.0
// Radix4 (oracle cfft_tab; prepare_radix4 puts point m at p = m's base-4 digits reversed, with a
// base-8 digit on top of m when log2(NC) is odd) takes m's digits from the top: the base level
// (butterfly_4 or butterfly_8) over the digit already in register bits, then one radix-4 level per
// lower digit with the table twiddles tw[j t NC / cur], j = p mod (cur / 4). Before a level whose
// digit sits in lane bits, each of its bits is swapped with a register bit that is not part of it
// (a lane-bit <-> register-bit swap: DPP quad_perm for lane bits 0 / 1, ds_bpermute for bit 2, DPP
// row_ror:8 for bit 3, v_permlane16_swap for bit 4). The schedule (qsched below) is the rule of
// tests/stftq_model.py, which checks it against the oracle bit for bit on the CPU.
//
//   NC    L x P     levels (m bits)                       swaps
//   128   16 x 8    b8(4-6), r4(2,3), r4(0,1)             2 before each radix-4 level
//   256   16 x 16   r4(6,7), r4(4,5), r4(2,3), r4(0,1)    2 before each of the last two
//   512   32 x 16   b8(6-8), r4(4,5), r4(2,3), r4(0,1)    1 (permlane16), 2, 2
//
// (The swaps other than permlane16 run as one LDS round trip of the frame's points, at
// bank-conflict-free swizzled places: SwzQ below.) Then Z[p] goes to the frame's LDS region (bin p
// at its swizzled place), each lane untangles the pairs
// (k, NC - k), k = l + L i (realfft.rs:142-157 as stftx), and the row leaves through the region
// as aligned 16-byte stores (|X| by the correctly rounded hypot, dB by glibc's log10f; mel as the
// k-ascending fma chain over each filter's band, as stftx).
#include "stft3_core.hpp"
#include "stftr_core.hpp"

#include <cstdlib>
#include <type_traits>

namespace thesia {

template <int NC>
struct GeoQ {
    static constexpr int L = NC == 512 ? 32 : 16;
    static constexpr int P = NC / L, FPW = 64 / L, F = NC + 1, SH = P / 4, KEEP = P - SH;
    static constexpr int B = NC == 128 ? 7 : NC == 256 ? 8 : 9;
    static constexpr int NL = L == 16 ? 4 : 5, NR = P == 8 ? 3 : 4;
    static constexpr int NLEV = (B % 2) ? 1 + (B - 3) / 2 : B / 2;
    // (the tables padded to 128-byte multiples: the frame regions after them start 128-byte
    // aligned, which the swizzled accesses below need)
    static constexpr int WL_STRIDE = 2 * P + 4, WL_FLOATS = (L * WL_STRIDE + 31) / 32 * 32;
    static constexpr int TW_FLOATS = 2 * (NC + NC / 32), SC_FLOATS = 2 * NC + 4;  // twiddles: tpad
    static constexpr int LOGT_FLOATS = 64;  // logf's table (exact_math.hpp kLogfT), LDS copy
    static constexpr int TAB_FLOATS = (WL_FLOATS + TW_FLOATS + SC_FLOATS + LOGT_FLOATS + 31) / 32 * 32;
    // a frame's region: the relayouts and the Z row (NC float2 at swizzled places; the untangle's
    // partner read of lane 0 at i = 0, whose value is not used, may reach NC + 15), later the staged
    // row (complex: 2F floats from sh <= 3, 16 floats further in the odd frame slots of a 16-lane
    // layout). The stride is 32 mod 64 dwords: a 32-lane LDS read spans two 16-lane frame slots,
    // which then fall on the two halves of the 64 banks.
    static constexpr int RS_NEED0 = 2 * F + 3 + (L == 16 ? 16 : 0), RS_NEED1 = 2 * NC + 32;
    static constexpr int RS_NEED = RS_NEED0 > RS_NEED1 ? RS_NEED0 : RS_NEED1;
    static constexpr int RS = (RS_NEED + 31) / 64 * 64 + 32;
    static_assert(L * P == NC && (1 << NL) == L && (1 << NR) == P && P % 4 == 0, "geometry");
    static_assert(RS >= RS_NEED && RS % 64 == 32 && TAB_FLOATS % 32 == 0 && WL_FLOATS % 32 == 0, "region");
};

struct QLev {
    int nd = 0;                       // digit bits: 2 (radix 4) or 3 (the radix-8 base)
    int dig[3] = {0, 0, 0};           // the digit's m bits, LSB first
    int nsw = 0;                      // lane bit <-> register bit swaps before the level
    int swx[3] = {0, 0, 0}, swy[3] = {0, 0, 0};
    int kind[10] = {}, bit[10] = {};  // m bit -> lane (0) / register (1) bit, after the swaps
    int pstart = 0;                   // the digit's lowest bit in p: j = p mod 2^pstart
};
struct QSched {
    QLev lev[5];
    int pbit[10] = {};  // m bit -> its bit in p
};

// tests/stftq_model.py schedule(): the digits from the top of m, each lane bit of a digit swapped
// with the lowest register bit holding none of the digit's bits
template <int NC>
constexpr QSched make_qsched() {
    using G = GeoQ<NC>;
    QSched s{};
    int dig[5][3] = {}, nd[5] = {}, n = 0;
    if (G::B % 2) {
        nd[0] = 3;
        dig[0][0] = G::B - 3;
        dig[0][1] = G::B - 2;
        dig[0][2] = G::B - 1;
        n = 1;
        for (int i = (G::B - 3) / 2 - 1; i >= 0; --i, ++n) {
            nd[n] = 2;
            dig[n][0] = 2 * i;
            dig[n][1] = 2 * i + 1;
        }
    } else {
        for (int i = G::B / 2 - 1; i >= 0; --i, ++n) {
            nd[n] = 2;
            dig[n][0] = 2 * i;
            dig[n][1] = 2 * i + 1;
        }
    }
    int pos = 0;
    for (int t = 0; t < n; ++t) {
        for (int c = 0; c < nd[t]; ++c) s.pbit[dig[t][c]] = pos + c;
        pos += nd[t];
    }
    int kind[10] = {}, bit[10] = {};
    for (int b = 0; b < G::B; ++b) {
        kind[b] = b < G::NL ? 0 : 1;
        bit[b] = b < G::NL ? b : b - G::NL;
    }
    for (int t = 0; t < n; ++t) {
        QLev& q = s.lev[t];
        q.nd = nd[t];
        int ps = 99;
        for (int c = 0; c < nd[t]; ++c) {
            q.dig[c] = dig[t][c];
            ps = s.pbit[dig[t][c]] < ps ? s.pbit[dig[t][c]] : ps;
        }
        q.pstart = ps;
        for (int c = 0; c < nd[t]; ++c) {
            const int b = dig[t][c];
            if (kind[b] != 0) continue;
            const int x = bit[b];
            int y = -1;
            for (int r = 0; r < G::NR && y < 0; ++r) {
                bool used = false;
                for (int cc = 0; cc < nd[t]; ++cc)
                    if (kind[dig[t][cc]] == 1 && bit[dig[t][cc]] == r) used = true;
                if (!used) y = r;
            }
            int other = -1;
            for (int bb = 0; bb < G::B; ++bb)
                if (kind[bb] == 1 && bit[bb] == y) other = bb;
            kind[b] = 1;
            bit[b] = y;
            kind[other] = 0;
            bit[other] = x;
            q.swx[q.nsw] = x;
            q.swy[q.nsw] = y;
            ++q.nsw;
        }
        for (int b = 0; b < G::B; ++b) {
            q.kind[b] = kind[b];
            q.bit[b] = bit[b];
        }
    }
    return s;
}

template <int NC>
struct QS {
    static constexpr QSched S = make_qsched<NC>();
};

namespace {

// a lane's value from lane ^ (1 << X) of its 16-lane row (X <= 3)
template <int X>
__device__ __forceinline__ float xlane(float v) {
    if constexpr (X == 2) {
        return __shfl_xor(v, 4, 64);
    } else {
        constexpr int ctrl = X == 0 ? 0xB1 : X == 1 ? 0x4E : 0x128;  // quad_perm / row_ror:8
        return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xF, 0xF, false));
    }
}

// lane bit X <-> register bit Y: the point at (lane bit u, register bit w) moves to (w, u)
template <int X, int Y, int P>
__device__ __forceinline__ void qswap(float2 (&v)[P], int lj) {
    if constexpr (X == 4) {
        static_for<0, P>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr (((r >> Y) & 1) == 0) pl16(v[r], v[r | (1 << Y)]);
        });
    } else {
        const unsigned hi = ((lj >> X) & 1) ? ~0u : 0u;
        static_for<0, P>([&](auto rc) {
            constexpr int r = decltype(rc)::value, r1 = r | (1 << Y);
            if constexpr (((r >> Y) & 1) == 0) {
                const float2 a = v[r], b = v[r1];
                const float2 send = bsel2(hi, a, b);
                const float2 recv = make_float2(xlane<X>(send.x), xlane<X>(send.y));
                v[r] = bsel2(hi, recv, a);
                v[r1] = bsel2(hi, b, recv);
            }
        });
    }
}

// The layout of a level's input (T > 0: the previous level's, after its swaps; T = 0: point m =
// lane + L register) and of its own (after its swaps): the point index m held at (lane, register)
// is lane_mbits + reg_mbits (disjoint bits).
template <int NC, int T, bool NEW>
__device__ __forceinline__ int lane_mbits(int lj) {
    using G = GeoQ<NC>;
    int m = 0;
    static_for<0, G::B>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        constexpr bool init = !NEW && T == 0;
        constexpr int kind = init ? (b < G::NL ? 0 : 1) : QS<NC>::S.lev[NEW ? T : T - 1].kind[b];
        constexpr int bit = init ? (b < G::NL ? b : b - G::NL) : QS<NC>::S.lev[NEW ? T : T - 1].bit[b];
        if constexpr (kind == 0) m |= ((lj >> bit) & 1) << b;
    });
    return m;
}
template <int NC, int T, bool NEW>
constexpr int reg_mbits(int r) {
    using G = GeoQ<NC>;
    int m = 0;
    for (int b = 0; b < G::B; ++b) {
        const bool init = !NEW && T == 0;
        const int kind = init ? (b < G::NL ? 0 : 1) : QS<NC>::S.lev[NEW ? T : T - 1].kind[b];
        const int bit = init ? (b < G::NL ? b : b - G::NL) : QS<NC>::S.lev[NEW ? T : T - 1].bit[b];
        if (kind == 1) m |= ((r >> bit) & 1) << b;
    }
    return m;
}
// LDS swizzles (round 6). The frame's points sit in its region at index
// x ^ G(x >> 4) (float2 units): a GF(2)-linear map of the index's bits >= 4 onto its bits 0-3,
// one 4-bit image per bit (REL: the relayouts' point index m; Z: the Z row's bin p). The images
// (scratch search over the rule) make every relayout's write (ds_write_b64: 16-lane groups,
// banks mod 32) and read (ds_read_b64: 32-lane groups, banks mod 64, two 16-lane frame slots RS
// apart) and the Z row's write conflict-free (round 5's one-float2-per-16 padding left them
// 2-8-way; no integer padding can serve n_fft 256's three layouts at once). Linear:
// swz(a ^ b) = swz(a) ^ swz(b) for disjoint bits, so an access is a per-lane byte base (128-byte
// aligned region + 8 swz(lane part)) XOR a compile-time constant (8 x the register part's bits
// 0-3) plus an immediate offset (its bits >= 4).
template <int NC> struct SwzQ;
template <> struct SwzQ<128> {
    static constexpr int REL[5] = {5, 10, 0, 0, 0}, Z[5] = {4, 0, 0, 0, 0};
};
template <> struct SwzQ<256> {
    static constexpr int REL[5] = {5, 10, 0, 0, 0}, Z[5] = {1, 2, 0, 0, 0};
};
template <> struct SwzQ<512> {
    static constexpr int REL[5] = {4, 9, 6, 0, 0}, Z[5] = {1, 2, 4, 0, 0};
};
template <int NC, bool ZR>
__host__ __device__ constexpr int swzq(int x) {
    int o = x;
    for (int h = 0; h < 5; ++h)
        if ((x >> (4 + h)) & 1) o ^= ZR ? SwzQ<NC>::Z[h] : SwzQ<NC>::REL[h];
    return o;
}
// swzq for a run-time x < 32 (only bit 4 can be high)
template <int NC, bool ZR>
__device__ __forceinline__ int swzq_small(int x) {
    constexpr int g = ZR ? SwzQ<NC>::Z[0] : SwzQ<NC>::REL[0];
    return x ^ ((x & 16) ? g : 0);
}
// twiddle table index: one float2 of padding per 32 (the levels' lanes read tw[j t] at strides
// that put 4-16 distinct j on one bank)
__host__ __device__ constexpr int tpad(int x) { return x + (x >> 5); }
__device__ __forceinline__ void ldsw2(float* base, uint32_t a, float2 v) {
    *reinterpret_cast<float2*>(reinterpret_cast<char*>(base) + a) = v;
}
__device__ __forceinline__ float2 ldsr2(const float* base, uint32_t a) {
    return *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(base) + a);
}
// the lane part of a relayout's swizzled point index (the layout of lane_mbits<NC, T, NEW>): the
// XOR of the images of the m bits the lane holds
template <int NC, int T, bool NEW>
__device__ __forceinline__ int lane_swz_m(int lj) {
    using G = GeoQ<NC>;
    int o = 0;
    static_for<0, G::B>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        constexpr bool init = !NEW && T == 0;
        constexpr int kind = init ? (b < G::NL ? 0 : 1) : QS<NC>::S.lev[NEW ? T : T - 1].kind[b];
        constexpr int bit = init ? (b < G::NL ? b : b - G::NL) : QS<NC>::S.lev[NEW ? T : T - 1].bit[b];
        if constexpr (kind == 0) o ^= ((lj >> bit) & 1) ? swzq<NC, false>(1 << b) : 0;
    });
    return o;
}
// the lane part of the Z row's swizzled bin index (the last level's layout)
template <int NC>
__device__ __forceinline__ int lane_swz_p(int lj) {
    constexpr int T = GeoQ<NC>::NLEV - 1;
    constexpr QLev q = QS<NC>::S.lev[T];
    int o = 0;
    static_for<0, GeoQ<NC>::B>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        if constexpr (q.kind[b] == 0) o ^= ((lj >> q.bit[b]) & 1) ? swzq<NC, true>(1 << QS<NC>::S.pbit[b]) : 0;
    });
    return o;
}

// the lane part of sum over m bits b with pbit[b] < PS held in lane bits of ((lane bit) << pbit)
template <int NC, int T, bool BELOW>
__device__ __forceinline__ int lane_pbits(int lj, int ps) {
    constexpr QLev q = QS<NC>::S.lev[T];
    int j = 0;
    static_for<0, GeoQ<NC>::B>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        constexpr int pb = QS<NC>::S.pbit[b];
        if constexpr (q.kind[b] == 0) {
            if (!BELOW || pb < ps) j |= ((lj >> q.bit[b]) & 1) << pb;
        }
    });
    return j;
}
// register index of digit value dv in the butterfly group of register base (level T)
template <int NC, int T>
constexpr int qreg(int base, int dv) {
    constexpr QLev q = QS<NC>::S.lev[T];
    int r = base;
    for (int c = 0; c < q.nd; ++c) r |= ((dv >> c) & 1) << q.bit[q.dig[c]];
    return r;
}
template <int NC, int T>
constexpr int reg_pbits(int r, int ps) {
    constexpr QLev q = QS<NC>::S.lev[T];
    int j = 0;
    for (int b = 0; b < GeoQ<NC>::B; ++b)
        if (q.kind[b] == 1 && QS<NC>::S.pbit[b] < ps) j |= ((r >> q.bit[b]) & 1) << QS<NC>::S.pbit[b];
    return j;
}

}  // namespace

// KIND: the output kind (kernels.hpp OUT_*). C: 1 mono, 2 stereo (interleaved); INF: f32 / s16.
// WV waves per block. VAR:
// ablations of the experiment library only (wrong output by design): 1 |X| by the f32 sqrt, 2 dB
// by v_log_f32, 4 no untangle / epilogue (the FFT and the Z row alone); 16 (exact, A/B): every
// swap as lane exchanges instead of the LDS relayout.
// DIR (round 6): any other geometry -- the viewer's win < n_fft and hops (lib.rs:43-46: 80 / 160 / 221 /
// 240 at n_fft 512 / 1024) -- with the same FFT and epilogue: every frame loads its n_fft samples
// itself (no ring: L2 holds the overlap; an odd start, where the frame's points straddle the
// sample pairs, reads its samples one by one), and the window step masks the product: x * w
// inside the window (bits unchanged), +0 in the centring pads, where the reference's frame holds
// +0 (lib.rs:377-385 pads the windowed frame and reads no sample there: x * 0 would be -0 for
// x < 0 and NaN for a non-finite x).
// RG (round 6, amp dB): the per-track range of the rows (a.trk_range: {ordered max, ordered min,
// NaN seen}, Batch::range) folded into the epilogue -- max / min / NaN of each frame's values,
// committed with one atomic triple per track a stream leaves -- instead of the separate pass over
// the rows (range_rows_kernel); max and min are exact, so the triple is the pass's.
template <int NC, int KIND, int C, int INF, int WV, int VAR = 0, bool DIR = false, bool RG = false>
__global__ void __launch_bounds__(64 * WV)
// two blocks per CU for mono input at n_fft 256 (12-wave blocks: 6 waves per SIMD, <= 80 VGPRs)
__attribute__((amdgpu_waves_per_eu(NC == 128 && C == 1 ? 6 : 1)))
stftq_kernel(StftLaunch a, uint64_t fps) {
    constexpr int OKQ = KIND == OUT_COMPLEX ? 0 : (KIND == OUT_MEL || KIND == OUT_MEL_AMP_DB) ? 2 : 1;
    using G = GeoQ<NC>;
    using CK = Chunk<C, INF>;
    using CT = typename CK::T;
    using ET = typename std::conditional<INF == IN_S16, int16_t, float>::type;
    constexpr int P = G::P, L = G::L, F = G::F, SH = G::SH, KEEP = G::KEEP, FPW = G::FPW;
    constexpr QSched S = QS<NC>::S;

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtl = lds;
    float2* twl = reinterpret_cast<float2*>(lds + G::WL_FLOATS);
    float2* scl = reinterpret_cast<float2*>(lds + G::WL_FLOATS + G::TW_FLOATS);
    float* wcl = lds + G::TAB_FLOATS;  // DIR: the window step's pad mask (same layout)
    float* work = lds + G::TAB_FLOATS + (DIR ? G::WL_FLOATS : 0);
    const exact::LogfEntry* logt = logf_tab_to_lds(lds + G::WL_FLOATS + G::TW_FLOATS + G::SC_FLOATS);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slot = lane / L;
    constexpr int kBlock = 64 * WV;

    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) {  // window: lane row (w[2m], w[2m+1])
        const int m = i >> 1, l = m % L, n = m / L;
        wtl[l * G::WL_STRIDE + 2 * n + (i & 1)] = a.wpad[i];
        if constexpr (DIR)  // the window step's mask: all ones inside the window, 0 in the pads
            wcl[l * G::WL_STRIDE + 2 * n + (i & 1)] = __uint_as_float(i >= a.pad_left && i < a.pad_left + a.win ? ~0u : 0u);
    }
    for (int i = threadIdx.x; i < NC; i += kBlock) {
        twl[tpad(i)] = a.tw1[i];
        scl[i] = a.sincos[i];
    }
    if (threadIdx.x == 0) scl[NC] = make_float2(0.f, 0.f);
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t stream = ((uint64_t)blockIdx.x * WV + wave) * FPW + slot;
    const uint64_t g0 = stream * fps;
    const uint64_t g1 = g0 + fps < total ? g0 + fps : total;
    const int hop = a.hop;
    float* region = work + (wave * FPW + slot) * G::RS;
    const uint32_t rbase = (uint32_t)(region - lds) * 4u;  // 128-byte aligned (GeoQ)
    // the staged row's start in the region: 16 floats further in the odd slots of a 16-lane layout,
    // so the two slots of a 32-lane ds_write_b32 fall on disjoint banks (RS is 0 mod 32)
    float* const srow = region + ((L == 16 && (slot & 1)) ? 16 : 0);
    const ET* in = static_cast<const ET*>(a.in);
    const float2 w8a = make_float2(a.xw8[0], a.xw8[1]), w8b = make_float2(a.xw8[2], a.xw8[3]);

    float2 raw[P];
    CT pre[SH];
    bool pre_ok = false;
    int hint = -1;
    uint64_t g_beg = 1, g_end = 0, base = 0;
    int64_t n = 0;
    // RG: the range of the rows this frame slot writes for its current track (r_trk)
    float r_max = -INFINITY, r_min = INFINITY;
    int r_nan = 0, r_trk = -1;
    auto r_flush = [&]() {  // the slot's L lanes (xor stays inside the group), then one atomic triple
#pragma unroll
        for (int m = L / 2; m >= 1; m >>= 1) {
            r_max = fmaxf(r_max, __shfl_xor(r_max, m));
            r_min = fminf(r_min, __shfl_xor(r_min, m));
            r_nan |= __shfl_xor(r_nan, m);
        }
        if ((lane & (L - 1)) == 0) {
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
        int lj = lane & (L - 1);  // the lane within its frame, opaque per frame (addresses formed
        asm volatile("" : "+v"(lj));  // in the loop, not held across it)
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
        // ---- rustfft Radix4 on the schedule ----
        static_for<0, G::NLEV>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            constexpr QLev q = S.lev[t];
            // the level's lane-bit <-> register-bit swaps: v_permlane16_swap for lane bit 4 (one
            // VALU per dword); the others as one LDS round trip of the frame's points (written at
            // their m, read back in the new layout: P stores + P loads where the DPP / bpermute
            // swaps cost 4-5 VALU per dword and swap)
            constexpr bool kPerm = q.nsw > 0 && q.swx[0] == 4 && (q.nsw < 2 || q.swx[1] == 4) &&
                                   (q.nsw < 3 || q.swx[2] == 4);
            if constexpr (q.nsw > 0 && ((VAR & 16) != 0 || kPerm)) {
                static_for<0, q.nsw>([&](auto sc) {
                    constexpr int s = decltype(sc)::value;
                    qswap<q.swx[s], q.swy[s], P>(v, lj);
                });
            } else if constexpr (q.nsw > 0) {
                wave_lds_sync();  // the region's previous readers are done
                {
                    const uint32_t wb = rbase + 8u * (uint32_t)lane_swz_m<NC, t, false>(lj);
                    static_for<0, P>([&](auto rc) {
                        constexpr int r = decltype(rc)::value;
                        constexpr int f = swzq<NC, false>(reg_mbits<NC, t, false>(r));
                        ldsw2(lds, (wb ^ (8u * (f & 15))) + 8u * (f & ~15), v[r]);
                    });
                }
                wave_lds_sync();
                {
                    const uint32_t rb = rbase + 8u * (uint32_t)lane_swz_m<NC, t, true>(lj);
                    static_for<0, P>([&](auto rc) {
                        constexpr int r = decltype(rc)::value;
                        constexpr int f = swzq<NC, false>(reg_mbits<NC, t, true>(r));
                        v[r] = ldsr2(lds, (rb ^ (8u * (f & 15))) + 8u * (f & ~15));
                    });
                }
            }
            constexpr int R = 1 << q.nd;
            constexpr int dmask = (1 << q.bit[q.dig[0]]) | (1 << q.bit[q.dig[1]]) | (q.nd == 3 ? (1 << q.bit[q.dig[2]]) : 0);
            constexpr int tstride = NC >> (q.pstart + 2);
            const int jl = t == 0 ? 0 : lane_pbits<NC, t, true>(lj, q.pstart);
            static_for<0, P>([&](auto bc) {
                constexpr int base_r = decltype(bc)::value;
                if constexpr ((base_r & dmask) == 0) {
                    if constexpr (t == 0 && R == 8) {
                        float2 b8[8];
                        static_for<0, 8>([&](auto dc) {
                            constexpr int rr = qreg<NC, t>(base_r, decltype(dc)::value);
                            b8[decltype(dc)::value] = v[rr];
                        });
                        rbfly8(b8, w8a, w8b);
                        static_for<0, 8>([&](auto dc) {
                            constexpr int rr = qreg<NC, t>(base_r, decltype(dc)::value);
                            v[rr] = b8[decltype(dc)::value];
                        });
                    } else {
                        constexpr int r0 = qreg<NC, t>(base_r, 0), r1 = qreg<NC, t>(base_r, 1);
                        constexpr int r2 = qreg<NC, t>(base_r, 2), r3 = qreg<NC, t>(base_r, 3);
                        if constexpr (t == 0) {
                            rbfly4(v[r0], v[r1], v[r2], v[r3]);
                        } else {
                            constexpr int jr = reg_pbits<NC, t>(base_r, q.pstart);
                            const int j = jl + jr;
                            rbfly(v[r0], v[r1], v[r2], v[r3], twl[tpad(j * tstride)], twl[tpad(2 * j * tstride)],
                                  twl[tpad(3 * j * tstride)]);
                        }
                    }
                }
            });
        });
        // ---- Z[p] to the region (bin p at its swizzled place) ----
        wave_lds_sync();  // (the fallback loads' reads of the region are done)
        {
            constexpr int T = G::NLEV - 1;
            const uint32_t zb = rbase + 8u * (uint32_t)lane_swz_p<NC>(lj);
            static_for<0, P>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                constexpr int f = swzq<NC, true>(reg_pbits<NC, T>(r, 99));
                ldsw2(lds, (zb ^ (8u * (f & 15))) + 8u * (f & ~15), v[r]);
            });
        }
        wave_lds_sync();
        // ---- untangle (realfft.rs:142-157, stftx's expression): pairs (k, NC - k), k = lj + L i ----
        // Z[k] at swz(lj) ^ swz(L i) (disjoint bits); Z[NC - k] = Z[c_i + (L - lj)], c_i = NC -
        // L (i + 1), at swz(L - lj) ^ swz(c_i) for lanes >= 1; lane 0's partner NC - L i carries
        // into c_i's bits, so its base is L and its constant swz(c_i + L) (a per-lane select), and
        // at i = 0 its partner is bin 0 itself, the Z[k] it just read
        const bool l0 = lj == 0;
        const uint32_t kb = rbase + 8u * (uint32_t)swzq_small<NC, true>(lj);
        const uint32_t pb = rbase + 8u * (uint32_t)(l0 ? L : swzq_small<NC, true>(L - lj));
        auto bin = [&](float2 b, float2 r, float2 sc) {
            const float s = sc.x, c = sc.y;
            const float xr = 0.5f * (((b.x + r.x) + c * (b.y + r.y)) - s * (b.x - r.x));
            const float xi = 0.5f * (((b.y - r.y) - s * (b.y + r.y)) - c * (b.x - r.x));
            return make_float2(xr, xi);
        };
        auto value = [&](float2 x) {  // the linear kinds (lib.rs:124, decibel.rs)
            constexpr bool power = KIND == OUT_POWER || KIND == OUT_POWER_DB;
            float val;
            if constexpr (power) val = x.x * x.x + x.y * x.y;  // num-complex norm_sqr
            else if constexpr ((VAR & 1) != 0) val = __builtin_amdgcn_sqrtf(x.x * x.x + x.y * x.y);
            else val = exact::hypotf_cr(x.x, x.y);  // num-complex norm
            if constexpr ((VAR & 2) != 0) {
                if constexpr (KIND == OUT_AMP_DB || KIND == OUT_POWER_DB) val = 20.0f * __builtin_amdgcn_logf(val);
            } else {
                if constexpr (KIND == OUT_POWER_DB) val = rdb(val, a.log_amin, 1e-36f, 10.0f, logt);
                if constexpr (KIND == OUT_AMP_DB) val = rdb(val, a.log_amin, 1e-18f, 20.0f, logt);
            }
            return val;
        };
        constexpr int NP = P / 2;
        float2 xo[OKQ == 0 ? 2 * NP + 1 : 1];
        float fo[OKQ == 0 ? 1 : 2 * NP + 1];
        static_for<0, ((VAR & 4) ? 0 : NP)>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int fk = swzq<NC, true>(L * i);
            constexpr int cp = NC - L * (i + 1);
            constexpr uint32_t xp = 8u * (swzq<NC, true>(cp) & 15), xp0 = 8u * (swzq<NC, true>(cp + L) & 15);
            const int k = lj + L * i;
            const float2 zk = ldsr2(lds, (kb ^ (8u * (fk & 15))) + 8u * (fk & ~15));
            float2 zp = ldsr2(lds, (pb ^ (l0 ? xp0 : xp)) + 8u * cp);
            if constexpr (i == 0) zp = l0 ? zk : zp;  // lane 0's bin 0 pairs with itself (NC - 0 = 0 mod NC)
            const float2 xk = bin(zk, zp, scl[k]);
            float2 xkp = bin(zp, zk, scl[NC - k]);
            if (i == 0 && lj == 0) xkp = make_float2(zk.x - zk.y, 0.0f);  // realfft.rs:157 (bin NC)
            if constexpr (OKQ == 0) {
                xo[2 * i] = xk;
                xo[2 * i + 1] = xkp;
            } else if constexpr (OKQ == 1) {
                fo[2 * i] = value(xk);
                fo[2 * i + 1] = value(xkp);
            } else {
                fo[2 * i] = exact::hypotf_cr(xk.x, xk.y);
                fo[2 * i + 1] = exact::hypotf_cr(xkp.x, xkp.y);
            }
        });
        {  // bin NC / 2 pairs with itself (lane 0 keeps it)
            const float2 zh = ldsr2(lds, rbase + 8u * swzq<NC, true>(NC / 2));
            const float2 xh = bin(zh, zh, scl[NC / 2]);
            if constexpr (OKQ == 0) xo[2 * NP] = xh;
            else if constexpr (OKQ == 1) fo[2 * NP] = value(xh);
            else fo[2 * NP] = exact::hypotf_cr(xh.x, xh.y);
        }
        wave_lds_sync();  // every Z read is done: the region takes the row
        if constexpr (OKQ == 2) {
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const int k = lj + L * i;
                region[k] = fo[2 * i];
                region[NC - k] = fo[2 * i + 1];
            }
            if (lj == 0) region[NC / 2] = fo[2 * NP];
            wave_lds_sync();
            // lib.rs:131 (the oracle's dot: one k-ascending fma chain per mel over its band)
            const int n_mels = a.n_mels;
            constexpr bool db = KIND == OUT_MEL_AMP_DB;
            float* out = static_cast<float*>(a.out) + g * (uint64_t)n_mels;
            for (int m = lj; m < n_mels; m += L) {
                const int4 bd = a.xmel_band[m];  // {first bin, bins, weight offset}
                float acc = 0.0f;
                for (int t2 = 0; t2 < bd.y; ++t2) acc = __builtin_fmaf(region[bd.x + t2], a.xmel_w[bd.z + t2], acc);
                if (valid) out[m] = db ? rdb(acc, a.log_amin, 1e-18f, 20.0f, logt) : acc;
            }
            wave_lds_sync();
        } else {
            constexpr int nfl = OKQ == 0 ? 2 * F : F;
            float* frow = static_cast<float*>(a.out) + g * (uint64_t)nfl;
            const int sh = (int)((reinterpret_cast<uintptr_t>(frow) >> 2) & 3);
            float* st = srow + sh;
            // (RG) this frame's values in this lane: every bin is in some lane's fo, bin NC / 2 in all
            float f_max = -INFINITY, f_min = INFINITY;
            int f_nan = 0;
            auto fold = [&](float x) {
                if constexpr (RG && OKQ == 1) {
                    f_max = fmaxf(f_max, x);
                    f_min = fminf(f_min, x);
                    f_nan |= x != x;
                }
            };
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const int k = lj + L * i;
                if constexpr (OKQ == 0) {
                    st[2 * k] = xo[2 * i].x;
                    st[2 * k + 1] = xo[2 * i].y;
                    st[2 * (NC - k)] = xo[2 * i + 1].x;
                    st[2 * (NC - k) + 1] = xo[2 * i + 1].y;
                } else {
                    st[k] = fo[2 * i];
                    st[NC - k] = fo[2 * i + 1];
                    fold(fo[2 * i]);
                    fold(fo[2 * i + 1]);
                }
            }
            if constexpr (OKQ == 1) fold(fo[2 * NP]);
            if (lj == 0) {
                if constexpr (OKQ == 0) {
                    st[NC] = xo[2 * NP].x;
                    st[NC + 1] = xo[2 * NP].y;
                } else {
                    st[NC / 2] = fo[2 * NP];
                }
            }
            wave_lds_sync();
            if (valid) store_row_b128<L>(frow, sh, srow, nfl, lj);
            wave_lds_sync();
            if constexpr (RG && OKQ == 1) {  // the slot's track changed: commit the previous one's
                const int t = valid ? hint : -1;
                if (t != r_trk) {  // uniform over the slot's lanes
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
    if constexpr (RG && OKQ == 1)
        if (r_trk >= 0) r_flush();  // the slot's last track
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
template <int NC>
static int ldsq_bytes(int wv, bool dir = false) {
    return (GeoQ<NC>::TAB_FLOATS + (dir ? GeoQ<NC>::WL_FLOATS : 0) + wv * GeoQ<NC>::FPW * GeoQ<NC>::RS) * 4;
}

template <int NC, int KIND, int C, int INF, int WV, int VAR = 0, bool DIR = false, bool RG = false>
static int launchq_k(const StftLaunch& a, hipStream_t s) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (VAR == 0 && KIND == OUT_AMP_DB && C == 1 && INF == IN_S16) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        const int v = e ? atoi(e) : 0;
        if (v == 1) return launchq_k<NC, KIND, C, INF, WV, 1, DIR, RG>(a, s);
        if (v == 3) return launchq_k<NC, KIND, C, INF, WV, 3, DIR, RG>(a, s);
        if (v == 4) return launchq_k<NC, KIND, C, INF, WV, 4, DIR, RG>(a, s);
        if (v == 12 && WV != 12) return launchq_k<NC, KIND, C, INF, 12, 0, DIR, RG>(a, s);
        if (v == 16) return launchq_k<NC, KIND, C, INF, WV, 16, DIR, RG>(a, s);
    }
#endif
    const int lds = ldsq_bytes<NC>(WV, DIR);
    if (lds > 163840) return -2;
    auto kern = stftq_kernel<NC, KIND, C, INF, WV, VAR, DIR, RG>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    constexpr uint64_t per_block = (uint64_t)WV * GeoQ<NC>::FPW;
    int grid = grid_for(reinterpret_cast<const void*>(kern), 64 * WV, lds, (a.total_frames + per_block - 1) / per_block,
                        a.grid, a.grid_share);
    const uint64_t streams = (uint64_t)grid * per_block;
    const uint64_t fps = (a.total_frames + streams - 1) / streams;
    grid = (int)((a.total_frames + fps * per_block - 1) / (fps * per_block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WV), lds, s, a, fps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int NC, int C, int INF, bool DIR = false>
static int launchq_c(const StftLaunch& a, hipStream_t s) {
    if ((a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB) && (!a.xmel_band || !a.xmel_w)) return -2;
    // 16-wave blocks (4 waves / SIMD, <= 128 VGPRs) for n_fft 512 / 1024: 3.59 -> 3.48 and 3.88
    // -> 3.70 ms on 1000 x 10 s amp-dB tracks; n_fft 256 stays at 12 (3.54 vs 3.69;
    // profiles/r05_stftq/ablations.txt)
    constexpr int WV = NC == 128 ? 12 : 16;
    switch (a.out_kind) {
        case OUT_COMPLEX: return launchq_k<NC, OUT_COMPLEX, C, INF, WV, 0, DIR>(a, s);
        case OUT_MAG: return launchq_k<NC, OUT_MAG, C, INF, WV, 0, DIR>(a, s);
        case OUT_POWER: return launchq_k<NC, OUT_POWER, C, INF, WV, 0, DIR>(a, s);
        case OUT_AMP_DB:  // (the range folded in when the batch asks for it: the C5 / viewer kind)
            return a.trk_range ? launchq_k<NC, OUT_AMP_DB, C, INF, WV, 0, DIR, true>(a, s)
                               : launchq_k<NC, OUT_AMP_DB, C, INF, WV, 0, DIR>(a, s);
        case OUT_POWER_DB: return launchq_k<NC, OUT_POWER_DB, C, INF, WV, 0, DIR>(a, s);
        case OUT_MEL: return launchq_k<NC, OUT_MEL, C, INF, WV, 0, DIR>(a, s);
        case OUT_MEL_AMP_DB: return launchq_k<NC, OUT_MEL_AMP_DB, C, INF, WV, 0, DIR>(a, s);
        default: return -2;
    }
}

// the canonical C5 geometry streams (win = n_fft, hop = n_fft / 4); any other (DIR) loads per frame
static bool q_canon(const StftLaunch& a) { return a.win == a.n_fft && a.hop * 4 == a.n_fft; }

template <int NC>
static int launchq_n(const StftLaunch& a, hipStream_t s) {
    if (!q_canon(a))  // the viewer's geometries: f32 mono / stereo (MultiTrack's mono pool)
        return a.channels == 2 ? launchq_c<NC, 2, IN_F32, true>(a, s) : launchq_c<NC, 1, IN_F32, true>(a, s);
    if (a.in_format == IN_S16) return a.channels == 2 ? launchq_c<NC, 2, IN_S16>(a, s) : launchq_c<NC, 1, IN_S16>(a, s);
    return a.channels == 2 ? launchq_c<NC, 2, IN_F32>(a, s) : launchq_c<NC, 1, IN_F32>(a, s);
}

bool stftq_supports(int n_fft, int win, int hop, int in_format, int channels) {
    if (!(n_fft == 256 || n_fft == 512 || n_fft == 1024) || !(channels == 1 || channels == 2)) return false;
    if (win == n_fft && hop * 4 == n_fft) return in_format == IN_F32 || in_format == IN_S16;
    // any other geometry (DIR): even win <= n_fft (the frame start t hop - n_fft / 2 is the
    // reference's t hop - win / 2 - pad_left, lib.rs:400-401), f32
    return in_format == IN_F32 && hop >= 1 && win >= 2 && win <= n_fft && win % 2 == 0;
}

int stftq_lds_bytes(const StftLaunch& a) {
    const bool dir = !q_canon(a);
    return a.n_fft == 256 ? ldsq_bytes<128>(12, dir) : a.n_fft == 512 ? ldsq_bytes<256>(16, dir) : ldsq_bytes<512>(16, dir);
}

int launch_stftq(const StftLaunch& a, hipStream_t s) {
    if (!stftq_supports(a.n_fft, a.win, a.hop, a.in_format, a.channels)) return -2;
    if (a.n_fft == 256) return launchq_n<128>(a, s);
    if (a.n_fft == 512) return launchq_n<256>(a, s);
    return launchq_n<512>(a, s);
}

}  // namespace thesia
