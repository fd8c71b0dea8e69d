// stft3_kernel.hpp -- the streaming STFT kernel template (stft3_kernels.hip: the canonical
// geometry win = n_fft, hop = n_fft/4; stft3v_kernels.hip: the viewer geometries, HQ > 0).
#pragma once
#include "stft3_core.hpp"

#include <cstdlib>
#include <type_traits>

namespace thesia {

// OK: 0 complex, 1 linear kinds, 2 mel kinds. C: 1 mono, 2 stereo (interleaved); INF: f32 / s16.
// VAR (experiments, THESIA_STFT_VARIANT): bit0 = per-pair partner exchange instead of the
// batched one (measured 0.07 ms slower); ablations (outputs wrong, timing only): bit1 = no mel
// projection, bit2 = no FFT (stages and transposes skipped), bit3 = no untangle / |X| / mel;
// bit4 = mel with 4 float4 steps per LDS round trip instead of 8; bit5 = the narrow (stride
// L + 2, ds_read2_b64) transpose instead of the wide one; bit6 = the previous mel4 (per-round
// setup reads); bit7 = four mel accumulators; bit8 = ablation: |X|^2 (no v_sqrt); bit9 = the
// sqrts not batched; bit10 (linear / complex kinds) = the other row-store method (stage_rows);
// bit11 (complex) = rows as whole 128-byte lines, the shared line carried (line_rows; the
// default for complex rows); bit17 (complex) = lane-wise 8-byte stores, chosen explicitly;
// bit12 = no wave-priority phases (s_setprio; previous); bit13 / bit14 = the FFT's twiddle reads
// and transposes at priority 1 / 2; bit15 = the mel rounds at priority 3; bit16 = the prefetch
// loads issued at priority 3.
// Product bits: 18-20 = the linear kind fixed at compile time (OUT_AMP .. OUT_POWER_DB; 0 = the
// launch's out_kind at run time), bit21 = the per-track range fold compiled in (with a fixed kind:
// a.trk_range is set). Without them every bin of the epilogue runs uniform branches on the kind
// and on the range flag (four s_cbranch per bin at amp dB).
#ifdef THESIA_MARKS
#define MARK(x) asm volatile("; MARK " #x)
#else
#define MARK(x)
#endif

// HQ > 0: a viewer geometry (lib.rs:43-46: win = 4 hop <= n_fft, hop even), whose hop of
// hop/2 = HQ L + rem points is not a whole number of the lane's rows. Lane j keeps the points
// of one residue mod L of the TRACK's point grid, so frame t (track-local) finds them in its
// column jc = (j - t rem) mod L, and a new frame shifts the ring by HQ rows where the previous
// column was >= rem and by HQ + 1 where it was < rem (a select per row), then takes HQ + 1
// prefetched rows (the new frame's rows P - HQ - 1 .. P - 1 of its column; the first of them
// repeats the ring's last row where the shift is HQ). The window row and the stage-1 twiddles
// are the column's; the transpose writes column jc and reads row j, so from stage 2 on (bins,
// untangle partners, outputs) the lane is j as in the canonical geometry.
// VODD: an odd hop (22.05 / 44.1 kHz: 221 / 441 samples), where every other frame starts between
// two complex points of the previous one. The streams then come in pairs that interleave the
// frames (stream 2s takes frames g, g + 2, ..., 2s + 1 the ones between), so a stream's hop is
// 2 hop samples = HQ L + rem points, and a frame starting at an odd sample reads the track on
// the point grid shifted by one sample (base + C elements): the same ring, on that grid. Its
// vector loads are then only dword-aligned (f32, s16 stereo) or, for int16 mono, 2-byte-aligned
// (a sample pair straddling two dwords). Complex rows are stored per row
// (a stream's rows are not contiguous).
template <int NC, int OK, int C, int INF, int VAR = 0, int WV = kWaves, int HQ = 0, int VODD = 0>
__global__ void __launch_bounds__(64 * WV, WV / 4)
stft3_kernel(StftLaunch a, uint64_t fps) {
    constexpr int kBlock = 64 * WV;
    constexpr bool kBatch = (VAR & 1) == 0;
    using G = Geo2<NC>;
    using G3 = Geo3<NC, WV>;
    using CK = Chunk<C, INF>;
    using CT = typename CK::T;
    using ET = typename std::conditional<INF == IN_S16, int16_t, float>::type;
    constexpr int P = G::P, L = G::L, FPW = G::FPW, F = G::F, SH = G3::SH;
    constexpr bool VIEW = HQ > 0;
    constexpr bool ODD = VODD != 0;
    static_assert(!ODD || (VIEW && !line_rows(OK, VAR)), "odd-hop streams");
    // odd-hop vector loads: dword-aligned, or 2-byte-aligned for int16 mono (a sample pair)
    constexpr int OALIGN = C == 1 && INF == IN_S16 ? 2 : 4;
    constexpr int NPRE = VIEW ? HQ + 1 : SH;  // rows prefetched per frame
    constexpr int KEEP = P - NPRE;            // ring rows carried into the next frame
    static_assert(KEEP > 0, "hop shorter than the frame");

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtl = lds;
    float2* twtab = reinterpret_cast<float2*>(lds + G3::WL_FLOATS);
    float* work = lds + G3::WL_FLOATS + G3::TW_FLOATS;
    // mel tables in LDS: weight rows, then the per-lane start bins, then the round table
    float4* mel_lds = reinterpret_cast<float4*>(lds + G3::BASE_FLOATS);
    int* k0_lds = reinterpret_cast<int*>(mel_lds + (OK == 2 ? a.mel4_rows * L : 0));
    int2* rd_lds = reinterpret_cast<int2*>(k0_lds + (OK == 2 ? a.mel4_rounds * L : 0));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slot = lane / L, j = lane % L;
    const int partner = slot * L + ((L - j) % L);

    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) {  // w/2 is exact (realfft's 1/2)
        const int m = i >> 1, jj = m % L, n1 = m / L;
        wtl[jj * G3::WL_STRIDE + 2 * n1 + (i & 1)] = a.wpad[i] * 0.5f;
    }
    if constexpr (OK == 2) {
        const int nw = a.mel4_rows * L;
        for (int i = threadIdx.x; i < nw; i += kBlock) mel_lds[i] = a.mel4_wt[i];
        for (int i = threadIdx.x; i < a.mel4_rounds * L; i += kBlock) k0_lds[i] = a.mel4_k0[i];
        for (int i = threadIdx.x; i < a.mel4_rounds; i += kBlock) rd_lds[i] = a.mel4_round[i];
    }
    // stage-1 twiddles with k1 pairs interleaved (TwTable4): [k1/2][j][k1&1]
    for (int i = threadIdx.x; i < P * L; i += kBlock) {
        const int k1 = i / L, jj = i % L;
        twtab[((k1 >> 1) * L + jj) * 2 + (k1 & 1)] = a.tw3[i];
    }
    float2 ub[G::CPL];
#pragma unroll
    for (int c = 0; c < G::CPL; ++c) ub[c] = a.sincos[j + c * L];
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t stream = ((uint64_t)blockIdx.x * WV + wave) * FPW + slot;
    // a stream's frames: g0 + GS it (ODD: a stream pair shares 2 fps frames, interleaved)
    constexpr uint64_t GS = ODD ? 2 : 1;
    const uint64_t g0 = (ODD ? (stream >> 1) * 2 * fps : stream * fps);
    const uint64_t g1 = g0 + GS * fps < total ? g0 + GS * fps : total;
    const uint64_t gpar = ODD ? (stream & 1) : 0;
    const int hop = a.hop;
    const int hop_s = ODD ? 2 * hop : hop;  // samples between a stream's frames
    float* region = work + (wave * FPW + slot) * G3::RS_OK(stage_rows(OK, VAR), OK) + G3::swz(slot);
    const ET* in = static_cast<const ET*>(a.in);

    float2 raw[P];
    CT pre[NPRE];
    const int rem = VIEW ? (hop_s >> 1) & (L - 1) : 0;
    bool pre_ok = false;
    int hint = -1;
    // the stream's current track, cached across frames (looked up again only past its end)
    uint64_t g_beg = 1, g_end = 0, base = 0;
    int64_t n = 0;
    // per-track range of the rows this stream writes (a.trk_range: linear kinds, staged rows),
    // committed with one atomic triple per track the stream leaves
    float r_max = -INFINITY, r_min = INFINITY;
    int r_nan = 0, r_trk = -1;
    float carry[32 / L];  // line_rows: floats j + c*L of the line the last row ended in
    auto r_flush = [&]() {
#pragma unroll
        for (int m = L / 2; m >= 1; m >>= 1) {  // the frame's L lanes (xor stays inside the group)
            r_max = fmaxf(r_max, __shfl_xor(r_max, m));
            r_min = fminf(r_min, __shfl_xor(r_min, m));
            r_nan |= __shfl_xor(r_nan, m);
        }
        if (j == 0) {
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
        MARK(top);
        // wave priority phases (measured): loads / window / FFT at priority 0,
        // untangle / |X| / mel / stores at 2. With 2 waves per SIMD, the wave in the LDS-latency-
        // bound chains (bpermute batch, |X| row, mel rounds) then issues first whenever it is
        // ready and the other wave's FFT (high ILP) fills the gaps: mel-128 5.13 -> 4.67 ms.
        if constexpr ((VAR & 4096) == 0) __builtin_amdgcn_s_setprio(0);
        const uint64_t g = g0 + gpar + GS * it;
        const bool valid = g < g1;
        // opaque per frame: keeps the untangle rotations (from ub) and the window reads (from
        // wj) inside the loop instead of hoisted as loop invariants into 100+ VGPRs
#pragma unroll
        for (int c = 0; c < G::CPL; ++c) asm volatile("" : "+v"(ub[c].x), "+v"(ub[c].y));
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
        // the frame's point grid (ODD: shifted by one sample for an odd start) and its column
        const int par = ODD ? (int)(start & 1) : 0;
        const uint64_t bse = base + (uint64_t)(par * C);
        const int64_t st = start - par;
        int jc = j;  // the frame's column (HQ > 0): (j - frame start in points) mod L
        if constexpr (VIEW) {
            if (valid) jc = (j - (int)((st >> 1) & (L - 1))) & (L - 1);
        } else {
            // opaque per frame here too: the addresses derived from the column are then formed
            // per frame instead of hoisted as loop invariants (which spilled 21-65 VGPRs at
            // NC 512 / 1024; the viewer instances, whose column varies, never did)
            asm volatile("" : "+v"(jc));
        }
        int wj = jc;
        asm volatile("" : "+v"(wj));
        const float4* wrow = reinterpret_cast<const float4*>(wtl + wj * G3::WL_STRIDE);
        // the vector loads of a frame at element offset e: naturally aligned (CT = 2 samples x C
        // channels), or on ODD grids OALIGN-aligned memcpy loads (dword: f32, s16 stereo at an even
        // element offset, else the generic loader; int16 mono: 2-byte, every offset)
        auto aligned = [&](uint64_t e) {
            return ODD ? (e * sizeof(ET)) % OALIGN == 0 : e % (2 * C) == 0;
        };
        auto ldc = [](const CT* p) -> CT {
            if constexpr (ODD) {
                CT v;
                __builtin_memcpy(&v, __builtin_assume_aligned(p, C == 1 && INF == IN_S16 ? 2 : 4), sizeof(CT));
                return v;
            } else {
                return *p;
            }
        };
        // ---- the frame's raw samples (a hop: shift by SH points + the prefetched new ones) ----
        // (a rotating slot map instead of the shift was measured 1.05 ms slower: the switch
        // over four slot maps keeps all P raw points live and spills in the hot loop)
        if (pre_ok) {
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
        } else if (valid && start >= 0 && start + 2 * NC <= n && aligned(bse + (uint64_t)st * C)) {
            const CT* src = reinterpret_cast<const CT*>(in + bse + (uint64_t)st * C) + jc;
            static_for<0, P / 8>([&](auto gc) {  // 8 loads in flight per chunk
                constexpr int g8 = decltype(gc)::value;
                static_for<0, 8>([&](auto ic) {
                    constexpr int n1 = 8 * g8 + decltype(ic)::value;
                    raw[n1] = CK::mix(ldc(src + L * n1));
                });
                pin_range<8 * g8, 8 * g8 + 8>(raw);
            });
        } else if (valid) {
            load_raw_generic<NC, INF>(a, region, jc, start, n, base, C, a.fold != 0, raw);
        } else {
#pragma unroll
            for (int n1 = 0; n1 < P; ++n1) raw[n1] = make_float2(0.f, 0.f);
        }
        MARK(loaded);
        // window (lib.rs:379, with the 1/2 of realfft.rs:148-154 folded in)
        float2 v[P];
        static_for<0, P / 2>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const float4 w = wrow[q];
            v[2 * q] = make_float2(raw[2 * q].x * w.x, raw[2 * q].y * w.y);
            v[2 * q + 1] = make_float2(raw[2 * q + 1].x * w.z, raw[2 * q + 1].y * w.w);
        });
        // ---- prefetch the next frame's hop of new samples (its points P-SH .. P-1) ----
        {
            const int64_t nstart = start + hop_s, nst = st + hop_s;
            const bool nxt = valid && g + GS < g1 && g + GS < g_end && nstart + 2 * NC <= n &&
                             nst + 2 * L * KEEP >= 0 &&
                             aligned(bse + (uint64_t)(nst + 2 * L * KEEP) * C);
            if constexpr ((VAR & 65536) != 0) __builtin_amdgcn_s_setprio(3);  // experiment
            if (nxt) {
                const int jn = (jc - rem) & (L - 1);  // the next frame's column (= j unless HQ > 0)
                const CT* src = reinterpret_cast<const CT*>(in + bse + (uint64_t)(nst + 2 * L * KEEP) * C) + jn;
#pragma unroll
                for (int q = 0; q < NPRE; ++q) pre[q] = ldc(src + L * q);
            }
            pre_ok = nxt;
            if constexpr ((VAR & 65536) != 0) __builtin_amdgcn_s_setprio(0);
        }
        MARK(prefetched);
        if constexpr ((VAR & 4) == 0) fft2<NC, TwTable4, G3::WIDE && (VAR & 32) == 0, (VAR & 8192) ? 1 : (VAR & 16384) ? 2 : 0>(v, region, j, TwTable4{reinterpret_cast<const float4*>(twtab) + wj, L}, wj);
        else pin(v);
        MARK(fft);
        if constexpr ((VAR & 4096) == 0) __builtin_amdgcn_s_setprio(2);
        if constexpr (OK == 2 && (VAR & 8) != 0) {  // ablation: no untangle / |X| / mel
            pin(v);
        } else if constexpr (OK == 2) {
            // |X| (lib.rs:124) in three batches: every |X|^2 of the lane, then every v_sqrt (a
            // transcendental whose result used right away stalls the wave: 0.34 ms per launch
            // measured), then the LDS row writes
            constexpr int NS = 2 * G::CPL * (L / 2) + 1;
            float mag[NS];
            mag[NS - 1] = 0.0f;
            untangle2<NC, kBatch>(v, j, partner, ub, [&](int, float xr, float xi, auto sc) {
                mag[decltype(sc)::value] = __builtin_fmaf(xr, xr, xi * xi);
            });
            if constexpr ((VAR & 512) == 0) {
                pin_f(mag);
#pragma unroll
                for (int i = 0; i < NS; ++i)
                    if constexpr ((VAR & 256) == 0) mag[i] = __builtin_amdgcn_sqrtf(mag[i]);
                pin_f(mag);
            } else {
#pragma unroll
                for (int i = 0; i < NS; ++i) mag[i] = __builtin_amdgcn_sqrtf(mag[i]);
            }
            static_for<0, G::CPL * (L / 2)>([&](auto ic) {
                constexpr int i = decltype(ic)::value, c = i / (L / 2), t = i % (L / 2);
                const int k = j + c * L + P * t;
                region[k] = mag[2 * i];
                region[NC - k] = mag[2 * i + 1];
            });
            if (j == 0) region[NC / 2] = mag[NS - 1];
            if (j == 0) {
#pragma unroll
                for (int k = F; k < G::F4; ++k) region[k] = 0.0f;
            }
            wave_lds_sync();
            MARK(untangled);
            if constexpr ((VAR & 32768) != 0) __builtin_amdgcn_s_setprio(3);  // experiment: mel at 3
            // U = 8 float4 steps per LDS round trip (the FFT's registers are free by now)
            if constexpr ((VAR & 2) == 0 && (VAR & 64) == 0)
                mel4<NC, (VAR & 16) ? 4 : 8, (VAR & 128) ? 4 : 1>(a, region, mel_lds, rd_lds, k0_lds, j, g, valid);
            if constexpr ((VAR & 64) != 0) mel4_v1<NC, 8>(a, region, mel_lds, rd_lds, k0_lds, j, g, valid);
        } else if constexpr (OK == 0 && line_rows(OK, VAR)) {
            // whole 128-byte lines: the stream's rows are contiguous (frame g's
            // row ends where g+1's begins), so the row is staged from its line start (sh floats
            // into the line) and leaves as whole lines, one float4 per lane; the line it shares
            // with the next frame is carried in registers (lane j: floats j + c*L of that line)
            // and written with the next row. Only a stream's first head and last tail are partial.
            static_assert(L <= 32 && 32 % L == 0, "a frame's lanes tile a 128-byte line");
            constexpr int CW = 32 / L;  // carry floats per lane
            float* crow = static_cast<float*>(a.out) + g * (2 * F);
            const int sh = (int)((reinterpret_cast<uintptr_t>(crow) >> 2) & 31);  // even
            float2* st = reinterpret_cast<float2*>(region + sh);
            untangle2<NC, kBatch>(v, j, partner, ub, [&](int k, float xr, float xi) {
                st[k] = make_float2(xr, xi);
            });
#pragma unroll
            for (int c = 0; c < CW; ++c)  // the previous row's tail (same stream)
                if (it > 0 && j + c * L < sh) region[j + c * L] = carry[c];
            wave_lds_sync();
            if (valid) {
                float* lb = crow - sh;  // 128-byte aligned
                const int tot = sh + 2 * F, nfull = tot >> 5, rem = tot & 31;
                const bool head = it == 0 && sh != 0;  // a stream's first head line: float by float
#pragma unroll
                for (int c = 0; c < CW; ++c)
                    if (head && j + c * L >= sh) lb[j + c * L] = region[j + c * L];
                for (int i = (head ? 8 : 0) + j; i < nfull * 8; i += L)
                    *reinterpret_cast<float4*>(__builtin_assume_aligned(lb + 4 * i, 16)) =
                        *reinterpret_cast<const float4*>(__builtin_assume_aligned(region + 4 * i, 16));
                const bool last = g + 1 == g1;  // the stream's last row: its tail line leaves partial
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const int e = j + c * L;
                    const float tail = region[nfull * 32 + (e < rem ? e : 0)];
                    if (!last) carry[c] = tail;
                    else if (e < rem) lb[nfull * 32 + e] = tail;
                }
            }
        } else if constexpr (OK == 0 && !stage_rows(OK, VAR)) {  // lane-wise 8-byte stores
            float2* crow = reinterpret_cast<float2*>(a.out) + g * F;
            untangle2<NC, kBatch>(v, j, partner, ub, [&](int k, float xr, float xi) {
                if (valid) st_out(crow + k, make_float2(xr, xi));
            });
        } else if constexpr (OK == 0) {
            float* crow = static_cast<float*>(a.out) + g * (2 * F);
            const int sh = (int)((reinterpret_cast<uintptr_t>(crow) >> 2) & 3);  // 0 or 2
            float2* st = reinterpret_cast<float2*>(region + sh);
            untangle2<NC, kBatch>(v, j, partner, ub, [&](int k, float xr, float xi) {
                st[k] = make_float2(xr, xi);
            });
            wave_lds_sync();
            if (valid) store_row_b128<L>(crow, sh, region, 2 * F, j);
        } else if constexpr (stage_rows(OK, VAR)) {
            constexpr int KD = (VAR >> 18) & 7;
            float* frow = static_cast<float*>(a.out) + g * F;
            const int sh = (int)((reinterpret_cast<uintptr_t>(frow) >> 2) & 3);
            float* st = region + sh;
            const bool rng = KD ? (VAR & (1 << 21)) != 0 : a.trk_range != nullptr;  // uniform
            if (rng) {
                const int t = valid ? hint : -1;
                if (t != r_trk) {  // uniform over the frame's lanes
                    if (r_trk >= 0) r_flush();
                    r_trk = t;
                }
            }
            // the row's values for kind K (compile time: no per-bin branches). A fixed kind takes
            // the range ops per VAR bit 21; the run-time kind switches once per frame and always
            // forms them (committed only with a.trk_range)
            auto rows = [&](auto kc) {
                constexpr int K = decltype(kc)::value;
                constexpr bool power = K == OUT_POWER || K == OUT_POWER_DB;
                constexpr bool db = K == OUT_AMP_DB || K == OUT_POWER_DB;
                constexpr bool R = KD ? (VAR & (1 << 21)) != 0 : true;
                untangle2<NC, kBatch>(v, j, partner, ub, [&](int k, float xr, float xi) {
                    const float p2 = __builtin_fmaf(xr, xr, xi * xi);
                    // amp dB from |X|^2 (amp_db_of: no v_sqrt); amp / power as is
                    const float val = db ? (power ? db_of(p2, a.log_amin, 1e-36f, 10.0f) : amp_db_of(p2, a.log_amin))
                                         : (power ? p2 : __builtin_amdgcn_sqrtf(p2));
                    st[k] = val;
                    if constexpr (R) {
                        r_max = fmaxf(r_max, val);
                        r_min = fminf(r_min, val);
                        r_nan |= val != val;
                    }
                });
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
        } else {  // lane-wise 4-byte stores
            const int kind = a.out_kind;
            const bool power = kind == OUT_POWER || kind == OUT_POWER_DB;
            const bool db = kind == OUT_AMP_DB || kind == OUT_POWER_DB;
            untangle2<NC, kBatch>(v, j, partner, ub, [&](int k, float xr, float xi) {
                const float p2 = __builtin_fmaf(xr, xr, xi * xi);
                region[k] = power ? p2 : __builtin_amdgcn_sqrtf(p2);
            });
            wave_lds_sync();
            float* frow = static_cast<float*>(a.out) + g * F;
            if (valid) {
                for (int k = j; k < F; k += L) {
                    float val = region[k];
                    if (db) val = power ? db_of(val, a.log_amin, 1e-36f, 10.0f)
                                        : db_of(val, a.log_amin, 1e-18f, 20.0f);
                    st_out(frow + k, val);
                }
            }
        }
    }
    if (r_trk >= 0) r_flush();  // (a.trk_range set: the stream's last track)
}

}  // namespace thesia
