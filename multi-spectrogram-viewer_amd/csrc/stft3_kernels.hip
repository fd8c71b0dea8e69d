// stft3_kernels.hip -- the streaming STFT kernel for the canonical geometry of the batch
// configs (win = n_fft, hop = n_fft/4, f32 mono or stereo input).
//
// Contract as stft_kernel / stft2_kernel (one launch = downmix -> reflect framing x Hann/n_fft
// -> real FFT -> |X| -> linear kinds or mel + dB for every frame of a batch). What changes is
// how frames meet their input: each 64-lane wave runs FPW independent frame STREAMS, and a
// stream walks consecutive frames g0..g1 of the batch. Lane j of a frame holds the points
// m = L*n1 + j (samples 2m, 2m+1 from the frame start), and the frame start moves by
// hop = 2*L*SH samples (SH = P/4) from one frame to the next, so the next frame's point n1 is
// this frame's point n1 + SH in the SAME lane. The downmixed, unwindowed samples of the
// current frame stay in registers (raw[P]); a new frame shifts them by SH and needs only its
// hop of new samples: SH loads per lane (16 B stereo / 8 B mono), issued one frame ahead.
// HBM and L2 then see each input byte once (not n_fft/hop = 4 times), and the loads' latency
// hides under the previous frame's FFT. Frames whose new samples cross a track end (reflect
// padding, lib.rs:410-435) or start a stream / track reload all n_fft samples (direct or
// reflected). The mel weights are copied into LDS once per block.
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
#ifdef THESIA_MARKS
#define MARK(x) asm volatile("; MARK " #x)
#else
#define MARK(x)
#endif

template <int NC, int OK, int C, int INF, int VAR = 0, int WV = kWaves>
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
    const uint64_t g0 = stream * fps;
    const uint64_t g1 = g0 + fps < total ? g0 + fps : total;
    const int hop = a.hop;
    float* region = work + (wave * FPW + slot) * G3::RS_OK(stage_rows(OK, VAR), OK);
    const ET* in = static_cast<const ET*>(a.in);

    float2 raw[P];
    CT pre[SH];
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
        const uint64_t g = g0 + it;
        const bool valid = g < g1;
        // opaque per frame: keeps the untangle rotations (from ub) and the window reads (from
        // wj) inside the loop instead of hoisted as loop invariants into 100+ VGPRs
#pragma unroll
        for (int c = 0; c < G::CPL; ++c) asm volatile("" : "+v"(ub[c].x), "+v"(ub[c].y));
        int wj = j;
        asm volatile("" : "+v"(wj));
        const float4* wrow = reinterpret_cast<const float4*>(wtl + wj * G3::WL_STRIDE);
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
        // ---- the frame's raw samples (a hop: shift by SH points + the prefetched new ones) ----
        // (a rotating slot map instead of the shift was measured 1.05 ms slower: the switch
        // over four slot maps keeps all P raw points live and spills in the hot loop)
        if (pre_ok) {
#pragma unroll
            for (int n1 = 0; n1 < P - SH; ++n1) raw[n1] = raw[n1 + SH];
#pragma unroll
            for (int q = 0; q < SH; ++q) raw[P - SH + q] = CK::mix(pre[q]);
        } else if (valid && start >= 0 && start + 2 * NC <= n && ((base + (uint64_t)start * C) % (2 * C)) == 0) {
            const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)start * C) + j;
            static_for<0, P / 8>([&](auto gc) {  // 8 loads in flight per chunk
                constexpr int g8 = decltype(gc)::value;
                static_for<0, 8>([&](auto ic) {
                    constexpr int n1 = 8 * g8 + decltype(ic)::value;
                    raw[n1] = CK::mix(src[L * n1]);
                });
                pin_range<8 * g8, 8 * g8 + 8>(raw);
            });
        } else if (valid) {
            load_raw_generic<NC, INF>(a, region, j, start, n, base, C, a.fold != 0, raw);
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
            const int64_t nstart = start + hop;
            const bool nxt = valid && g + 1 < g1 && g + 1 < g_end && nstart + 2 * NC <= n &&
                             nstart + 2 * L * (P - SH) >= 0 &&
                             ((base + (uint64_t)(nstart + 2 * L * (P - SH)) * C) % (2 * C)) == 0;
            if constexpr ((VAR & 65536) != 0) __builtin_amdgcn_s_setprio(3);  // experiment
            if (nxt) {
                const CT* src = reinterpret_cast<const CT*>(in + base + (uint64_t)(nstart + 2 * L * (P - SH)) * C) + j;
#pragma unroll
                for (int q = 0; q < SH; ++q) pre[q] = src[L * q];
            }
            pre_ok = nxt;
            if constexpr ((VAR & 65536) != 0) __builtin_amdgcn_s_setprio(0);
        }
        MARK(prefetched);
        if constexpr ((VAR & 4) == 0) fft2<NC, TwTable4, G3::WIDE && (VAR & 32) == 0, (VAR & 8192) ? 1 : (VAR & 16384) ? 2 : 0>(v, region, j, TwTable4{reinterpret_cast<const float4*>(twtab) + wj, L});
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
            const int kind = a.out_kind;
            const bool power = kind == OUT_POWER || kind == OUT_POWER_DB;
            const bool db = kind == OUT_AMP_DB || kind == OUT_POWER_DB;
            float* frow = static_cast<float*>(a.out) + g * F;
            const int sh = (int)((reinterpret_cast<uintptr_t>(frow) >> 2) & 3);
            float* st = region + sh;
            const bool rng = a.trk_range != nullptr;  // uniform
            if (rng) {
                const int t = valid ? hint : -1;
                if (t != r_trk) {  // uniform over the frame's lanes
                    if (r_trk >= 0) r_flush();
                    r_trk = t;
                }
            }
            untangle2<NC, kBatch>(v, j, partner, ub, [&](int k, float xr, float xi) {
                const float p2 = __builtin_fmaf(xr, xr, xi * xi);
                // amp dB from |X|^2 (amp_db_of: no v_sqrt); amp / power as is
                const float val = db ? (power ? db_of(p2, a.log_amin, 1e-36f, 10.0f) : amp_db_of(p2, a.log_amin))
                                     : (power ? p2 : __builtin_amdgcn_sqrtf(p2));
                st[k] = val;
                if (rng) {
                    r_max = fmaxf(r_max, val);
                    r_min = fminf(r_min, val);
                    r_nan |= val != val;
                }
            });
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

// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
template <int NC, int OK, int VAR, int WV = kWaves>
static int lds3_bytes(const StftLaunch& a) {
    return (Geo3<NC, WV>::BASE_FLOATS_OK(stage_rows(OK, VAR), OK) +
            (OK == 2 ? (a.mel4_rows * 4 + a.mel4_rounds) * Geo2<NC>::L + 2 * a.mel4_rounds : 0)) * 4;
}

template <int NC, int OK, int C, int INF, int VAR = 0, int WV = kWaves>
static int launch3_k(const StftLaunch& a, hipStream_t stream) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (VAR == 0 && WV == kWaves && NC == 1024 && OK == 2 && C == 2 && INF == IN_F32) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        switch (e ? atoi(e) : 0) {
            case 1: return launch3_k<NC, OK, C, INF, 1>(a, stream);
            case 2: return launch3_k<NC, OK, C, INF, 2>(a, stream);
            case 4: return launch3_k<NC, OK, C, INF, 4>(a, stream);
            case 6: return launch3_k<NC, OK, C, INF, 6>(a, stream);
            case 8: return launch3_k<NC, OK, C, INF, 8>(a, stream);
            case 12: return launch3_k<NC, OK, C, INF, 12>(a, stream);
            case 16: return launch3_k<NC, OK, C, INF, 16>(a, stream);
            case 32: return launch3_k<NC, OK, C, INF, 32>(a, stream);  // narrow transpose
            case 64: return launch3_k<NC, OK, C, INF, 64>(a, stream);  // previous mel4
            case 128: return launch3_k<NC, OK, C, INF, 128>(a, stream);  // 4 mel accumulators
            case 256: return launch3_k<NC, OK, C, INF, 256>(a, stream);  // ablation: no sqrt
            case 512: return launch3_k<NC, OK, C, INF, 512>(a, stream);  // unbatched sqrt
            case 258: return launch3_k<NC, OK, C, INF, 258>(a, stream);  // ablation: no sqrt, no mel
            case 1000: return launch3_k<NC, OK, C, INF, 0, 12>(a, stream);  // 3 waves/SIMD
            case 4096: return launch3_k<NC, OK, C, INF, 4096>(a, stream);  // no priority phases
            case 8192: return launch3_k<NC, OK, C, INF, 8192>(a, stream);  // transposes at prio 1
            case 16384: return launch3_k<NC, OK, C, INF, 16384>(a, stream);  // transposes at prio 2
            case 32768: return launch3_k<NC, OK, C, INF, 32768>(a, stream);  // mel rounds at prio 3
            case 65536: return launch3_k<NC, OK, C, INF, 65536>(a, stream);  // prefetch issue at prio 3
            case 40960: return launch3_k<NC, OK, C, INF, 40960>(a, stream);  // + transposes at 1
            default: break;
        }
    }
    if constexpr (VAR == 0 && WV == kWaves && NC == 1024 && OK != 2 && C == 2 && INF == IN_F32) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        switch (e ? atoi(e) : 0) {
            case 4: return launch3_k<NC, OK, C, INF, 4>(a, stream);  // ablation: no FFT
            case 1028: return launch3_k<NC, OK, C, INF, 1028>(a, stream);
            case 4096: return launch3_k<NC, OK, C, INF, 4096>(a, stream);  // no priority phases
            default: break;
        }
    }
#endif
    // row-store methods (thesia_batch_set_option ROW_STORE; measured). Complex rows
    // leave as whole 128-byte lines by default (6.83 vs 6.98 ms lane-wise, 7.10 LDS-staged 16-byte,
    // one process); the alternatives are compiled for the headline geometry only.
    if constexpr (VAR == 0 && WV == kWaves && OK == 0) {
        if constexpr (NC == 1024 && C == 2 && INF == IN_F32) {
            if (a.row_alt == 1) return launch3_k<NC, OK, C, INF, 1024>(a, stream);
            if (a.row_alt == 3) return launch3_k<NC, OK, C, INF, 131072>(a, stream);  // lane-wise
        }
        return launch3_k<NC, OK, C, INF, 2048>(a, stream);
    }
    if constexpr (VAR == 0 && WV == kWaves && NC == 1024 && OK == 1 && C == 2 && INF == IN_F32) {
        if (a.row_alt == 1) return launch3_k<NC, OK, C, INF, 1024>(a, stream);
    }
    constexpr int kBlock = 64 * WV;
    const int lds = lds3_bytes<NC, OK, VAR, WV>(a);
    if (lds > 163840) return -2;
    auto kern = stft3_kernel<NC, OK, C, INF, VAR, WV>;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -1;
    if (a.total_frames == 0) return 0;
    constexpr uint64_t per_block = Geo3<NC, WV>::STREAMS;
    int grid = grid_for(reinterpret_cast<const void*>(kern), kBlock, lds,
                        (a.total_frames + per_block - 1) / per_block, a.grid);
    const uint64_t streams = (uint64_t)grid * per_block;
    const uint64_t fps = (a.total_frames + streams - 1) / streams;
    grid = (int)((a.total_frames + fps * per_block - 1) / (fps * per_block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, stream, a, fps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#ifndef THESIA_WV3_SMALL
#define THESIA_WV3_SMALL 12  // waves per block for mono linear kinds at n_fft <= 512 (3 per SIMD)
#endif
template <int NC, int C, int INF>
static int launch3_c(const StftLaunch& a, hipStream_t s) {
    // linear kinds of mono input at n_fft <= 512 fit 168 VGPRs without spills
    constexpr int WVS = NC <= 256 && C == 1 ? THESIA_WV3_SMALL : kWaves;
    if (a.out_kind == OUT_COMPLEX) return launch3_k<NC, 0, C, INF>(a, s);
    if (a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB) return launch3_k<NC, 2, C, INF>(a, s);
    return launch3_k<NC, 1, C, INF, 0, WVS>(a, s);
}

template <int NC>
static int launch3_nc(const StftLaunch& a, hipStream_t s) {
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch3_c<NC, 2, IN_S16>(a, s) : launch3_c<NC, 1, IN_S16>(a, s);
    return a.channels == 2 ? launch3_c<NC, 2, IN_F32>(a, s) : launch3_c<NC, 1, IN_F32>(a, s);
}

int stft3_lds_bytes(const StftLaunch& a) {
    const bool mel = a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB;
    const int ok = a.out_kind == OUT_COMPLEX ? 0 : mel ? 2 : 1;
    switch (a.n_fft / 2) {
        case 128: return ok == 0 ? lds3_bytes<128, 0, 0>(a) : ok == 1 ? lds3_bytes<128, 1, 0>(a) : lds3_bytes<128, 2, 0>(a);
        case 256: return ok == 0 ? lds3_bytes<256, 0, 0>(a) : ok == 1 ? lds3_bytes<256, 1, 0>(a) : lds3_bytes<256, 2, 0>(a);
        case 512: return ok == 0 ? lds3_bytes<512, 0, 0>(a) : ok == 1 ? lds3_bytes<512, 1, 0>(a) : lds3_bytes<512, 2, 0>(a);
        case 1024: return ok == 0 ? lds3_bytes<1024, 0, 0>(a) : ok == 1 ? lds3_bytes<1024, 1, 0>(a) : lds3_bytes<1024, 2, 0>(a);
        default: return 1 << 30;
    }
}

bool stft3_supports(int n_fft, int win, int hop, int in_format, int channels) {
    return (n_fft == 256 || n_fft == 512 || n_fft == 1024 || n_fft == 2048) && win == n_fft &&
           hop * 4 == n_fft && (in_format == IN_F32 || in_format == IN_S16) &&
           (channels == 1 || channels == 2);
}

int launch_stft3(const StftLaunch& a, hipStream_t s) {
    switch (a.n_fft / 2) {
        case 128: return launch3_nc<128>(a, s);
        case 256: return launch3_nc<256>(a, s);
        case 512: return launch3_nc<512>(a, s);
        case 1024: return launch3_nc<1024>(a, s);
        default: return -2;
    }
}

}  // namespace thesia
