// stft2_kernels.hip -- the fused STFT kernel for n_fft 256..2048 at 4 waves per SIMD.
//
// Same contract as stft_kernel (stft_kernels.hip): one launch runs, for every frame of a
// batch, downmix (lib.rs:42) -> reflect framing x Hann/n_fft (lib.rs:367-440) -> real FFT
// (realfft.rs:105-159) -> |X| / |X|^2 / dB (lib.rs:124-133, decibel.rs:33-100) or the
// mel projection + dB (lib.rs:130-134). What differs is the register / LDS budget, sized
// so that two 512-thread blocks share a CU (16 waves, 4 per SIMD):
//  * the FFT runs in place: one float2 v[P] per lane through both stages (the stage-2
//    inputs come back from the LDS transpose into the same registers);
//  * the transpose rows have stride S = L + 2 (S/2 odd): the stage-2 reads are ds_read_b64,
//    conflict-free; writes stay ds_write_b32 (re, then im, through one region per frame);
//  * the untangle works on bin PAIRS (k, NC-k): with A = Z_k + conj Z_{NC-k},
//    B = Z_k - conj Z_{NC-k}, (p, q) = e^{-i pi k/NC} B,
//        X_k = (A.re + q, A.im - p) / 2,   X_{NC-k} = (A.re - q, -A.im - p) / 2,
//    which is realfft.rs:148-154 for both bins of the pair from one complex product; each
//    lane receives the 16 partner values it needs with one ds_bpermute per component;
//  * the 1/2 of realfft.rs:148-154 is folded into the window (w/2 is exact, and scaling a
//    linear transform's input by 2^-1 scales every rounded intermediate exactly);
//  * the mel projection reads the |X| row with ds_read_b128 and float4 weights (4 bins per
//    step, steps start at a multiple of 4; the extra leading bins carry zero weight, so the
//    fma chain is term-for-term the oracle's k-ascending dot).
// Parity: the FFT order is not rustfft's (tolerance, tests/tolerances.py); the window
// product, downmix and dB epilogue follow the reference's evaluation order.
#include "stft2_core.hpp"

#include <cstdlib>

namespace thesia {

// OK: 0 complex, 1 linear kinds (|X|, |X|^2, dB), 2 mel kinds. PR: wave-priority phases as in
// stft3 (loads / window / FFT at 0, untangle / |X| / mel / stores at 2); PR = 0 (experiment
// variant 4096) without.
template <int NC, int OK, int INF, int PR = 1>
__global__ void __launch_bounds__(kBlock, 4)
stft2_kernel(StftLaunch a, uint64_t tiles_per_block) {
    using G = Geo2<NC>;
    constexpr int P = G::P, L = G::L, FPW = G::FPW, F = G::F, TILE = G::PASS_FRAMES;

    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wtab = lds;
    float* work = lds + G::WIN_FLOATS;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slot = lane / L, j0 = lane % L;
    const int partner0 = slot * L + ((L - j0) % L);

    for (int i = threadIdx.x; i < 2 * NC; i += kBlock) wtab[i] = a.wpad[i] * 0.5f;  // exact
    float2 ub[G::CPL];  // untangle bases (sin, cos)(pi (j + cL) / NC), realfft.rs:88-93
#pragma unroll
    for (int c = 0; c < G::CPL; ++c) ub[c] = a.sincos[j0 + c * L];
    __syncthreads();

    const uint64_t total = a.total_frames;
    const uint64_t n_tiles = (total + TILE - 1) / TILE;
    const uint64_t t_begin = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t t_end = t_begin + tiles_per_block < n_tiles ? t_begin + tiles_per_block : n_tiles;
    const int half_win = a.win / 2;
    const int C = a.channels;
    const bool fold = a.fold != 0;
    int hint = -1;
    float* region = work + (wave * FPW + slot) * G::RS;

    for (uint64_t tile = t_begin; tile < t_end; ++tile) {
        const uint64_t g = tile * TILE + (uint64_t)(wave * FPW + slot);
        const bool valid = g < total;
        if constexpr (PR != 0) __builtin_amdgcn_s_setprio(0);
        // opaque per pass: keeps the 2*(L/2)*CPL untangle rotations derived from ub inside the
        // loop instead of hoisted (and spilled) as loop invariants
#pragma unroll
        for (int c = 0; c < G::CPL; ++c) asm volatile("" : "+v"(ub[c].x), "+v"(ub[c].y));
        // the lane's column and partner opaque per pass too: the addresses derived from them
        // are formed per pass instead of hoisted (the complex / NC 512-1024 instances spilled)
        int j = j0, partner = partner0;
        asm volatile("" : "+v"(j), "+v"(partner));
        float2 v[P];
        if (valid) {
            hint = find_track(a.trk_frame0, a.n_tracks, g, hint);
            const uint64_t t = g - a.trk_frame0[hint];
            const int64_t n = (int64_t)a.trk_len[hint];
            const uint64_t base = a.trk_in_off[hint];
            const int64_t start = (int64_t)t * a.hop - half_win - a.pad_left;
            if (!load_direct2<NC, INF>(a, j, start, n, base, C, fold, wtab, v))
                load_frame_generic<NC, INF>(a, region, j, start, n, base, C, fold, wtab, v);
        } else {
#pragma unroll
            for (int n1 = 0; n1 < P; ++n1) v[n1] = make_float2(0.f, 0.f);
        }
        {
            // twiddle bases re-read every pass (24 VGPRs the 4-waves/SIMD budget lacks)
            TwBases<NC> tw;
            load_tw2<NC>(a, j, tw.b, tw.a);
            fft2<NC>(v, region, j, tw);
        }
        if constexpr (PR != 0) __builtin_amdgcn_s_setprio(2);
        if constexpr (OK == 2) {
            untangle2<NC>(v, j, partner, ub, [&](int k, float xr, float xi) {
                region[k] = __builtin_amdgcn_sqrtf(xr * xr + xi * xi);  // |X| (lib.rs:124)
            });
            if (j == 0) {
#pragma unroll
                for (int k = F; k < G::F4; ++k) region[k] = 0.0f;
            }
            wave_lds_sync();
            mel4<NC>(a, region, a.mel4_wt, a.mel4_round, a.mel4_k0, j, g, valid);
            continue;
        }
        if constexpr (OK == 0) {
            float2* crow = reinterpret_cast<float2*>(a.out) + g * F;  // row base: immediate offsets
            untangle2<NC>(v, j, partner, ub, [&](int k, float xr, float xi) {
                if (valid) crow[k] = make_float2(xr, xi);
            });
        } else {
            // linear kinds: the row goes through the frame's LDS region, then out with one
            // coalesced store per L bins (the epilogue stays out of the untangle's registers)
            const int kind = a.out_kind;
            const bool power = kind == OUT_POWER || kind == OUT_POWER_DB;
            const bool db = kind == OUT_AMP_DB || kind == OUT_POWER_DB;
            untangle2<NC>(v, j, partner, ub, [&](int k, float xr, float xi) {
                const float p2 = xr * xr + xi * xi;  // num-complex norm_sqr
                region[k] = power ? p2 : __builtin_amdgcn_sqrtf(p2);
            });
            wave_lds_sync();
            float* frow = static_cast<float*>(a.out) + g * F;
            if (valid) {
                for (int k = j; k < F; k += L) {
                    float val = region[k];
                    if (db) val = power ? db_of(val, a.log_amin, 1e-36f, 10.0f)
                                        : db_of(val, a.log_amin, 1e-18f, 20.0f);
                    frow[k] = val;
                }
            }
        }
    }
}

// --------------------------------------------------------------------------------------
// host-side dispatch
// --------------------------------------------------------------------------------------
template <int NC, int OK, int INF, int PR = 1>
static int launch2_k(const StftLaunch& a, hipStream_t stream) {
#ifdef THESIA_EXPERIMENTS
    if constexpr (PR == 1) {
        const char* e = getenv("THESIA_STFT_VARIANT");
        if (e && atoi(e) == 4096) return launch2_k<NC, OK, INF, 0>(a, stream);
    }
#endif
    constexpr int lds = Geo2<NC>::LDS_BYTES;
    auto kern = stft2_kernel<NC, OK, INF, PR>;
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
            return -1;
        attr_set = true;
    }
    const uint64_t n_tiles = (a.total_frames + Geo2<NC>::PASS_FRAMES - 1) / Geo2<NC>::PASS_FRAMES;
    if (n_tiles == 0) return 0;
    int grid = grid_for(reinterpret_cast<const void*>(kern), kBlock, lds, n_tiles, a.grid, a.grid_share);
    const uint64_t tpb = (n_tiles + grid - 1) / grid;
    grid = (int)((n_tiles + tpb - 1) / tpb);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, stream, a, tpb);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int NC, int INF>
static int launch2_fmt(const StftLaunch& a, hipStream_t s) {
    if (a.out_kind == OUT_COMPLEX) return launch2_k<NC, 0, INF>(a, s);
    if (a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB) return launch2_k<NC, 2, INF>(a, s);
    return launch2_k<NC, 1, INF>(a, s);
}

template <int NC>
static int launch2_nc(const StftLaunch& a, hipStream_t s) {
    return a.in_format == IN_S16 ? launch2_fmt<NC, IN_S16>(a, s) : launch2_fmt<NC, IN_F32>(a, s);
}

bool stft2_supports(int n_fft) {
    return n_fft == 256 || n_fft == 512 || n_fft == 1024 || n_fft == 2048;
}

int launch_stft2(const StftLaunch& a, hipStream_t s) {
    switch (a.n_fft / 2) {
        case 128: return launch2_nc<128>(a, s);
        case 256: return launch2_nc<256>(a, s);
        case 512: return launch2_nc<512>(a, s);
        case 1024: return launch2_nc<1024>(a, s);
        default: return -2;
    }
}

int stft2_kernel_info(int n_fft, int* lds_bytes, int* tile_frames, int* lanes_per_frame) {
    int lds = 0, tile = 0, L = 0;
    switch (n_fft / 2) {
#define THESIA_INFO2(NC) \
        case NC: lds = Geo2<NC>::LDS_BYTES; tile = Geo2<NC>::PASS_FRAMES; L = Geo2<NC>::L; break;
        THESIA_INFO2(128) THESIA_INFO2(256) THESIA_INFO2(512) THESIA_INFO2(1024)
#undef THESIA_INFO2
        default: return -2;
    }
    if (lds_bytes) *lds_bytes = lds;
    if (tile_frames) *tile_frames = tile;
    if (lanes_per_frame) *lanes_per_frame = L;
    return 0;
}

}  // namespace thesia
