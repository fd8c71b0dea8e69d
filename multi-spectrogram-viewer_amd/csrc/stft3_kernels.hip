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
#include "stft3_kernel.hpp"

namespace thesia {


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
                        (a.total_frames + per_block - 1) / per_block, a.grid, a.grid_share);
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
    // amp dB (the default kind, the C5 / viewer rows): the kind and the range fold at compile
    // time (stft3_kernel.hpp, VAR bits 18-21)
    bool fixed = a.out_kind == OUT_AMP_DB && a.row_alt == 0;
#ifdef THESIA_EXPERIMENTS
    if (getenv("THESIA_STFT3_RTKIND")) fixed = false;  // A/B: the run-time kind
    // ablation (ranges not written): the fold's cost
    if (fixed && getenv("THESIA_STFT3_NOFOLD")) return launch3_k<NC, 1, C, INF, OUT_AMP_DB << 18, WVS>(a, s);
#endif
    constexpr int KDB = OUT_AMP_DB << 18, KRG = 1 << 21;
    if (fixed)
        return a.trk_range ? launch3_k<NC, 1, C, INF, KDB | KRG, WVS>(a, s) : launch3_k<NC, 1, C, INF, KDB, WVS>(a, s);
    return launch3_k<NC, 1, C, INF, 0, WVS>(a, s);
}

template <int NC>
static int launch3_nc(const StftLaunch& a, hipStream_t s) {
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch3_c<NC, 2, IN_S16>(a, s) : launch3_c<NC, 1, IN_S16>(a, s);
    return a.channels == 2 ? launch3_c<NC, 2, IN_F32>(a, s) : launch3_c<NC, 1, IN_F32>(a, s);
}

int stft3_lds_bytes(const StftLaunch& a) {
    if (stft3v_supports(a.n_fft, a.win, a.hop, a.in_format, a.channels)) return stft3v_lds_bytes(a);
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
    return ((n_fft == 256 || n_fft == 512 || n_fft == 1024 || n_fft == 2048) && win == n_fft &&
            hop * 4 == n_fft && (in_format == IN_F32 || in_format == IN_S16) &&
            (channels == 1 || channels == 2)) ||
           stft3v_supports(n_fft, win, hop, in_format, channels);  // the viewer geometries
}

int launch_stft3(const StftLaunch& a, hipStream_t s) {
    if (stft3v_supports(a.n_fft, a.win, a.hop, a.in_format, a.channels)) return launch_stft3v(a, s);
    if (a.win != a.n_fft || a.hop * 4 != a.n_fft) return -2;
    switch (a.n_fft / 2) {
        case 128: return launch3_nc<128>(a, s);
        case 256: return launch3_nc<256>(a, s);
        case 512: return launch3_nc<512>(a, s);
        case 1024: return launch3_nc<1024>(a, s);
        default: return -2;
    }
}

}  // namespace thesia
