// stft3v_kernels.hip -- the streaming kernel (stft3_kernel.hpp) at the viewer's own geometries:
// win = round(40 ms sr / 4) 4 <= n_fft = next_pow2(win), hop = win / 4 (lib.rs:43-46,93-99;
// SURVEY.md §8 viewer-defaults row). The hop of hop/2 points is HQ rows of L points plus rem
// points, rem = 0 or L/2 for every rate with an even hop:
//   48 kHz    1920 / 480 / 2048: NC 1024, L 32, 240 points = 7 rows + 16
//   24 kHz     960 / 240 / 1024: NC  512, L 16, 120 points = 7 rows + 8
//   16 kHz     640 / 160 / 1024: NC  512, L 16,  80 points = 5 rows
//    8 kHz     320 /  80 /  512: NC  256, L 16,  40 points = 2 rows + 8
// and the odd hops (VODD: streams in pairs interleaving the frames, a stream's hop 2 hop samples,
// odd frames on the point grid shifted by one sample):
//   44.1 kHz  1764 / 441 / 2048: NC 1024, L 32, 441 points a stream hop = 13 rows + 25
//   22.05 kHz  884 / 221 / 1024: NC  512, L 16, 221 points = 13 rows + 13
// (odd hops: vector loads at every sample, dword-aligned or, int16 mono, 2-byte). Any geometry
// with an even win <= n_fft and one of these row counts runs here.
#include "stft3_kernel.hpp"

namespace thesia {

namespace {

template <int NC, int OK, int VAR, int WV>
int lds3v_bytes(const StftLaunch& a) {
    return (Geo3<NC, WV>::BASE_FLOATS_OK(stage_rows(OK, VAR), OK) +
            (OK == 2 ? (a.mel4_rows * 4 + a.mel4_rounds) * Geo2<NC>::L + 2 * a.mel4_rounds : 0)) * 4;
}

template <int NC, int HQ, int OK, int C, int INF, int VAR, int WV, int VODD>
int launch3v_k(const StftLaunch& a, hipStream_t stream) {
    constexpr int kBlock = 64 * WV;
    const int lds = lds3v_bytes<NC, OK, VAR, WV>(a);
    if (lds > 163840) return -2;
    auto kern = stft3_kernel<NC, OK, C, INF, VAR, WV, HQ, VODD>;
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

template <int NC, int HQ, int C, int INF, int VODD>
int launch3v_c(const StftLaunch& a, hipStream_t s) {
    // as launch3_c: complex rows as whole 128-byte lines (VAR 2048; per row, VAR 1024, where a
    // stream's rows are not contiguous), 12-wave blocks for mono linear kinds at n_fft <= 512
    constexpr int WVS = NC <= 256 && C == 1 ? 12 : kWaves;
    if (a.out_kind == OUT_COMPLEX) return launch3v_k<NC, HQ, 0, C, INF, VODD ? 1024 : 2048, kWaves, VODD>(a, s);
    if (a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB) return launch3v_k<NC, HQ, 2, C, INF, 0, kWaves, VODD>(a, s);
    // amp dB rows without the range fold (the viewer's): the kind at compile time (VAR bits 18-20)
    bool fixed = a.out_kind == OUT_AMP_DB && !a.trk_range;
#ifdef THESIA_EXPERIMENTS
    if (getenv("THESIA_STFT3_RTKIND")) fixed = false;  // A/B: the run-time kind
#endif
    if (fixed) return launch3v_k<NC, HQ, 1, C, INF, OUT_AMP_DB << 18, WVS, VODD>(a, s);
    return launch3v_k<NC, HQ, 1, C, INF, 0, WVS, VODD>(a, s);
}

template <int NC, int HQ>
int launch3v_nc(const StftLaunch& a, hipStream_t s) {
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch3v_c<NC, HQ, 2, IN_S16, 0>(a, s) : launch3v_c<NC, HQ, 1, IN_S16, 0>(a, s);
    return a.channels == 2 ? launch3v_c<NC, HQ, 2, IN_F32, 0>(a, s) : launch3v_c<NC, HQ, 1, IN_F32, 0>(a, s);
}

template <int NC, int HQ>
int launch3v_nc_odd(const StftLaunch& a, hipStream_t s) {
    if (a.in_format == IN_S16)
        return a.channels == 2 ? launch3v_c<NC, HQ, 2, IN_S16, 1>(a, s) : launch3v_c<NC, HQ, 1, IN_S16, 1>(a, s);
    return a.channels == 2 ? launch3v_c<NC, HQ, 2, IN_F32, 1>(a, s) : launch3v_c<NC, HQ, 1, IN_F32, 1>(a, s);
}

// the instantiated (NC, rows per stream hop) pairs; odd hops: a stream hop of 2 hop samples
int view_rows(int n_fft, int hop) {
    const int NC = n_fft / 2;
    const int L = NC == 1024 ? Geo2<1024>::L : NC == 512 ? Geo2<512>::L : NC == 256 ? Geo2<256>::L : 0;
    if (!L || hop <= 0) return 0;
    if (hop % 2) {
        const int hq = hop / L;
        return (NC == 1024 || NC == 512) && hq == 13 ? hq : 0;
    }
    const int hq = (hop / 2) / L;
    const bool ok = (NC == 1024 && hq == 7) || (NC == 512 && (hq == 7 || hq == 5)) || (NC == 256 && hq == 2);
    return ok ? hq : 0;
}

}  // namespace

bool stft3v_supports(int n_fft, int win, int hop, int in_format, int channels) {
    // the streaming start rule (frame start = t hop - n_fft / 2) needs win / 2 + pad_left =
    // n_fft / 2, i.e. an even win (lib.rs:400-401); the canonical geometry is stft3's own
    return view_rows(n_fft, hop) > 0 && win <= n_fft && win % 2 == 0 && win >= 2 &&
           !(win == n_fft && hop * 4 == n_fft) && (in_format == IN_F32 || in_format == IN_S16) &&
           (channels == 1 || channels == 2);
}

int stft3v_lds_bytes(const StftLaunch& a) {
    const bool mel = a.out_kind == OUT_MEL || a.out_kind == OUT_MEL_AMP_DB;
    const int ok = a.out_kind == OUT_COMPLEX ? 0 : mel ? 2 : 1;
    switch (a.n_fft / 2) {
        case 256: return ok == 0 ? lds3v_bytes<256, 0, 2048, kWaves>(a) : ok == 1 ? lds3v_bytes<256, 1, 0, kWaves>(a) : lds3v_bytes<256, 2, 0, kWaves>(a);
        case 512: return ok == 0 ? lds3v_bytes<512, 0, 2048, kWaves>(a) : ok == 1 ? lds3v_bytes<512, 1, 0, kWaves>(a) : lds3v_bytes<512, 2, 0, kWaves>(a);
        case 1024: return ok == 0 ? lds3v_bytes<1024, 0, 2048, kWaves>(a) : ok == 1 ? lds3v_bytes<1024, 1, 0, kWaves>(a) : lds3v_bytes<1024, 2, 0, kWaves>(a);
        default: return 1 << 30;
    }
}

int launch_stft3v(const StftLaunch& a, hipStream_t s) {
    switch (a.n_fft / 2 * 16 + view_rows(a.n_fft, a.hop)) {
        case 1024 * 16 + 7: return launch3v_nc<1024, 7>(a, s);
        case 512 * 16 + 7: return launch3v_nc<512, 7>(a, s);
        case 512 * 16 + 5: return launch3v_nc<512, 5>(a, s);
        case 256 * 16 + 2: return launch3v_nc<256, 2>(a, s);
        case 1024 * 16 + 13: return launch3v_nc_odd<1024, 13>(a, s);
        case 512 * 16 + 13: return launch3v_nc_odd<512, 13>(a, s);
        default: return -2;
    }
}

}  // namespace thesia
