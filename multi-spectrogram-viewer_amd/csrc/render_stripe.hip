// render_stripe.hip -- the display of a track in ONE pass: grey (display.rs:44-54) + vertical
// Lanczos3 + horizontal Lanczos3 (image 0.23.12 resize: vertical_sample into an f32 image, then
// horizontal_sample; display.rs:57) + colormap (display.rs:24-42), with the f32 intermediate
// [nheight, T] of the separable resize never written: it lives in registers for 8 frames.
//
// A block owns a strip of output columns [c0, c1) x 256 or 512 output rows of one track; lane =
// output row, and each wave (64 rows) runs on its own after the block has staged the strip's step
// table
// (no block barrier in the frame loop). A wave walks the strip's frames in 8-frame steps,
// ascending:
//   * the dB rows of a chunk of FC frames (the bins its rows' taps reach: a contiguous piece of
//     each frame row) are loaded into registers one chunk ahead, turned into grey values and
//     stored transposed into the wave's LDS tile [grey row][frame] once the chunk before is done;
//   * vertical: v[u] = sum_i grey[l_row + i][f_u] * wv_row[i] for the step's 8 frames, the row's
//     taps zero-padded to KV (registers), ds_read_b128 per tap and 4 frames;
//   * horizontal: the columns whose supports meet the step (at most A: accumulators acc[k] for
//     columns cs + k, in registers) take acc[k] += v[u] * w[u] for u ascending, with the step's
//     weights from LDS (the host regroups each column's taps by step, zero outside its support);
//   * a column whose support ends in the step is finished: colormap, its 3 bytes packed with
//     its neighbours' into the wave's RGB staging in LDS, which leaves as contiguous 48-byte row
//     pieces every 16 columns; the accumulators shift down one slot.
// Ring mode (HG > 0, round 6; render path 5, for groups with fewer than 3 frames per column): the
// horizontal slots are replaced by a per-lane LDS ring of the wave's vertical sums over the strip's
// last RING frames (each lane reads only its own row's entries: no cross-lane hazard); once a
// step has formed the last frame of a column's support, the column is summed over exactly its
// taps (HG float4 groups of weights staged per strip column, zero-padded; the ring mirrors its
// first 4 HG slots after its end so a column's frames are contiguous) and closed as above.
// Every sum runs in the reference's order (t = 0; t += x * w, no fused multiply-add: the kernel
// is built with -ffp-contract=off). The padded terms are (+0 weight) x (finite value) = +-0,
// which leave a sum's bits unchanged (a sum is never -0: it starts at +0 and x + -x rounds to
// +0), so the bytes equal the two-pass path's and the oracle's.
#include "kernels.hpp"
#include "display_common.hpp"

#include <cstdint>

namespace thesia {

namespace {

#ifdef THESIA_MARKS
#define SMARK(x) asm volatile("; MARK " #x)
#else
#define SMARK(x)
#endif

constexpr int kRgbStride = 13;  // dwords per row of a wave's RGB staging (16 columns = 12 dwords)
constexpr int kSumStride = 17;  // floats per row of a wave's finished sums (16 columns)
constexpr int kLutFloats = 32;  // the colormap as 10 x {stop i, stop i + 1} (8 bytes each)

__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }

// the values are formed here (not sunk past this point), and no memory access is moved across
// it: bounds the LDS reads in flight (their registers) where the compiler would hoist a whole
// step's worth
template <int N>
__device__ __forceinline__ void pin_mem(float (&a)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i]));
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void wave_sync() {  // cross-lane LDS ordering within the wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A accumulators (columns meeting a step), AW the step table's row stride (A rounded up to 4; its
// entries past A are zero and never read into a sum)
template <int KV, int A, int AW, int FC, int NPF, int WV, int HG = 0>
__global__ void __launch_bounds__(64 * WV) render_stripe_kernel(StripeLaunch L) {
    constexpr int kRows = 64 * WV;  // output rows per block (lane = row)
    constexpr bool kRing = HG > 0;
    constexpr int MIR = 4 * HG;  // ring slots mirrored after its end
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr int TS = FC + 4;   // tile row stride (floats): 16-byte rows for the b128 reads
    constexpr int SPC = FC / 8;  // steps per chunk
    const RenderDesc r = L.desc[blockIdx.z];
    // the grey values' (max, min): the device-side global range where the call has one
    const float gmax = r.grange ? r.grange[0] : L.max, gmin = r.grange ? r.grange[1] : L.min;
    const GreyMap gm(gmax, gmin);
    const uint32_t nw = r.nw;
    const uint32_t c0 = blockIdx.x * L.strip;
    if (c0 >= nw) return;  // block-uniform
    const uint32_t c1 = c0 + L.strip < nw ? c0 + L.strip : nw;
    const uint32_t R0 = blockIdx.y * kRows;
    const uint32_t nh = L.nh;
    if (R0 >= nh) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = rfl(tid >> 6);
    const uint32_t row = R0 + (uint32_t)tid;
    const bool live = row < nh;
    const uint32_t oz = r.oz;

    // LDS: colormap pairs (128 B) | the strip's steps' first columns hdr[hdr_cap] (padded to 16 B)
    // | their weights wts[wts_cap] ([step][frame][slot]) | per wave: tile[tile_cap][TS],
    // finished sums [64 rows][kSumStride] (also the RGB staging [64 rows][kRgbStride dwords])
    uint2* lut = reinterpret_cast<uint2*>(sm);
    int* hdr = reinterpret_cast<int*>(sm + kLutFloats);
    float* wts = reinterpret_cast<float*>(hdr + ((L.hdr_cap + 3) & ~3));
    const int ring_n = kRing ? L.ring : 0;  // a power of 2
    const int ring_slots = kRing ? ring_n + MIR + 1 : 0;  // (the last one: a dummy mirror target)
    const int wave_floats = L.tile_cap * TS + 64 * kSumStride + ring_slots * 64;
    float* tile = wts + L.wts_cap + wave * wave_floats;
    float* fsum = tile + L.tile_cap * TS;
    float* ring = fsum + 64 * kSumStride;  // ring mode: [slot][64 lanes]
    // the RGB staging reuses the sums' space (every lane has read its sums before it is written)
    uint32_t* rgbst = reinterpret_cast<uint32_t*>(fsum);

    // the strip's steps [s_lo, s_hi]: from the first column's first frame to the last column's last
    const int s_lo = r.hl[c0] >> 3;
    const int s_hi = (r.hl[c1 - 1] + r.hc[c1 - 1] - 1) >> 3;
    const int nst = s_hi - s_lo + 1;  // <= hdr_cap (host)
    const int* gh = r.hst + s_lo;
    const float* gw = r.hsw + (uint64_t)s_lo * 8 * AW;
    if (tid < 10) lut[tid] = colormap_pair(L.cmap, tid);
    if constexpr (kRing) {
        // the strip's columns: {first frame, last frame} and their taps, HG float4 per column
        // (zero-padded); hdr_cap >= 2 strip, wts_cap >= strip 4 HG (host)
        const int ncol = (int)(c1 - c0);
        for (int k = tid; k < ncol; k += kRows) {
            const int c = (int)c0 + k;
            hdr[2 * k] = r.hl[c];
            hdr[2 * k + 1] = r.hl[c] + r.hc[c] - 1;
        }
        for (int i = tid; i < ncol * 4 * HG; i += kRows) {
            const int k = i / (4 * HG), t = i - k * 4 * HG, c = (int)c0 + k;
            wts[i] = t < r.hc[c] ? r.hw[r.ho[c] + t] : 0.0f;
        }
    } else {
        for (int i = tid; i < nst; i += kRows) hdr[i] = gh[i];
        for (int i = tid; i < nst * 2 * AW; i += kRows)  // nst x 8 x AW floats <= wts_cap (host)
            reinterpret_cast<float4*>(wts)[i] = reinterpret_cast<const float4*>(gw)[i];
    }
    __syncthreads();  // the only block barrier: the waves run on their own from here

    // a finished column c: its sum into the lane's row of the wave's staging; every 16 columns
    // (or at c1) the row's 16 sums are colormapped and packed (3 bytes a pixel, 12 dwords), and
    // the wave's 64 rows leave as contiguous 48-byte row pieces
    const uint32_t wr0 = R0 + 64u * (uint32_t)wave;
    auto flush = [&](uint32_t c) {  // columns [c & ~15, c] of rows wr0 .. wr0 + 63
        const uint32_t cb = c & ~15u;
        const int n = (int)(c - cb) + 1;  // uniform
        // all 16 slots straight-line (their sum reads, then their LUT reads, each batch in flight
        // together): a partial piece's slots past n hold stale or unwritten sums, whose bytes
        // land past 3n in the row piece and are never stored
        float sv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) sv[k] = fsum[lane * kSumStride + k];
        uint32_t px[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) px[k] = colormap_rgb(sv[k], lut);
        // 16 pixels x 3 bytes -> 12 dwords (bytes 3k .. 3k + 2 of the row piece)
        uint32_t d[12];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t a = px[4 * q], b = px[4 * q + 1], e = px[4 * q + 2], f = px[4 * q + 3];
            d[3 * q] = a | (b << 24);
            d[3 * q + 1] = (b >> 8) | (e << 16);
            d[3 * q + 2] = (e >> 16) | (f << 8);
        }
        wave_sync();  // every lane's sums read
#pragma unroll
        for (int k = 0; k < 12; ++k) rgbst[lane * kRgbStride + k] = d[k];
        wave_sync();
        const int nbytes = 3 * n;  // per row
        const uint32_t rows = nh - wr0 < 64u ? nh - wr0 : 64u;
        uint8_t* gbase = L.rgb + r.rgb_off + ((uint64_t)wr0 * nw + cb) * 3;
        if (L.dword_rgb) {  // row pieces start 4-byte aligned (nw, rgb_off multiples of 4)
            const int nd = nbytes / 4;  // n is a multiple of 4 here
            for (int e = lane; e < (int)rows * nd; e += 64) {
                const int rr = e / nd, k = e - rr * nd;
                reinterpret_cast<uint32_t*>(gbase + (uint64_t)rr * nw * 3)[k] = rgbst[rr * kRgbStride + k];
            }
        } else {
            const uint8_t* sb = reinterpret_cast<const uint8_t*>(rgbst);
            for (int b = lane; b < (int)rows * nbytes; b += 64) {
                const int rr = b / nbytes, k = b - rr * nbytes;
                gbase[(uint64_t)rr * nw * 3 + k] = sb[rr * kRgbStride * 4 + k];
            }
        }
        wave_sync();
    };
#ifdef THESIA_EXPERIMENTS
    const int abl = L.abl;  // timing ablations: 1 no staging past chunk 0, 2 no emission, 4 no horizontal sums
#else
    constexpr int abl = 0;
#endif
    auto close_col = [&](uint32_t c, float t) {  // c in [c0, c1), ascending
        if (abl & 2) {
            if (t == 1.2345e-30f) fsum[lane] = t;  // keep the sums live
            return;
        }
        fsum[lane * kSumStride + (c & 15)] = t;
        if ((c & 15) == 15 || c + 1 == c1) flush(c);
    };

    // this wave's rows with vertical work: [rlo, rhi) (rows below oz take only the zero fill)
    const uint32_t rlo = wr0 > oz ? wr0 : oz;
    const uint32_t rhi = wr0 + 64 < nh ? wr0 + 64 : nh;
    if (wr0 >= nh) return;
    if (rlo >= rhi) {  // every row of the wave above the track's band: colormap(+0)
        for (uint32_t c = c0; c < c1; ++c) close_col(c, 0.0f);
        return;
    }
    // the wave's grey rows [ya, ya + nt): every tap of rows [rlo, rhi); the staged ones are those
    // inside the track's band [top, H) (bins H - 1 - y, contiguous in a frame row); the others
    // stay zero (the image's zero fill above the band, padded taps below it)
    const int H = (int)r.H, bins = (int)L.bins, top = H - bins;
    const int ya = r.vl[rlo];
    const int nt = r.vl[rhi - 1] + KV - ya;  // <= tile_cap (host)
    const int ys0 = ya > top ? ya : top;
    const int ys1 = ya + nt < H ? ya + nt : H;
    const int nb = ys1 > ys0 ? ys1 - ys0 : 0;  // staged bins per frame
    const int b_lo = H - ys1;                  // lowest staged bin
    const int tot = FC * nb;                   // <= 64 * NPF (host)
    const uint32_t mrec = nb > 1 ? (uint32_t)((0x100000000ull + (uint32_t)nb - 1) / (uint32_t)nb) : 0u;
    const uint32_t T = r.T;
    const float* sp = L.spec + r.spec_off;
    const int F0 = 8 * s_lo;
    for (int i = lane; i < L.tile_cap * TS; i += 64) tile[i] = 0.0f;

    // staging: element e of chunk k = (frame fi, staged bin bi), consecutive e = consecutive bins
    // of one frame (coalesced). Out-of-range elements are clamped to the last one and frames
    // past T to frame T - 1 (duplicate loads / identical stores; frames past T only ever meet
    // zero horizontal weights, so any finite value will do): no per-element branches
    float pf[NPF];
    // where the registers fit under 128 VGPRs (4 waves / SIMD), each staged element's place is
    // formed once per wave and kept for every chunk: pk[j] = its offset in the chunk's frame rows
    // (fi bins + bi < 2^16) | its float index in the wave's tile (< 2^16) << 16; the chunk's loads
    // take a uniform base, and frames past T read +0 through the buffer's range check (frames
    // past T only ever meet zero horizontal weights, and the grey value of +0 is finite). Otherwise the
    // (frame, bin) of each element is formed again per chunk, frames clamped to T - 1.
    constexpr bool kKeep = NPF == 8 || (KV <= 8 && A <= 12);
    uint32_t pk[kKeep ? NPF : 1];
    const uint32_t emax = (uint32_t)(tot > 0 ? tot - 1 : 0);
    const int q0 = H - 1 - b_lo - ya;  // tile row of staged bin bi: q0 - bi
    // the track's dB rows as a buffer resource: 32-bit byte offsets (a track's rows < 2^30
    // floats, host), one buffer_load per element
    const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(sp), (short)0, kKeep ? (int)(T * (uint32_t)bins * 4u) : -1, 0x00020000);
    if constexpr (kKeep) {
#pragma unroll
        for (int j = 0; j < NPF; ++j) {
            if (64 * j >= tot) break;  // uniform
            uint32_t e = (uint32_t)(lane + 64 * j);
            e = e < emax ? e : emax;
            const uint32_t fi = nb > 1 ? __umulhi(e, mrec) : e;
            const uint32_t bi = e - fi * (uint32_t)nb;
            pk[j] = (fi * (uint32_t)bins + bi) | ((uint32_t)((q0 - (int)bi) * TS + (int)fi) << 16);
        }
    }
    auto issue = [&](int k) {  // chunk k's dB values -> registers
        const uint32_t fb = (uint32_t)(F0 + k * FC);
        if constexpr (kKeep) {
            const uint32_t base = (fb * (uint32_t)bins + (uint32_t)b_lo) * 4u;  // uniform
#pragma unroll
            for (int j = 0; j < NPF; ++j) {
                if (64 * j >= tot) break;  // uniform
                pf[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    rsc, (pk[j] & 0xffffu) * 4u + base, 0, 0));
            }
            return;
        }
        // opaque per call: the element indices are formed per chunk, not hoisted out of the
        // frame loop into NPF x 3 registers held across it
        int li = lane;
        asm volatile("" : "+v"(li));
#pragma unroll
        for (int j = 0; j < NPF; ++j) {
            if (64 * j >= tot) break;  // uniform
            uint32_t e = (uint32_t)(li + 64 * j);
            e = e < emax ? e : emax;
            const uint32_t fi = nb > 1 ? __umulhi(e, mrec) : e;
            const uint32_t bi = e - fi * (uint32_t)nb;
            uint32_t f = fb + fi;
            f = f < T ? f : T - 1;
            pf[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rsc, (f * (uint32_t)bins + (uint32_t)b_lo + bi) * 4u, 0, 0));
        }
    };
    auto commit = [&](int) {  // registers -> grey values in the tile (its previous chunk read)
        float* t = tile;
        if constexpr (kKeep) {
#pragma unroll
            for (int j = 0; j < NPF; ++j) {
                if (64 * j >= tot) break;  // uniform
                t[pk[j] >> 16] = gm(pf[j]);
            }
            return;
        }
        int lc = lane;  // (recomputing: opaque, as in issue())
        asm volatile("" : "+v"(lc));
#pragma unroll
        for (int j = 0; j < NPF; ++j) {
            if (64 * j >= tot) break;  // uniform
            int fi, bi;
            {
                uint32_t e = (uint32_t)(lc + 64 * j);
                e = e < emax ? e : emax;
                const uint32_t f = nb > 1 ? __umulhi(e, mrec) : e;
                fi = (int)f;
                bi = (int)(e - f * (uint32_t)nb);
            }
            t[(q0 - bi) * TS + fi] = gm(pf[j]);
        }
    };

    // this lane's vertical taps (zero-padded to KV; rows without vertical work: all zero)
    const bool vrow = live && row >= oz;
    int q = 0;
    float wv[KV];
    {
        int n = 0;
        const float* w = r.vw;
        if (vrow) {
            q = r.vl[row] - ya;
            n = r.vc[row];
            w = r.vw + r.vo[row];
        }
#pragma unroll
        for (int i = 0; i < KV; ++i) wv[i] = i < n ? w[i] : 0.0f;
        // landed before the frame loop: a first use inside it would wait (vmcnt 0) for the
        // chunk prefetch issued behind these loads, every step
#pragma unroll
        for (int i = 0; i < KV; ++i) asm volatile("" : "+v"(wv[i]));
        asm volatile("" : "+v"(q));
    }

    const int nchunks = (nst + SPC - 1) / SPC;
    if constexpr (kRing) {  // finite ring entries (padded taps read them with +0 weights)
        for (int i = 0; i < ring_slots; ++i) ring[i * 64 + lane] = 0.0f;
    }
    if (nb) {
        issue(0);
        wave_sync();  // tile zeroed
        commit(0);
    }
    wave_sync();
    float acc[kRing ? 1 : A];
#pragma unroll
    for (int k = 0; k < (kRing ? 1 : A); ++k) acc[k] = 0.0f;
    uint32_t cc = c0;  // ring mode: the next column to close
    // slot a <-> column ca(s) + a of the step's table (columns before c0, finished by the strip
    // on the left, and from c1 on are summed too and never stored)
    for (int k = 0; k < nchunks; ++k) {
        SMARK(issue);
        if (k + 1 < nchunks && nb && !(abl & 1)) issue(k + 1);
        SMARK(steps);
        const float* t = tile + q * TS;
        for (int u8 = 0; u8 < SPC; ++u8) {
            const int si = k * SPC + u8;
            if (si >= nst) break;  // uniform
            const int ca = kRing ? 0 : rfl(hdr[si]);
            SMARK(vert);
            // vertical sums of the step's 8 frames (resize_v_px order), 4 frames at a time: one
            // ds_read_b128 per tap, a batch of taps' reads in flight
            float v[8];
            constexpr int KB = KV % 8 == 0 ? 8 : KV % 4 == 0 ? 4 : KV;  // taps per batch of reads (divides KV)
            static_assert(KV % KB == 0, "tap batches");
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const float* tq = t + 8 * u8 + 4 * hf;
                float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
#pragma unroll
                for (int i0 = 0; i0 < KV; i0 += KB) {
                    float4 g[KB];
#pragma unroll
                    for (int i = 0; i < KB; ++i) g[i] = *reinterpret_cast<const float4*>(tq + (i0 + i) * TS);
#pragma unroll
                    for (int i = 0; i < KB; ++i) {
                        const float w = wv[i0 + i];
                        a0 = a0 + g[i].x * w;
                        a1 = a1 + g[i].y * w;
                        a2 = a2 + g[i].z * w;
                        a3 = a3 + g[i].w * w;
                    }
                    float ap[4] = {a0, a1, a2, a3};
                    pin_mem(ap);  // bound the reads in flight (registers)
                    a0 = ap[0]; a1 = ap[1]; a2 = ap[2]; a3 = ap[3];
                }
                v[4 * hf] = a0;
                v[4 * hf + 1] = a1;
                v[4 * hf + 2] = a2;
                v[4 * hf + 3] = a3;
            }
            if constexpr (kRing) {
                // the step's frames into the lane's ring (slot f mod RING, mirrored after the end
                // for f mod RING < 4 HG), then every column whose support ends by this step's last
                // frame: t = 0; t += v[f] * w over its taps, ascending (resize_h's order; the
                // padded taps add (+0 weight) x (finite entry) = +-0)
                SMARK(ring);
                const int fb = F0 + 8 * si;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int sl = (fb + u) & (ring_n - 1);  // uniform
                    const int ml = sl < MIR ? sl + ring_n : ring_n + MIR;
                    ring[sl * 64 + lane] = v[u];
                    ring[ml * 64 + lane] = v[u];
                }
                const int fend = fb + 7;
                while (cc < c1) {  // uniform
                    const int last = rfl(hdr[2 * (cc - c0) + 1]);
                    if (last > fend) break;
                    const int s0 = rfl(hdr[2 * (cc - c0)]) & (ring_n - 1);
                    const float* rb = ring + s0 * 64 + lane;
                    const float4* wb = reinterpret_cast<const float4*>(wts) + (cc - c0) * HG;
                    float xs[4 * HG];
#pragma unroll
                    for (int i = 0; i < 4 * HG; ++i) xs[i] = rb[i * 64];
                    float4 ws[HG];
#pragma unroll
                    for (int g = 0; g < HG; ++g) ws[g] = wb[g];
                    float t = 0.0f;
#pragma unroll
                    for (int g = 0; g < HG; ++g) {
                        t = t + xs[4 * g] * ws[g].x;
                        t = t + xs[4 * g + 1] * ws[g].y;
                        t = t + xs[4 * g + 2] * ws[g].z;
                        t = t + xs[4 * g + 3] * ws[g].w;
                    }
                    close_col(cc, t);
                    ++cc;
                }
                continue;
            }
            // horizontal: every slot's chain takes the step's frames in ascending order (the
            // resize_h order; slots outside a column's support add (+0 weight) x v = +-0); the
            // weights of frame u + 1 are read while frame u is summed
            SMARK(horiz);
            constexpr int A4 = (A + 3) / 4;  // float4 weight reads per frame
            const float4* wu = reinterpret_cast<const float4*>(wts + si * 8 * AW);
            float4 xc[A4];
#pragma unroll
            for (int a4 = 0; a4 < A4; ++a4) xc[a4] = wu[a4];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                float4 xn[A4];
                if (u + 1 < 8) {
#pragma unroll
                    for (int a4 = 0; a4 < A4; ++a4) xn[a4] = wu[(u + 1) * (AW / 4) + a4];
                }
                if (!(abl & 4)) {
#pragma unroll
                    for (int a = 0; a < A; ++a) {
                        const float4 x = xc[a / 4];
                        const float wgt = (a & 3) == 0 ? x.x : (a & 3) == 1 ? x.y : (a & 3) == 2 ? x.z : x.w;
                        acc[a] = acc[a] + v[u] * wgt;
                    }
                } else {
                    acc[u & (A - 1) & 7] += v[u];  // keep the vertical sums live
                }
                pin_mem(acc);
                if (u + 1 < 8) {
#pragma unroll
                    for (int a4 = 0; a4 < A4; ++a4) xc[a4] = xn[a4];
                }
            }
            // the columns whose supports end in this step (all of the strip's at its last):
            // finished, the slots shift down
            SMARK(close);
            const int cn = si + 1 < nst ? rfl(hdr[si + 1]) : (int)c1;
            for (int c = ca; c < cn; ++c) {  // uniform
                if (c >= (int)c0 && c < (int)c1) close_col((uint32_t)c, acc[0]);
#pragma unroll
                for (int a = 0; a + 1 < A; ++a) acc[a] = acc[a + 1];
                acc[A - 1] = 0.0f;
            }
        }
        SMARK(commit);
        if (k + 1 < nchunks && nb && !(abl & 1)) {
            wave_sync();  // every lane's reads of the buffer chunk k + 1 overwrites are done
            commit(k + 1);
            wave_sync();
        }
    }
}

template <int KV, int A, int AW, int FC, int NPF, int HG = 0>
const void* stripe_kernel(int waves) {
    return waves == 8 ? reinterpret_cast<const void*>(render_stripe_kernel<KV, A, AW, FC, NPF, 8, HG>)
                      : reinterpret_cast<const void*>(render_stripe_kernel<KV, A, AW, FC, NPF, 4, HG>);
}

}  // namespace

int render_stripe_lds_bytes(int fc, int tile_cap, int hdr_cap, int wts_cap, int waves, int ring_slots) {
    return (kLutFloats + ((hdr_cap + 3) & ~3) + wts_cap +
            waves * (tile_cap * (fc + 4) + 64 * kSumStride + 64 * ring_slots)) * 4;
}

int launch_render_stripe(const StripeLaunch& L, hipStream_t s) {
    if (L.n == 0 || L.nh == 0) return 0;
    if (L.n > 65535 || L.strip == 0 || (L.strip & 15) || (L.waves != 4 && L.waves != 8)) return -2;
    if (L.hg && (L.ring < 8 || (L.ring & (L.ring - 1)))) return -2;
    const void* kern = nullptr;
    // ring mode (render path 5): KV 7 / 8 / 12 / 16 x HG 2 / 3 / 4 / 6 tap groups, FC 16 or 8
#define THESIA_STRIPE_RING(KV_, HG_, FC_)                                                      \
    if (L.hg == HG_ && L.kv == KV_ && L.fc == FC_ && L.npf == 16)                            \
        kern = stripe_kernel<KV_, 1, 4, FC_, 16, HG_>(L.waves);
#define THESIA_STRIPE_RING_KV(KV_)                                                             \
    THESIA_STRIPE_RING(KV_, 2, 16) THESIA_STRIPE_RING(KV_, 3, 16) THESIA_STRIPE_RING(KV_, 4, 16)   \
    THESIA_STRIPE_RING(KV_, 6, 16) THESIA_STRIPE_RING(KV_, 2, 8) THESIA_STRIPE_RING(KV_, 3, 8)     \
    THESIA_STRIPE_RING(KV_, 4, 8) THESIA_STRIPE_RING(KV_, 6, 8)
    if (L.hg) {
        THESIA_STRIPE_RING_KV(7) THESIA_STRIPE_RING_KV(8) THESIA_STRIPE_RING_KV(12) THESIA_STRIPE_RING_KV(16)
    }
#undef THESIA_STRIPE_RING_KV
#undef THESIA_STRIPE_RING
    // the instances (host plan_stripe picks among them): KV 7 / 8 (the groups that upsample
    // vertically: Lanczos3's 6-7 taps per row, 7 where no row has 8) with 8 / 9 / 10 / 12 (and for
    // KV 8, 16) accumulators (9 and 10 on the 12-wide step table: the 48 kHz / 512 and 22.05 kHz /
    // 256 C5 groups meet at most 9 columns per step); KV 12 / 16 (downsampling) with 16
#define THESIA_STRIPE(KV_, A_, AW_, FC_, NPF_)                                                     \
    if (!L.hg && L.kv == KV_ && L.acc == A_ && L.slots == AW_ && L.fc == FC_ && L.npf == NPF_)    \
        kern = stripe_kernel<KV_, A_, AW_, FC_, NPF_>(L.waves);
    THESIA_STRIPE(7, 8, 8, 16, 8) THESIA_STRIPE(7, 8, 8, 16, 16) THESIA_STRIPE(7, 8, 8, 8, 16)
    THESIA_STRIPE(7, 9, 12, 16, 8) THESIA_STRIPE(7, 9, 12, 16, 16) THESIA_STRIPE(7, 9, 12, 8, 16)
    THESIA_STRIPE(7, 10, 12, 16, 8) THESIA_STRIPE(7, 10, 12, 16, 16) THESIA_STRIPE(7, 10, 12, 8, 16)
    THESIA_STRIPE(7, 12, 12, 16, 8) THESIA_STRIPE(7, 12, 12, 16, 16) THESIA_STRIPE(7, 12, 12, 8, 16)
    THESIA_STRIPE(8, 8, 8, 16, 8) THESIA_STRIPE(8, 8, 8, 16, 16) THESIA_STRIPE(8, 8, 8, 8, 16)
    THESIA_STRIPE(8, 9, 12, 16, 8) THESIA_STRIPE(8, 9, 12, 16, 16) THESIA_STRIPE(8, 9, 12, 8, 16)
    THESIA_STRIPE(8, 10, 12, 16, 8) THESIA_STRIPE(8, 10, 12, 16, 16) THESIA_STRIPE(8, 10, 12, 8, 16)
    THESIA_STRIPE(8, 12, 12, 16, 8) THESIA_STRIPE(8, 12, 12, 16, 16) THESIA_STRIPE(8, 12, 12, 8, 16)
    THESIA_STRIPE(8, 16, 16, 16, 8) THESIA_STRIPE(8, 16, 16, 16, 16) THESIA_STRIPE(8, 16, 16, 8, 16)
    THESIA_STRIPE(12, 16, 16, 16, 16) THESIA_STRIPE(12, 16, 16, 8, 16)
    THESIA_STRIPE(16, 16, 16, 16, 16) THESIA_STRIPE(16, 16, 16, 8, 16)
#undef THESIA_STRIPE
    if (!kern) return -2;
    const int lds = render_stripe_lds_bytes(L.fc, L.tile_cap, L.hdr_cap, L.wts_cap, L.waves,
                                            L.hg ? L.ring + 4 * L.hg + 1 : 0);
    if (lds > 163840) return -2;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    const uint32_t rows = 64u * (uint32_t)L.waves;
    const dim3 grid((L.nw_max + L.strip - 1) / L.strip, (L.nh + rows - 1) / rows, L.n);
    StripeLaunch a = L;
    void* args[] = {&a};
    if (hipLaunchKernel(kern, grid, dim3(rows), args, lds, s) != hipSuccess) return -1;
    return 0;
}

}  // namespace thesia
