// render_stripe.hip -- the display of a track in ONE pass: grey (display.rs:44-54) + vertical
// Lanczos3 + horizontal Lanczos3 (image 0.23.12 resize: vertical_sample into an f32 image, then
// horizontal_sample; display.rs:57) + colormap (display.rs:24-42), with the f32 intermediate
// [nheight, T] of the separable resize never written: it lives in registers for 8 frames.
//
// A block owns a strip of output columns [c0, c1) x 256 output rows of one track; lane = output
// row. It walks the strip's frames in 8-frame steps, ascending:
//   * the dB rows of a chunk of FC frames (the bins its rows' taps reach: a contiguous piece of
//     each frame row) are loaded into registers one chunk ahead, turned into grey values and
//     stored transposed into an LDS tile [grey row][frame] (double-buffered, one barrier per
//     chunk);
//   * vertical: v[u] = sum_i grey[l_row + i][f_u] * wv_row[i] for the step's 8 frames, the row's
//     taps zero-padded to KV (registers), two ds_read_b128 per tap;
//   * horizontal: the columns whose supports meet the step (at most A: accumulators acc[k] for
//     columns cs + k, in registers) take acc[k] += v[u] * w[u] for u ascending, with the step's
//     weights from LDS (the host regroups each column's taps by step, zero outside its support);
//   * a column whose support ends in the step is finished: colormap, its 3 bytes packed with
//     its neighbours', the accumulators shift down one slot.
// Every sum runs in the reference's order (t = 0; t += x * w, no fused multiply-add: the kernel
// is built with -ffp-contract=off). The padded terms are (+0 weight) x (finite value) = +-0,
// which leave a sum's bits unchanged (a sum is never -0: it starts at +0 and x + -x rounds to
// +0), so the bytes equal the two-pass path's and the oracle's.
#include "kernels.hpp"
#include "display_common.hpp"

#include <cstdint>

namespace thesia {

namespace {

constexpr int kRows = 256;  // output rows per block (lane = row)
constexpr int kPf = 16;     // staged dB values per thread and chunk (registers)

__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }

// the 12 RGB bytes of 4 consecutive columns of one row, packed into 3 dwords
struct Pack {
    uint32_t d0 = 0, d1 = 0, d2 = 0;
    __device__ __forceinline__ void put(int p, const uint8_t* px) {  // p = column & 3 (uniform)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const int o = 3 * p + ch;
            const uint32_t v = (uint32_t)px[ch] << (8 * (o & 3));
            if ((o >> 2) == 0) d0 |= v;
            else if ((o >> 2) == 1) d1 |= v;
            else d2 |= v;
        }
    }
};

template <int KV, int A, int FC>
__global__ void __launch_bounds__(256) render_stripe_kernel(StripeLaunch L) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr int TS = FC + 4;  // tile row stride (floats): 16-byte rows for the b128 reads
    constexpr int SPC = FC / 8;  // steps per chunk
    const RenderDesc r = L.desc[blockIdx.z];
    const uint32_t nw = r.nw;
    const uint32_t c0 = blockIdx.x * L.strip;
    if (c0 >= nw) return;  // block-uniform
    const uint32_t c1 = c0 + L.strip < nw ? c0 + L.strip : nw;
    const uint32_t R0 = blockIdx.y * kRows;
    const uint32_t nh = L.nh;
    if (R0 >= nh) return;
    const int tid = threadIdx.x;
    const int wave = rfl(tid >> 6);
    const uint32_t row = R0 + (uint32_t)tid;
    const bool live = row < nh;
    const uint32_t oz = r.oz;
    uint8_t* orow = L.rgb + r.rgb_off + (uint64_t)row * nw * 3;

    uint8_t* cm = reinterpret_cast<uint8_t*>(sm);  // 32 B
    if (tid < 30) cm[tid] = L.cmap[tid];

    // finished column c of this lane: colormap, pack, store every 4 columns (or at c1 - 1)
    Pack pk;
    auto emit = [&](uint32_t c, float t) {
        uint8_t px[3];
        colormap_px(t, cm, px);
        const int p = (int)(c & 3);
        pk.put(p, px);
        if (p == 3 || c + 1 == c1) {
            if (live) {
                uint8_t* o = orow + (uint64_t)(c & ~3u) * 3;
                if (L.dword_rgb) {  // 12 bytes at a 4-byte aligned address
                    uint32_t* o4 = reinterpret_cast<uint32_t*>(o);
                    o4[0] = pk.d0;
                    o4[1] = pk.d1;
                    o4[2] = pk.d2;
                } else {
                    const uint32_t w[3] = {pk.d0, pk.d1, pk.d2};
                    for (int b = 0; b < 3 * (p + 1); ++b) o[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
                }
            }
            pk = Pack{};
        }
    };

    // rows with vertical work: [rlo, rhi) (rows below oz take only the zero fill: +0 sums)
    const uint32_t rlo = R0 > oz ? R0 : oz;
    const uint32_t rhi = R0 + kRows < nh ? R0 + kRows : nh;
    __syncthreads();  // colormap bytes
    if (rlo >= rhi) {  // the whole block is above the track's band: colormap(+0) everywhere
        for (uint32_t c = c0; c < c1; ++c) emit(c, 0.0f);
        return;
    }
    // this wave has no row with vertical work (every row above the band, or past the image)
    const uint32_t wr0 = R0 + 64u * (uint32_t)wave;
    const bool wskip = wr0 + 63 < oz || wr0 >= nh;

    // LDS: colormap (32 B = 8 floats) | tile[2][tile_cap][TS] | hdr[hdr_cap] | wts[wts_cap]
    float* tile = sm + 8;
    int4* hdr = reinterpret_cast<int4*>(tile + 2 * L.tile_cap * TS);
    float* wts = reinterpret_cast<float*>(hdr + L.hdr_cap);

    // the strip's steps [s_lo, s_hi]: from the first column's first frame to the last column's last
    const int s_lo = r.hl[c0] >> 3;
    const int s_hi = (r.hl[c1 - 1] + r.hc[c1 - 1] - 1) >> 3;
    const int nst = s_hi - s_lo + 1;  // <= hdr_cap (host)
    const int4* gh = reinterpret_cast<const int4*>(r.hst) + s_lo;
    const int w0 = gh[0].z;
    const int wend = gh[nst - 1].z + 8 * gh[nst - 1].y;  // wend - w0 <= wts_cap (host)
    for (int i = tid; i < nst; i += 256) hdr[i] = gh[i];
    for (int i = tid; i < wend - w0; i += 256) wts[i] = r.hsw[w0 + i];

    // the block's grey rows [ya, ya + nt): every tap of rows [rlo, rhi); the staged ones are
    // those inside the track's band [top, H) (bins H - 1 - y, contiguous in a frame row); the
    // others stay zero (the image's zero fill above the band, and padded taps below it)
    const int H = (int)r.H, bins = (int)L.bins, top = H - bins;
    const int ya = r.vl[rlo];
    const int nt = r.vl[rhi - 1] + KV - ya;  // <= tile_cap (host)
    const int ys0 = ya > top ? ya : top;
    const int ys1 = ya + nt < H ? ya + nt : H;
    const int nb = ys1 > ys0 ? ys1 - ys0 : 0;  // staged bins per frame
    const int b_lo = H - ys1;                  // lowest staged bin
    const int tot = FC * nb;                   // <= 256 * kPf (host)
    const uint32_t mrec = nb > 1 ? (uint32_t)((0x100000000ull + (uint32_t)nb - 1) / (uint32_t)nb) : 0u;
    const uint32_t T = r.T;
    const float* sp = L.spec + r.spec_off;
    const int F0 = 8 * s_lo;
    for (int i = tid; i < 2 * nt * TS; i += 256) {  // both buffers: rows [0, nt)
        const int b = i / (nt * TS), e = i - b * nt * TS;
        tile[b * L.tile_cap * TS + e] = 0.0f;
    }

    float pf[kPf];
    auto issue = [&](int k) {  // chunk k's dB values -> registers
        const int fb = F0 + k * FC;
#pragma unroll
        for (int j = 0; j < kPf; ++j) {
            if (256 * j >= tot) break;  // uniform
            const uint32_t e = (uint32_t)(tid + 256 * j);
            float v = 0.0f;
            if ((int)e < tot) {
                const uint32_t fi = nb > 1 ? __umulhi(e, mrec) : e;
                const uint32_t bi = e - fi * (uint32_t)nb;
                const uint32_t f = (uint32_t)fb + fi;
                if (f < T) v = sp[(uint64_t)f * bins + (uint32_t)b_lo + bi];
            }
            pf[j] = v;
        }
    };
    auto commit = [&](int k) {  // registers -> grey values in tile buffer k & 1
        float* t = tile + (k & 1) * L.tile_cap * TS;
        const int fb = F0 + k * FC;
        // the element indices are formed again here, not kept from issue() across the steps
        int tidc = tid;
        asm volatile("" : "+v"(tidc));
#pragma unroll
        for (int j = 0; j < kPf; ++j) {
            if (256 * j >= tot) break;  // uniform
            const uint32_t e = (uint32_t)(tidc + 256 * j);
            if ((int)e < tot) {
                const uint32_t fi = nb > 1 ? __umulhi(e, mrec) : e;
                const uint32_t bi = e - fi * (uint32_t)nb;
                const int q = H - 1 - (b_lo + (int)bi) - ya;
                t[q * TS + (int)fi] = (uint32_t)fb + fi < T ? grey_of(pf[j], L.max, L.min) : 0.0f;
            }
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
    }

    const int nchunks = (nst + SPC - 1) / SPC;
    issue(0);
    __syncthreads();  // tile zeroed
    commit(0);
    float acc[A];
#pragma unroll
    for (int k = 0; k < A; ++k) acc[k] = 0.0f;
    int cs = (int)c0;  // accumulator k <-> column cs + k
    for (int k = 0; k < nchunks; ++k) {
        __syncthreads();  // chunk k in its buffer; chunk k - 1's readers done with the other one
        if (k + 1 < nchunks) issue(k + 1);
        if (!wskip) {
            const float* t = tile + (k & 1) * L.tile_cap * TS + q * TS;
            for (int u8 = 0; u8 < SPC; ++u8) {
                const int si = k * SPC + u8;
                if (si >= nst) break;  // uniform
                // vertical sums of the step's 8 frames (resize_v_px order)
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = 0.0f;
                const float* tq = t + 8 * u8;
#pragma unroll
                for (int i = 0; i < KV; ++i) {
                    const float4 g0 = *reinterpret_cast<const float4*>(tq + i * TS);
                    const float4 g1 = *reinterpret_cast<const float4*>(tq + i * TS + 4);
                    v[0] = v[0] + g0.x * wv[i];
                    v[1] = v[1] + g0.y * wv[i];
                    v[2] = v[2] + g0.z * wv[i];
                    v[3] = v[3] + g0.w * wv[i];
                    v[4] = v[4] + g1.x * wv[i];
                    v[5] = v[5] + g1.y * wv[i];
                    v[6] = v[6] + g1.z * wv[i];
                    v[7] = v[7] + g1.w * wv[i];
                }
                // horizontal: the step's columns [cs, ce), frames ascending (resize_h order)
                const int4 h = hdr[si];
                const int ca = rfl(h.x), na = rfl(h.y), wo = rfl(h.z) - w0;
                const int ce = ca + na < (int)c1 ? ca + na : (int)c1;
                const float* wb = wts + wo + 8 * (cs - ca);
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    if (cs + a < ce) {  // uniform
                        const float4 x0 = *reinterpret_cast<const float4*>(wb + 8 * a);
                        const float4 x1 = *reinterpret_cast<const float4*>(wb + 8 * a + 4);
                        float s = acc[a];
                        s = s + v[0] * x0.x;
                        s = s + v[1] * x0.y;
                        s = s + v[2] * x0.z;
                        s = s + v[3] * x0.w;
                        s = s + v[4] * x1.x;
                        s = s + v[5] * x1.y;
                        s = s + v[6] * x1.z;
                        s = s + v[7] * x1.w;
                        acc[a] = s;
                    }
                }
                // the columns whose supports end in this step: finished, slots shift down
                int cn = (int)c1;
                if (si + 1 < nst) {
                    const int nx = rfl(hdr[si + 1].x);
                    cn = nx > (int)c0 ? nx : (int)c0;
                }
                while (cs < cn) {  // uniform
                    emit((uint32_t)cs, acc[0]);
#pragma unroll
                    for (int a = 0; a + 1 < A; ++a) acc[a] = acc[a + 1];
                    acc[A - 1] = 0.0f;
                    ++cs;
                }
            }
        }
        if (k + 1 < nchunks) commit(k + 1);
    }
    if (wskip && live && row < oz)  // rows above the band: colormap(+0)
        for (uint32_t c = c0; c < c1; ++c) emit(c, 0.0f);
}

template <int KV, int A, int FC>
const void* stripe_kernel() {
    return reinterpret_cast<const void*>(render_stripe_kernel<KV, A, FC>);
}

}  // namespace

int render_stripe_lds_bytes(int fc, int tile_cap, int hdr_cap, int wts_cap) {
    return 32 + 2 * tile_cap * (fc + 4) * 4 + hdr_cap * 16 + wts_cap * 4;
}

int launch_render_stripe(const StripeLaunch& L, hipStream_t s) {
    if (L.n == 0 || L.nh == 0) return 0;
    if (L.n > 65535 || L.strip == 0 || (L.strip & 3)) return -2;
    const void* kern = nullptr;
#define THESIA_STRIPE(KV_, A_, FC_) \
    if (L.kv == KV_ && L.slots == A_ && L.fc == FC_) kern = stripe_kernel<KV_, A_, FC_>();
    THESIA_STRIPE(8, 8, 16) THESIA_STRIPE(8, 16, 16) THESIA_STRIPE(8, 16, 8)
    THESIA_STRIPE(12, 16, 16) THESIA_STRIPE(12, 16, 8)
    THESIA_STRIPE(16, 16, 16) THESIA_STRIPE(16, 16, 8)
#undef THESIA_STRIPE
    if (!kern) return -2;
    const int lds = render_stripe_lds_bytes(L.fc, L.tile_cap, L.hdr_cap, L.wts_cap);
    if (lds > 163840) return -2;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    const dim3 grid((L.nw_max + L.strip - 1) / L.strip, (L.nh + kRows - 1) / kRows, L.n);
    StripeLaunch a = L;
    void* args[] = {&a};
    if (hipLaunchKernel(kern, grid, dim3(256), args, lds, s) != hipSuccess) return -1;
    return 0;
}

}  // namespace thesia
