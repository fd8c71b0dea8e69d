// row_pattern.hip -- the complex-output STFT kernel's memory pattern with the arithmetic taken
// out (diagnosis of its box-to-box time spread). Geometry of the C4 shard:
// 2 813 000 frames; per frame a 4 096-byte hop of input read (8 float4 per lane of a 32-lane
// frame) and an 8 200-byte row of 1 025 float2 written. 256 blocks x 8 waves x 2 streams; a
// stream walks consecutive frames, so its rows are contiguous. Row store patterns:
//   lane8  -- lane-wise 8-byte stores (the shipped kernel)
//   b128   -- 16-byte aligned float4 stores inside each row, the row's partial chunks scalar
//   lines  -- whole 128-byte lines only (the line two rows share written once, with the later
//             row); a stream's first and last lines partial
// plus the copy ceilings on the same byte counts: read 1 : write 2 as two contiguous write
// streams, and a pure fill. Build: hipcc --offload-arch=gfx950 -O3 row_pattern.hip -o row_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint64_t TF = 2813000, RF = 2050;  // frames, floats per row
constexpr int STREAMS = 256 * 16;

__device__ __forceinline__ float hop_sum(const float4* in, uint64_t g, int j) {
    const float4* src = in + g * 256 + j;  // 4 096 B per frame
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float4 v = src[32 * q];
        s += v.x + v.y + v.z + v.w;
    }
    return s;
}

template <int MODE>
__global__ void __launch_bounds__(512) rows(const float4* __restrict__ in, float* __restrict__ out, uint64_t fps) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, slot = lane >> 5, j = lane & 31;
    const uint64_t stream = (uint64_t)blockIdx.x * 16 + wave * 2 + slot;
    const uint64_t g0 = stream * fps, g1 = g0 + fps < TF ? g0 + fps : TF;
    for (uint64_t g = g0; g < g1; ++g) {
        const float s = hop_sum(in, g, j);
        float* row = out + g * RF;
        if (MODE == 0) {
            float2* r2 = reinterpret_cast<float2*>(row);
            for (int k = j; k < (int)(RF / 2); k += 32) r2[k] = make_float2(s, (float)k);
        } else if (MODE == 1) {
            const int sh = (int)((reinterpret_cast<uintptr_t>(row) >> 2) & 3);
            float* ab = row - sh;
            const int nch = (sh + (int)RF + 3) >> 2;
            for (int i = j; i < nch; i += 32) {
                const int e0 = 4 * i;
                if (e0 >= sh && e0 + 4 <= sh + (int)RF) {
                    *reinterpret_cast<float4*>(ab + e0) = make_float4(s, 1.f, 2.f, (float)i);
                } else {
                    for (int e = 0; e < 4; ++e)
                        if (e0 + e >= sh && e0 + e < sh + (int)RF) ab[e0 + e] = s;
                }
            }
        } else {
            // lines [first, last) of this row: the row's head line only on the stream's first
            // frame (else the previous row wrote it), its tail line (shared with the next row)
            // now only on the stream's last frame
            const int sh = (int)((reinterpret_cast<uintptr_t>(row) >> 2) & 31);
            float* lb = row - sh;
            const int tot = sh + (int)RF, nfull = tot >> 5, rem = tot & 31;
            const int c0 = (g > g0 || sh == 0) ? 0 : 8;
            if (c0 && j >= sh) lb[j] = s;
            for (int i = c0 + j; i < nfull * 8; i += 32)
                *reinterpret_cast<float4*>(lb + 4 * i) = make_float4(s, 1.f, 2.f, (float)i);
            if (g + 1 == g1 && j < rem) lb[nfull * 32 + j] = s;
        }
    }
}

__global__ void copy12(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        out[i] = v;
        out[i + n] = v;
    }
}
__global__ void fill(float4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

#define CK(x) do { if ((x) != hipSuccess) { printf("hip error %d at %d\n", (int)(x), __LINE__); return 1; } } while (0)

int main() {
    const size_t in_bytes = TF * 4096 + 4096 * 8, out_bytes = TF * RF * 4 + 256;
    float4* in;
    float* out;
    CK(hipMalloc(&in, in_bytes));
    CK(hipMalloc(&out, out_bytes));
    CK(hipMemset(in, 0, in_bytes));
    CK(hipMemset(out, 0, out_bytes));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    const uint64_t fps = (TF + STREAMS - 1) / STREAMS;
    const double alg = (double)TF * 4096 + (double)TF * RF * 4;
    auto time = [&](const char* name, auto launch, double bytes) -> int {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(s));
            launch();
            CK(hipEventRecord(e));
            CK(hipEventSynchronize(e));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, s, e));
            best = ms < best ? ms : best;
        }
        printf("{\"probe\": \"%s\", \"ms\": %.3f, \"GBps\": %.0f}\n", name, best, bytes / best / 1e6);
        fflush(stdout);
        return 0;
    };
    for (int round = 0; round < 2; ++round) {
        if (time("rows lane8", [&] { hipLaunchKernelGGL(rows<0>, dim3(256), dim3(512), 0, 0, in, out, fps); }, alg)) return 1;
        if (time("rows b128", [&] { hipLaunchKernelGGL(rows<1>, dim3(256), dim3(512), 0, 0, in, out, fps); }, alg)) return 1;
        if (time("rows lines", [&] { hipLaunchKernelGGL(rows<2>, dim3(256), dim3(512), 0, 0, in, out, fps); }, alg)) return 1;
        // same bytes, patterns the hardware likes best
        const size_t n4 = TF * 4096 / 16;
        for (int grid : {2048, 8192})
            if (time(grid == 2048 ? "copy 1:2 grid 2048" : "copy 1:2 grid 8192",
                     [&] { hipLaunchKernelGGL(copy12, dim3(grid), dim3(256), 0, 0, in, reinterpret_cast<float4*>(out), n4); },
                     3.0 * n4 * 16)) return 1;
        if (time("fill", [&] { hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, reinterpret_cast<float4*>(out), TF * RF / 4); },
                 (double)TF * RF * 4)) return 1;
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
