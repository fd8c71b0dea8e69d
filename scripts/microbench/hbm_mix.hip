// hbm_mix.hip -- practical HBM ceilings on gfx950 for the STFT kernels' traffic mixes:
// float4 grid-stride copy (1:1), read-once-write-twice (1:2, the complex-output kernel's mix)
// and pure write. Build: hipcc --offload-arch=gfx950 -O3 hbm_mix.hip -o hbm_mix
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void copy1(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}
__global__ void copy12(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        out[2 * i] = v;
        out[2 * i + 1] = v;
    }
}
__global__ void fill(float4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

#define CK(x) do { if ((x) != hipSuccess) { printf("hip error %d at %d\n", (int)(x), __LINE__); return 1; } } while (0)

int main() {
    const size_t n_in = 11520000000ull / 16;  // float4 elements of 11.52 GB
    float4 *in, *out;
    CK(hipMalloc(&in, n_in * 16));
    CK(hipMalloc(&out, 2 * n_in * 16));
    CK(hipMemset(in, 0, n_in * 16));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        for (int k = 0; k < 3; ++k) {
            double bytes = k == 0 ? 2.0 * n_in * 16 : k == 1 ? 3.0 * n_in * 16 : 2.0 * n_in * 16;
            auto launch = [&]() {
                if (k == 0) hipLaunchKernelGGL(copy1, dim3(grid), dim3(256), 0, 0, in, out, n_in);
                else if (k == 1) hipLaunchKernelGGL(copy12, dim3(grid), dim3(256), 0, 0, in, out, n_in);
                else hipLaunchKernelGGL(fill, dim3(grid), dim3(256), 0, 0, out, 2 * n_in);
            };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(s));
            for (int it = 0; it < 5; ++it) launch();
            CK(hipEventRecord(e));
            CK(hipEventSynchronize(e));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, s, e));
            ms /= 5;
            printf("{\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.3f, \"GBps\": %.0f}\n",
                   k == 0 ? "copy 1:1" : k == 1 ? "read1 write2" : "fill", grid, ms, bytes / ms / 1e6);
        }
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
