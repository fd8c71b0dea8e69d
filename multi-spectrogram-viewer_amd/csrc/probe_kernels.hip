// probe_kernels.hip -- the box's own HBM ceiling for a kernel's read : write mix, measured in
// the caller's process on the caller's buffers (bench.py puts it beside the complex-output
// kernel's roofline: the same 11.52 GB read once and 23.07 GB written). Not part
// of the reference surface; a measurement aid.
#include "engine.hpp"
#include "kernels.hpp"

namespace thesia {

// every float4 of src read once, every float4 of dst written once (dst element i takes src
// element i mod n_src): coalesced 16-byte loads and stores, grid-stride
__global__ void __launch_bounds__(256) hbm_mix_kernel(const float4* __restrict__ src, size_t n_src,
                                                      float4* __restrict__ dst, size_t n_dst) {
    const size_t step = (size_t)gridDim.x * blockDim.x;
    const size_t k = n_dst / n_src;  // whole copies of src in dst
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_src; i += step) {
        const float4 v = src[i];
        for (size_t m = 0; m < k; ++m) dst[i + m * n_src] = v;
    }
    for (size_t i = k * n_src + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_dst; i += step)
        dst[i] = src[i - k * n_src];
}

int hbm_mix(const void* src, size_t src_bytes, void* dst, size_t dst_bytes, int grid, hipStream_t s) {
    const size_t ns = src_bytes / 16, nd = dst_bytes / 16;
    if (ns == 0) return -1;
    hipLaunchKernelGGL(hbm_mix_kernel, dim3(grid), dim3(256), 0, s, static_cast<const float4*>(src), ns,
                       static_cast<float4*>(dst), nd);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace thesia
