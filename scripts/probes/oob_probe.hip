// Range checking of a raw buffer_load_dwordx4 that straddles the descriptor's end or starts below
// its base (negative 32-bit offset): which of the four dwords come back as the data, which as 0?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* src, float* out, int nrec, int off) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, nrec, 0x00020000);
    typedef float v4 __attribute__((ext_vector_type(4)));
    v4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)off, 0, 0);
    if (threadIdx.x == 0) { out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w; }
}
int main() {
    float h[64];
    for (int i = 0; i < 64; ++i) h[i] = 100.0f + i;
    float *d, *o;
    hipMalloc(&d, sizeof h); hipMalloc(&o, 16);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    const int cases[][2] = {{64, 0}, {64, 32}, {40, 32}, {44, 32}, {36, 32}, {64, -4}, {64, -8}, {64, -12}};
    for (auto& c : cases) {
        // base at element 16 so that negative offsets stay inside the allocation
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d + 16, o, c[0], c[1]);
        float r[4];
        hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
        printf("num_records %d offset %d -> %g %g %g %g\n", c[0], c[1], r[0], r[1], r[2], r[3]);
    }
    return 0;
}
