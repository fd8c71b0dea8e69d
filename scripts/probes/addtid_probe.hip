// Where does ds_write_addtid_b32 put lane L's dword for a given M0 and offset? (round-4 probe; its
// output, profiles/r04_close/addtid_probe.txt, did not follow M0 + offset + 4 lane: not used)
// One block of two waves; wave w writes (w << 16 | lane) with M0 = m0[w], offset = OFF; the whole LDS (160 KiB)
// is then copied out and the host prints the dword index of a few lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
template <int OFF>
__global__ void k(unsigned m0a, unsigned m0b, unsigned* out) {
    extern __shared__ unsigned lds[];
    for (int i = threadIdx.x; i < 40960; i += blockDim.x) lds[i] = 0xffffffffu;
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned m0 = __builtin_amdgcn_readfirstlane(w ? m0b : m0a);
    const unsigned val = ((unsigned)w << 16) | lane;
    asm volatile("s_mov_b32 m0, %0\n\tds_write_addtid_b32 %1 offset:%c2\n\ts_waitcnt lgkmcnt(0)" :: "s"(m0), "v"(val), "i"(OFF) : "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 40960; i += blockDim.x) out[i] = lds[i];
}
template <int OFF>
static void run(unsigned a, unsigned b) {
    unsigned* d; hipMalloc(&d, 40960 * 4);
    hipFuncSetAttribute((const void*)k<OFF>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    hipLaunchKernelGGL(k<OFF>, dim3(1), dim3(128), 163840, 0, a, b, d);
    std::vector<unsigned> h(40960);
    hipMemcpy(h.data(), d, 40960 * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    printf("OFF %d m0 %u %u:", OFF, a, b);
    for (int i = 0; i < 40960; ++i)
        if (h[i] != 0xffffffffu && ((h[i] & 0xffff) == 0 || (h[i] & 0xffff) == 1 || (h[i] & 0xffff) == 63))
            printf(" [w%u l%u @byte %d]", h[i] >> 16, h[i] & 0xffff, i * 4);
    int n = 0;
    for (int i = 0; i < 40960; ++i) n += h[i] != 0xffffffffu;
    printf(" written %d\n", n);
}
int main() {
    run<0>(0, 1024);
    run<0>(4, 65536);
    run<0>(40000, 70000);
    run<17600>(0, 47000);
    run<17600>(60000, 65184);
    run<256>(100, 1000);
    return 0;
}
