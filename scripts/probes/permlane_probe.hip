// Probe: which lanes v_permlane16_swap / v_permlane32_swap exchange, and which builtin result is
// the new vdst (stftr_kernels.hip relies on: result[0] = vdst after, result[1] = vsrc after;
// 16: vdst's odd 16-lane rows <-> vsrc's even rows; 32: vdst's lanes 32..63 <-> vsrc's 0..31).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* o) {
    const unsigned l = threadIdx.x;
    auto a = __builtin_amdgcn_permlane16_swap(1000u + l, 2000u + l, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(1000u + l, 2000u + l, false, false);
    o[l] = a[0]; o[64 + l] = a[1]; o[128 + l] = b[0]; o[192 + l] = b[1];
}

int main() {
    unsigned* d; unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* nm[4] = {"pl16 vdst", "pl16 vsrc", "pl32 vdst", "pl32 vsrc"};
    int bad = 0;
    for (int r = 0; r < 4; ++r) {
        printf("%s:", nm[r]);
        for (int l = 0; l < 64; ++l) printf(" %u", h[r * 64 + l]);
        printf("\n");
    }
    for (unsigned l = 0; l < 64; ++l) {
        const bool odd = (l >> 4) & 1, hi = l >= 32;
        unsigned e16d = odd ? 2000 + (l - 16) : 1000 + l;   // vdst: odd rows take vsrc's even row
        unsigned e16s = odd ? 2000 + l : 1000 + (l + 16);   // vsrc: even rows take vdst's odd row
        unsigned e32d = hi ? 2000 + (l - 32) : 1000 + l;
        unsigned e32s = hi ? 2000 + l : 1000 + (l + 32);
        bad += h[l] != e16d || h[64 + l] != e16s || h[128 + l] != e32d || h[192 + l] != e32s;
    }
    printf("expected semantics: %s (%d lanes differ)\n", bad ? "NO" : "yes", bad);
    hipFree(d);
    return bad ? 2 : 0;
}
