// Probe: what hipPointerGetAttributes / hipHostGetFlags report for pageable (malloc), page-locked
// (hipHostMalloc) and registered (hipHostRegister) host memory on this runtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

static void show(const char* name, void* p) {
    hipPointerAttribute_t a{};
    hipError_t e = hipPointerGetAttributes(&a, p);
    unsigned flags = 0;
    hipError_t f = hipHostGetFlags(&flags, p);
    printf("%-12s getattr %-28s type %d | hostGetFlags %-28s flags %u\n", name, hipGetErrorName(e), (int)a.type,
           hipGetErrorName(f), flags);
    (void)hipGetLastError();
}

int main() {
    const size_t n = 6u << 20;
    void* pg = malloc(n);
    void* small = malloc(4096);
    void* hm = nullptr;
    if (hipHostMalloc(&hm, n, hipHostMallocDefault) != hipSuccess) return 1;
    void* rg = malloc(n);
    if (hipHostRegister(rg, n, hipHostRegisterDefault) != hipSuccess) return 1;
    show("malloc 6MB", pg);
    show("malloc 4KB", small);
    show("hostMalloc", hm);
    show("registered", rg);
    show("reg+1MB", static_cast<char*>(rg) + (1 << 20));
    return 0;
}
