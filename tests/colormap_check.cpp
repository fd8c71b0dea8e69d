// colormap_rgb (csrc/display_common.hpp: the paired-stop, branch-free colormap the display
// kernels use) against the oracle's or_grey_to_color (display.rs:24-42) on every 32-bit pattern
// `step` apart: usage colormap_check liboracle.so step -> "n mismatches"
#include "display_common.hpp"

#include <dlfcn.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    void* h = dlopen(argv[1], RTLD_NOW);
    if (!h) return 3;
    auto ref = reinterpret_cast<int (*)(float, uint8_t*)>(dlsym(h, "or_grey_to_color"));
    auto stops = reinterpret_cast<const uint8_t*>(dlsym(h, "OR_COLORMAP"));
    if (!ref || !stops) return 4;
    const uint64_t step = strtoull(argv[2], nullptr, 10);
    uint2 lut[10];
    for (int i = 0; i < 10; ++i) lut[i] = thesia::colormap_pair(stops, i);
    const unsigned nt = std::thread::hardware_concurrency() ? std::thread::hardware_concurrency() : 4;
    std::atomic<uint64_t> n{0}, bad{0};
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; ++w)
        th.emplace_back([&, w] {
            uint64_t nn = 0, bb = 0;
            for (uint64_t b = (uint64_t)w * step; b <= 0xFFFFFFFFull; b += (uint64_t)nt * step) {
                const uint32_t u = (uint32_t)b;
                float t;
                std::memcpy(&t, &u, 4);
                uint8_t o[3];
                ref(t, o);
                const uint32_t px = thesia::colormap_rgb(t, lut);
                bb += px != ((uint32_t)o[0] | (uint32_t)o[1] << 8 | (uint32_t)o[2] << 16);
                ++nn;
            }
            n += nn;
            bad += bb;
        });
    for (auto& t : th) t.join();
    std::printf("%llu %llu\n", (unsigned long long)n.load(), (unsigned long long)bad.load());
    return 0;
}
