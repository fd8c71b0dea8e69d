// engine.cpp -- plans, batches, streams, device buffers and display helpers of libthesia.
#include "engine.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <memory>

#include "host_tables.hpp"

namespace thesia {

// ------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------
static thread_local std::string g_err;

int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
void clear_error() { g_err.clear(); }
const char* last_error() { return g_err.c_str(); }

// ------------------------------------------------------------------------------------
// device buffers / streams
// ------------------------------------------------------------------------------------
// The library's block cache (round 5; replaces the stream-ordered memory pool of rounds 3-4, see
// DESIGN.md §10.1 for what round 5's lost greys were). Blocks come from plain hipMalloc and
// freed ones are kept here for reuse, keyed by device and size class, so add_tracks pays no
// hipFree (each one synchronises the device: ~160 us, profiles/r03_viewer):
//   * a block is handed out again at once only on the stream of its last use (DevBuf::use: in
//     order behind that work), on any other stream once an event recorded there at its release
//     has completed (engine.hpp states the invariant);
//   * classes are 2^k and 3 * 2^(k-2) (<= 33 % slack) up to 64 MiB, whole 2 MiB steps above;
//   * the cache holds at most kCacheCap bytes per device (a release past it is a hipFree) and
//     is emptied by trim_pool() (thesia_pool_trim, MultiTrack destruction, and before a failed
//     hipMalloc is retried).
namespace {
struct CachedBlock {
    void* p;
    size_t cap;
    hipStream_t st;
    hipEvent_t ev;
};
struct DevCache {
    std::vector<CachedBlock> free;
    size_t cached = 0;  // bytes in free
    size_t live = 0;    // bytes handed out
};
std::mutex g_cache_mu;
std::map<int, DevCache> g_cache;
constexpr size_t kCacheCap = size_t(4) << 30;

size_t cache_class(size_t n) {
    constexpr size_t kMin = 4096, kBig = size_t(64) << 20, kStep = size_t(2) << 20;
    if (n <= kMin) return kMin;
    if (n > kBig) return (n + kStep - 1) / kStep * kStep;
    size_t b = kMin;
    while (b < n) b <<= 1;  // 2^k >= n
    return (b / 4) * 3 >= n ? (b / 4) * 3 : b;
}

int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) {
        (void)hipGetLastError();
        d = 0;
    }
    return d;
}
}  // namespace

#ifdef THESIA_POOL_DIAG
// Diagnostic build only (scripts/build_variant.sh pooldiag "-DTHESIA_POOL_DIAG" engine.cpp; round 6,
// VERDICT r05 item 1): the rounds 3-4 allocator (the library's own stream-ordered pool,
// hipMallocFromPoolAsync / hipFreeAsync on the allocation stream), every allocation and release
// logged to stderr with its stream, so a failing call's block lifetimes can be read back.
static hipMemPool_t diag_pool() {
    static hipMemPool_t pool = [] {
        hipMemPool_t q = nullptr;
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = 0;
        if (hipMemPoolCreate(&q, &props) != hipSuccess) return (hipMemPool_t) nullptr;
        uint64_t thr = ~uint64_t(0);
        (void)hipMemPoolSetAttribute(q, hipMemPoolAttrReleaseThreshold, &thr);
        return q;
    }();
    return pool;
}
#endif

void DevBuf::release() {
    if (!p) return;
#ifdef THESIA_POOL_DIAG
    fprintf(stderr, "POOLDIAG free %p %zu st %p\n", p, bytes, (void*)st);
    (void)hipFreeAsync(p, st);
    p = nullptr;
    bytes = 0;
    return;
#endif
    if (pooled) {
        const size_t cap = cache_class(bytes);
        std::lock_guard<std::mutex> g(g_cache_mu);
        DevCache& c = g_cache[dev];
        c.live -= cap;
        hipEvent_t ev = nullptr;
        bool ok = c.cached + cap <= kCacheCap;
        if (ok && foreign) {
            // last used on another stream: the event recorded there at that use orders the reuse;
            // no stream is kept (it may be gone), so every allocation waits for the event
            ev = use_ev;
            use_ev = nullptr;
        } else if (ok) {
            ok = hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess && hipEventRecord(ev, st) == hipSuccess;
        }
        if (ok && ev) {
            c.free.push_back(CachedBlock{p, cap, foreign ? nullptr : st, ev});
            c.cached += cap;
        } else {
            (void)hipGetLastError();
            if (ev) (void)hipEventDestroy(ev);
            (void)hipFree(p);  // (a device synchronisation: behind every use, on any stream)
        }
    } else {
        (void)hipFree(p);
    }
    p = nullptr;
    bytes = 0;
    foreign = false;
}

void DevBuf::used_on(hipStream_t s) {
    if (!p || !s) return;
    if (s == st) {
        // the allocation stream: the release event is recorded there; an earlier use on another
        // stream is ordered into it first
        if (foreign && use_ev) (void)hipStreamWaitEvent(st, use_ev, 0);
        foreign = false;
        return;
    }
    if (!use_ev && hipEventCreateWithFlags(&use_ev, hipEventDisableTiming) != hipSuccess) use_ev = nullptr;
    // (an earlier use on a third stream is ordered into s, so the one event covers both)
    if (use_ev && foreign) (void)hipStreamWaitEvent(s, use_ev, 0);
    if (use_ev && hipEventRecord(use_ev, s) == hipSuccess) {
        foreign = true;
        return;
    }
    (void)hipGetLastError();
    (void)hipStreamSynchronize(s);  // no event: the work is done before the block can be released
    foreign = false;
}

int trim_pool() {
    std::lock_guard<std::mutex> g(g_cache_mu);
    for (auto& kv : g_cache) {
        for (CachedBlock& b : kv.second.free) {
            (void)hipEventSynchronize(b.ev);
            (void)hipEventDestroy(b.ev);
            (void)hipFree(b.p);
        }
        kv.second.free.clear();
        kv.second.cached = 0;
    }
    (void)hipGetLastError();
    return THESIA_OK;
}

int pool_bytes(uint64_t* reserved, uint64_t* used) {
    std::lock_guard<std::mutex> g(g_cache_mu);
    uint64_t r = 0, u = 0;
    auto it = g_cache.find(current_device());
    if (it != g_cache.end()) {
        u = it->second.live;
        r = it->second.live + it->second.cached;
    }
    if (reserved) *reserved = r;
    if (used) *used = u;
    return THESIA_OK;
}

int DevBuf::alloc(size_t n) {
    release();
    if (n == 0) n = 16;
    hipStream_t s = default_stream();
    const int d = current_device();
#ifdef THESIA_POOL_DIAG
    {
        const hipError_t e = hipMallocFromPoolAsync(&p, n, diag_pool(), s);
        fprintf(stderr, "POOLDIAG alloc %p %zu st %p rc %d\n", p, n, (void*)s, (int)e);
        if (e != hipSuccess) {
            p = nullptr;
            return set_error(THESIA_ERR_DEVICE, "hipMallocFromPoolAsync failed");
        }
        pooled = true;
        dev = d;
        st = s;
        bytes = n;
        return THESIA_OK;
    }
#endif
    const size_t cap = cache_class(n);
    {
        std::lock_guard<std::mutex> g(g_cache_mu);
        DevCache& c = g_cache[d];
        for (size_t i = c.free.size(); i-- > 0;) {  // the most recently released first
            CachedBlock& b = c.free[i];
            if (b.cap != cap) continue;
            if (b.st != s || !b.st) {  // (a block last used on a caller's stream: the event only)
                const hipError_t q = hipEventQuery(b.ev);
                if (q != hipSuccess) {
                    (void)hipGetLastError();
                    continue;
                }
            }
            p = b.p;
            (void)hipEventDestroy(b.ev);
            c.free.erase(c.free.begin() + (std::ptrdiff_t)i);
            c.cached -= cap;
            c.live += cap;
            break;
        }
    }
    if (!p) {
        hipError_t e = hipMalloc(&p, cap);
        if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
            // the cache's idle blocks may be what is missing: hand them back, retry once
            (void)hipGetLastError();
            if (trim_pool() == THESIA_OK) e = hipMalloc(&p, cap);
        }
        if (e != hipSuccess) {
            p = nullptr;
            return set_error(THESIA_ERR_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
        std::lock_guard<std::mutex> g(g_cache_mu);
        g_cache[d].live += cap;
    }
    pooled = true;
    dev = d;
    st = s;
    foreign = false;
    bytes = n;
    return THESIA_OK;
}

int DevBuf::upload(const void* host, size_t n) {
    int rc = alloc(n);
    if (rc) return rc;
    if (n && host) THESIA_HIP(copy_ordered(p, host, n, hipMemcpyHostToDevice));
    return THESIA_OK;
}

bool host_pinned(const void* p) {
    hipPointerAttribute_t a{};
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// A copy ordered after everything already enqueued on stream s. Page-locked host memory (or
// device to device): an async copy on s. Pageable host memory: the same async copy on s, then s is
// synchronised, so the caller may reuse or free the host range when this returns. (Round 5 had
// the pageable case drain s, make a blocking null-stream copy and synchronise the whole device,
// after a diagnosis that blamed the ordering of pageable copies for lost greys; round 6's probe,
// scripts/probes/pool_probe.hip, found pageable uploads on a non-blocking stream ordered with the
// kernels behind them, 4 x 92 MiB, profiles/r06_pool/pool_probe.txt.)
hipError_t copy_on(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
    if (!bytes) return hipSuccess;
    const void* host = kind == hipMemcpyHostToDevice ? src : kind == hipMemcpyDeviceToHost ? dst : nullptr;
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s);
    if (e == hipSuccess && host && !host_pinned(host)) e = hipStreamSynchronize(s);
    return e;
}

hipError_t copy_ordered(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    hipStream_t s = default_stream();
    hipError_t e = copy_on(dst, src, bytes, kind, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e;
}

hipStream_t default_stream() {
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = streams.find(dev);
    if (it != streams.end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
    streams[dev] = s;
    return s;
}

// ------------------------------------------------------------------------------------
// plans
// ------------------------------------------------------------------------------------
size_t Plan::row_bins() const {
    if (out_kind == OUT_MEL || out_kind == OUT_MEL_AMP_DB) return n_mels;
    return NC + 1;
}

static bool is_pow2(size_t v) { return v && !(v & (v - 1)); }

// mel filterbank -> per-lane fma rounds (stft_kernels.hip mel_rounds). Round r gives lane j
// of a frame mel r*L + j; the round runs len_r = the longest nonzero band among its mels,
// each lane from k0 = min(band start, F - len_r) so the window stays inside the |X| row.
// The weights are the filterbank's own f32 values (zeros outside the band), so the lane's
// fma chain over k ascending matches the dense k-ascending dot term for term.
static int build_mel(Plan* p) {
    const size_t F = p->NC + 1, M = p->n_mels;
    int L = 0;
    if (stft_kernel_info((int)p->n_fft, nullptr, nullptr, &L) != 0 || L <= 0)
        return set_error(THESIA_ERR_UNSUPPORTED, "unsupported n_fft");
    const size_t R = (M + L - 1) / L;
    std::vector<int2> rounds(R);
    std::vector<int> k0((size_t)R * L, 0);
    std::vector<float> wt;
    size_t rows = 0;
    for (size_t r = 0; r < R; ++r) {
        std::vector<long> lo(L, 0), hi(L, 0);
        long len = 0;
        for (int j = 0; j < L; ++j) {
            const size_t m = r * L + j;
            if (m >= M) continue;
            long l0 = -1, h0 = -1;
            for (size_t k = 0; k < F; ++k)
                if (p->mel_fb[k * M + m] != 0.0f) {
                    if (l0 < 0) l0 = (long)k;
                    h0 = (long)k + 1;
                }
            if (l0 >= 0) { lo[j] = l0; hi[j] = h0; len = std::max(len, h0 - l0); }
        }
        rounds[r] = int2{(int)rows, (int)len};
        wt.resize((rows + (size_t)len) * L, 0.0f);
        for (int j = 0; j < L; ++j) {
            const size_t m = r * L + j;
            const long s = std::min(lo[j], (long)F - len);
            k0[r * L + j] = (int)s;
            if (m >= M) continue;
            for (long it = 0; it < len; ++it)
                wt[(rows + (size_t)it) * L + j] = p->mel_fb[(size_t)(s + it) * M + m];
        }
        rows += (size_t)len;
    }
    if (wt.empty()) wt.assign(1, 0.0f);
    int rc = p->mel_round.upload(rounds.data(), std::max<size_t>(R, 1) * sizeof(int2));
    if (!rc) rc = p->mel_k0.upload(k0.data(), std::max<size_t>(k0.size(), 1) * sizeof(int));
    if (!rc) rc = p->mel_wt.upload(wt.data(), wt.size() * sizeof(float));
    p->mel_rounds = (int)R;
    p->mel_wt_rows = rows;
    return rc;
}

// The same projection in stft2_kernel's float4 layout (stft2_core.hpp mel4). Round r holds
// L filters, one per lane; each lane's entry packs its start bin k0 (a multiple of 4) and its
// mel index: k0 | m << 16 (m = 0xFFFF: idle lane). A round runs len4 float4 steps (its widest
// band, padded to whole 4-step batches), so k0 may move left within a band's slack; rounds
// stay inside the zero-padded row of F4 = ceil4(F) bins.
//
// Bank-aware placement (L = 32): a ds_read_b128 of the |X| row is served in 16-lane groups
// G1 = {0-3, 12-15, 20-27} and G2 = {4-11, 16-19, 28-31} (MI355X_MICROARCH.md, LDS table);
// a lane reading float4 k0/4 + s occupies the 4-bank slot (k0/4 + s) mod 16 at every step s,
// so a group is conflict-free iff its lanes' k0/4 mod 16 differ (or their k0 are equal:
// broadcast). Filters are dealt, least slack first, to the group and k0 that keep slots free.
// Unit-sum mel-128 @ 48 kHz / 2048: 140 -> 64 LDS cycles per frame for the |X| reads.
static int build_mel4(Plan* p) {
    const long F = (long)p->NC + 1, F4 = (F + 3) / 4 * 4;
    const size_t M = p->n_mels;
    int L = 0;
    if (stft_kernel_info((int)p->n_fft, nullptr, nullptr, &L) != 0 || L <= 0)
        return set_error(THESIA_ERR_UNSUPPORTED, "unsupported n_fft");
    const size_t R = (M + L - 1) / L;
    std::vector<int2> rounds(R);
    std::vector<int> k0m((size_t)R * L, 0xFFFF << 16);
    std::vector<float> wt;
    size_t rows = 0;
    static const int kG1[16] = {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27};
    static const int kG2[16] = {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31};
    for (size_t r = 0; r < R; ++r) {
        const int nm = (int)std::min<size_t>(L, M - r * L);
        std::vector<long> lo(nm, 0), hi(nm, 0);
        long len4 = 0;
        for (int i = 0; i < nm; ++i) {
            const size_t m = r * L + i;
            long l0 = -1, h0 = -1;
            for (long k = 0; k < F; ++k)
                if (p->mel_fb[(size_t)k * M + m] != 0.0f) {
                    if (l0 < 0) l0 = k;
                    h0 = k + 1;
                }
            if (l0 < 0) l0 = h0 = 0;  // empty filter: any start, all-zero weights
            lo[i] = l0 / 4 * 4;
            hi[i] = h0;
            len4 = std::max(len4, (h0 - lo[i] + 3) / 4);
        }
        // pad the round to whole 4-step batches (zero weights; mel4 issues a batch's LDS
        // reads together), as long as the round still fits the F4-bin row
        if ((len4 + 3) / 4 * 4 * 4 <= F4) len4 = (len4 + 3) / 4 * 4;
        // per filter: the k0 range [kmin, kmax] (multiples of 4) that covers its band
        std::vector<long> kmin(nm), kmax(nm), k0(nm);
        for (int i = 0; i < nm; ++i) {
            kmax[i] = std::min(lo[i], F4 - 4 * len4);
            kmin[i] = std::max(0L, std::min(kmax[i], (hi[i] - 4 * len4 + 3) / 4 * 4));
            k0[i] = kmax[i];
        }
        std::vector<int> lane_of(nm);
        if (L == 32) {
            std::vector<int> order(nm);
            for (int i = 0; i < nm; ++i) order[i] = i;
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
                return kmax[a] - kmin[a] < kmax[b] - kmin[b];
            });
            std::vector<long> used[2];  // k0 values placed in each group
            for (int i : order) {
                int best_g = -1;
                long best_k = kmax[i];
                int best_cost = 1 << 30;
                for (int g = 0; g < 2; ++g) {
                    if (used[g].size() >= 16) continue;
                    for (long k = kmax[i]; k >= kmin[i]; k -= 4) {
                        int cost = 0;
                        bool same = false;
                        for (long u : used[g]) {
                            if (u == k) same = true;
                            else if (((u / 4) & 15) == ((k / 4) & 15)) ++cost;
                        }
                        if (same) cost = 0;
                        cost = cost * 64 + (int)used[g].size();  // then balance the groups
                        if (cost < best_cost) { best_cost = cost; best_g = g; best_k = k; }
                    }
                }
                lane_of[i] = (best_g == 0 ? kG1 : kG2)[used[best_g].size()];
                used[best_g].push_back(best_k);
                k0[i] = best_k;
            }
        } else {
            for (int i = 0; i < nm; ++i) lane_of[i] = i;
        }
        rounds[r] = int2{(int)rows, (int)len4};
        wt.resize((rows + (size_t)len4) * L * 4, 0.0f);
        for (int j = 0; j < L; ++j) k0m[r * L + j] = (int)(F4 - 4 * len4) | (0xFFFF << 16);
        for (int i = 0; i < nm; ++i) {
            const size_t m = r * L + i;
            const int j = lane_of[i];
            k0m[r * L + j] = (int)k0[i] | (int)(m << 16);
            for (long it = 0; it < len4; ++it)
                for (int u = 0; u < 4; ++u) {
                    const long k = k0[i] + 4 * it + u;
                    wt[((rows + (size_t)it) * L + j) * 4 + u] = k < F ? p->mel_fb[(size_t)k * M + m] : 0.0f;
                }
        }
        rows += (size_t)len4;
    }
    if (wt.empty()) wt.assign(4, 0.0f);
    int rc = p->mel4_round.upload(rounds.data(), std::max<size_t>(R, 1) * sizeof(int2));
    if (!rc) rc = p->mel4_k0.upload(k0m.data(), std::max<size_t>(k0m.size(), 1) * sizeof(int));
    if (!rc) rc = p->mel4_wt.upload(wt.data(), wt.size() * sizeof(float));
    p->mel4_rounds = (int)R;
    p->mel4_wt_rows = rows;
    // the same rounds as one stream of 4-step chunks (stft5 mel4p)
    {
        std::vector<int> xo;
        bool ok = true;
        for (size_t r = 0; r < R && ok; ++r) {
            const int nch = rounds[r].y / 4;
            if (rounds[r].y <= 0 || rounds[r].y % 4 != 0 || rounds[r].x != (int)(xo.size() / L) * 4) ok = false;
            for (int cc = 0; cc < nch && ok; ++cc)
                for (int j = 0; j < L; ++j) {
                    const int km = k0m[r * L + j];
                    const int v = ((km & 0xFFFF) + 16 * cc) | (((km >> 16) & 0x7FFF) << 16) |
                                  (cc == nch - 1 ? (int)0x80000000u : 0);
                    xo.push_back(v);
                }
        }
        // the kernel runs a fixed 4 or 8 chunks (no guards: guarded loads made the compiler's
        // LDS wait counts assume the shorter path); padding chunks read bin 0 with zero weights
        // and never emit
        const int C = ok ? (int)(xo.size() / L) : 0;
        const int CP = C == 0 || C > 8 ? 0 : C <= 4 ? 4 : 8;
        if (CP) {
            xo.resize((size_t)CP * L, 0);
            if (rows < (size_t)CP * 4) {
                wt.resize((size_t)CP * 4 * L * 4, 0.0f);
                rows = (size_t)CP * 4;
                p->mel4_wt_rows = rows;
                if (!rc) rc = p->mel4_wt.upload(wt.data(), wt.size() * sizeof(float));
            }
        }
        p->mel_chunks = CP;
        if (!rc && p->mel_chunks) rc = p->mel_xo.upload(xo.data(), xo.size() * sizeof(int));
    }
    return rc;
}

// stft5's packed mel stream (kernels.hpp melp_*), S float4 steps per chunk. Every filter is
// padded to whole chunks: its first chunk starts at a multiple of 4 bins at or before its band
// and the weights outside the band are zero, so the lane's k-ascending fma chain adds only +0
// terms around the band and each mel is the same chain as mel4's (bit-exact with it). The
// filters are dealt to the 32 lanes largest first onto the least loaded lane (LPT) and a lane
// runs its filters back to back: a frame costs the largest lane load in chunks (mel-128 @ 48 kHz
// / 2048: 11 chunks of 2 steps, where the rounds pad every lane to the round's widest band and
// take 32 steps). Placement: which lane runs which filter sequence, the order of a lane's
// filters and each filter's start within its slack are searched (seeded random restarts +
// coordinate descent) for the fewest LDS cycles of the |X| reads (a ds_read_b128 is served in
// build_mel4's 16-lane groups; per group, the lanes of one 16-byte slot mod 16 cost one cycle
// per distinct address).
static const int kLdsG[2][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31}};

// L: lanes per frame (32: stft5, two frames per wave; 64: stftr, one frame per wave, whose
// b128 read groups are build_mel4's for each half); region: the floats of a frame's LDS region.
static int build_melp(Plan* p, int S, Plan::Melp& out, int L = 32, int region = kStft5Region) {
    out.chunks = 0;
    out.steps = S;
    const long F = (long)p->NC + 1, F4 = (F + 3) / 4 * 4;
    const int M = (int)p->n_mels;
    if (p->NC != 1024 || F4 != kMelpOut || M <= 0 || kMelpOut + M + kMelpDummies > region)
        return THESIA_OK;  // not stft5's geometry / the mel slots do not fit the region
    const int NG = L / 16;  // 16-lane groups of a ds_read_b128
    struct Flt { long kmin, kmax; int ch; };
    std::vector<Flt> fl(M);
    for (int m = 0; m < M; ++m) {
        long lo = -1, hi = -1;
        for (long k = 0; k < F; ++k)
            if (p->mel_fb[(size_t)k * M + m] != 0.0f) {
                if (lo < 0) lo = k;
                hi = k + 1;
            }
        if (lo < 0) lo = hi = 0;  // empty filter: one chunk of zero weights (its mel is +0)
        const long lo4 = lo / 4 * 4;
        const int ch = (int)((std::max(1L, (hi - lo4 + 3) / 4) + S - 1) / S);
        const long span = 4L * S * ch;
        if (span > F4) return THESIA_OK;
        fl[m] = Flt{std::max(0L, (hi - span + 3) / 4 * 4), std::min(lo4, F4 - span), ch};
    }
    std::vector<int> order(M);
    for (int m = 0; m < M; ++m) order[m] = m;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return fl[a].ch > fl[b].ch; });
    std::vector<std::vector<int>> seq(L);
    std::vector<int> load(L, 0);
    for (int f : order) {
        const int j = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        seq[j].push_back(f);
        load[j] += fl[f].ch;
    }
    const int C = *std::max_element(load.begin(), load.end());
    if (C > 64) return THESIA_OK;

    auto glane = [&](int g, int i) { return kLdsG[g & 1][i] + 32 * (g >> 1); };
    std::vector<int> grp(L);
    for (int g = 0; g < NG; ++g)
        for (int i = 0; i < 16; ++i) grp[glane(g, i)] = g;
    std::vector<long> offs((size_t)L * C);  // |X| float offset per (lane, chunk); -1 = idle
    auto cell = [&](int c, int g) {
        long seen[16][16];
        int cnt[16] = {0}, worst = 0;
        for (int i = 0; i < 16; ++i) {
            const long o = offs[(size_t)glane(g, i) * C + c];
            if (o < 0) continue;
            const int s = (int)((o / 4) & 15);
            bool dup = false;
            for (int t = 0; t < cnt[s]; ++t) dup = dup || seen[s][t] == o;
            if (!dup) seen[s][cnt[s]++] = o;
            worst = std::max(worst, cnt[s]);
        }
        return worst;
    };
    std::vector<int> lane_of(M), c0_of(M), best_lane, best_c0;
    std::vector<long> k0(M), best_k0;
    long best = -1;
    uint64_t rs = 0x9E3779B97F4A7C15ull;  // fixed seed: the plan's tables are deterministic
    auto rnd = [&](uint64_t n) {
        rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
        return (int)(rs % n);
    };
    std::vector<int> perm(L);
    for (int trial = 0; trial < 48; ++trial) {
        for (int s = 0; s < L; ++s) perm[s] = s;
        auto sq = seq;
        if (trial > 0) {
            for (int s = L - 1; s > 0; --s) std::swap(perm[s], perm[rnd(s + 1)]);
            for (auto& q : sq)
                for (int t = (int)q.size() - 1; t > 0; --t) std::swap(q[t], q[rnd(t + 1)]);
        }
        std::fill(offs.begin(), offs.end(), -1L);
        for (int s = 0; s < L; ++s) {
            int c = 0;
            for (int f : sq[s]) {
                lane_of[f] = perm[s];
                c0_of[f] = c;
                k0[f] = fl[f].kmax;
                for (int i = 0; i < fl[f].ch; ++i) offs[(size_t)perm[s] * C + c + i] = k0[f] + 4L * S * i;
                c += fl[f].ch;
            }
        }
        for (int pass = 0; pass < 2; ++pass)
            for (int f = 0; f < M; ++f) {
                const int j = lane_of[f], g = grp[j];
                long bk = k0[f];
                int bc = 1 << 30;
                for (long k = fl[f].kmax; k >= fl[f].kmin; k -= 4) {
                    for (int i = 0; i < fl[f].ch; ++i) offs[(size_t)j * C + c0_of[f] + i] = k + 4L * S * i;
                    int cost = 0;
                    for (int i = 0; i < fl[f].ch; ++i) cost += cell(c0_of[f] + i, g);
                    if (cost < bc) { bc = cost; bk = k; }
                }
                k0[f] = bk;
                for (int i = 0; i < fl[f].ch; ++i) offs[(size_t)j * C + c0_of[f] + i] = bk + 4L * S * i;
            }
        long total = 0;
        for (int c = 0; c < C; ++c)
            for (int g = 0; g < NG; ++g) total += cell(c, g);
        if (best < 0 || total < best) {
            best = total;
            best_lane = lane_of;
            best_c0 = c0_of;
            best_k0 = k0;
        }
    }
    // tables: meta rows r = 0 .. C + 1 ({woff(r-1), keep(r-1), xoff(r), 0}); weight rows of
    // chunks 0 .. C (chunk C: the pipeline's read-ahead padding, zero weights)
    std::fill(offs.begin(), offs.end(), -1L);
    std::vector<int> woff((size_t)(C + 1) * L), keep((size_t)(C + 1) * L, -1);
    for (int j = 0; j < L; ++j)
        for (int c = 0; c <= C; ++c) woff[(size_t)c * L + j] = (kMelpOut + M + (j & (kMelpDummies - 1))) * 4;
    std::vector<float> wt((size_t)(C + 1) * S * L * 4, 0.0f);
    for (int f = 0; f < M; ++f) {
        const int j = best_lane[f];
        for (int i = 0; i < fl[f].ch; ++i) {
            const int c = best_c0[f] + i;
            offs[(size_t)j * C + c] = best_k0[f] + 4L * S * i;
            for (int u = 0; u < S; ++u)
                for (int e = 0; e < 4; ++e) {
                    const long k = best_k0[f] + 4L * (S * i + u) + e;
                    wt[(((size_t)c * S + u) * L + j) * 4 + e] = k < F ? p->mel_fb[(size_t)k * M + f] : 0.0f;
                }
        }
        const int cl = best_c0[f] + fl[f].ch - 1;
        woff[(size_t)cl * L + j] = (kMelpOut + f) * 4;
        keep[(size_t)cl * L + j] = 0;
    }
    // idle chunks read an address another lane of their group reads (a broadcast: no cycle)
    std::vector<int> xoff((size_t)(C + 1) * L, 0);
    for (int c = 0; c < C; ++c)
        for (int g = 0; g < NG; ++g) {
            long any = 0;
            for (int i = 0; i < 16; ++i)
                if (offs[(size_t)glane(g, i) * C + c] >= 0) { any = offs[(size_t)glane(g, i) * C + c]; break; }
            for (int i = 0; i < 16; ++i) {
                const int j = glane(g, i);
                const long o = offs[(size_t)j * C + c];
                xoff[(size_t)c * L + j] = (int)((o >= 0 ? o : any) * 4);
            }
        }
    std::vector<int4> meta((size_t)(C + 2) * L);
    for (int r = 0; r <= C + 1; ++r)
        for (int j = 0; j < L; ++j) {
            const int c = r - 1;
            meta[(size_t)r * L + j] = int4{c >= 0 ? woff[(size_t)c * L + j] : 0, c >= 0 ? keep[(size_t)c * L + j] : -1,
                                           r <= C ? xoff[(size_t)r * L + j] : 0, 0};
        }
    int rc = out.meta.upload(meta.data(), meta.size() * sizeof(int4));
    if (!rc) rc = out.wt.upload(wt.data(), wt.size() * sizeof(float));
    if (!rc) out.chunks = C;
    return rc;
}

// rustfft's prepare_radix4 (oracle cfft_tab): spec[j] = sig[...] in the digit order the
// radix-4 passes expect; run on indices it gives the source of every position
static void prepare_radix4_order(size_t size, const int* sig, int* spec, size_t stride) {
    if (size == 16) {
        for (size_t i = 0; i < 4; ++i) prepare_radix4_order(4, sig + i * stride, spec + i * 4, stride * 4);
    } else if (size == 8 || size == 4) {
        for (size_t i = 0; i < size; ++i) spec[i] = sig[i * stride];
    } else {
        for (size_t i = 0; i < 4; ++i)
            prepare_radix4_order(size / 4, sig + i * stride, spec + i * (size / 4), stride * 4);
    }
}

int plan_create(const thesia_plan_desc& d, Plan** out) {
    *out = nullptr;
    if (!is_pow2(d.n_fft) || d.n_fft < 2 || d.n_fft > 4096)
        return set_error(THESIA_ERR_UNSUPPORTED, "n_fft must be a power of two in [2, 4096]");
    if (d.win_length == 0 || d.win_length > d.n_fft)
        return set_error(THESIA_ERR_INVALID_ARG, "win_length must be in [1, n_fft]");
    if (d.hop_length == 0) return set_error(THESIA_ERR_INVALID_ARG, "hop_length must be > 0");
    if (d.output < THESIA_OUT_COMPLEX || d.output > THESIA_OUT_MEL_AMP_DB)
        return set_error(THESIA_ERR_INVALID_ARG, "unknown output kind");
    Plan* p = new Plan();
    p->desc = d;
    p->desc.window = nullptr;
    p->desc.mel_fb = nullptr;
    p->out_kind = d.output;
    p->n_fft = d.n_fft;
    p->NC = d.n_fft / 2;
    p->win = d.win_length;
    p->hop = d.hop_length;
    p->pad_left = (d.n_fft - d.win_length) / 2;  // lib.rs:400
    // window: given, or hann(win, false) / n_fft (lib.rs:138-140, :407)
    if (d.window) {
        p->window.assign(d.window, d.window + d.win_length);
    } else {
        p->window = hann(d.win_length, false);
        for (auto& w : p->window) w = w / (float)d.n_fft;
    }
    std::vector<float> wpad(d.n_fft, 0.0f);
    for (size_t k = 0; k < d.win_length; ++k) wpad[p->pad_left + k] = p->window[k];
    // W_NC^m, m < NC (f64-evaluated like rustfft's twiddles) and the realfft sin_cos table
    std::vector<float> tw(2 * std::max<size_t>(p->NC, 1));
    for (size_t m = 0; m < p->NC; ++m) {
        const double ang = -2.0 * 3.14159265358979323846 * (double)m / (double)p->NC;
        tw[2 * m] = (float)std::cos(ang);
        tw[2 * m + 1] = (float)std::sin(ang);
    }
    // stft2's lane-major stage-1 twiddle bases: row b < TB holds W_NC^{j*b}, row TB + a holds
    // W_NC^{j*TB*a}, column j < L (the same f64-rounded values as tw)
    std::vector<float> tw2;
    {
        int L = 0;
        if (stft_kernel_info((int)d.n_fft, nullptr, nullptr, &L) == 0 && L > 0 && p->NC >= (size_t)L) {
            const size_t P = p->NC / (size_t)L, TB = P < 8 ? P : 8, TA = P / TB;
            tw2.resize(2 * (TB + TA) * (size_t)L);
            for (size_t row = 0; row < TB + TA; ++row)
                for (size_t j = 0; j < (size_t)L; ++j) {
                    const size_t e = (row < TB ? j * row : j * TB * (row - TB)) % p->NC;
                    tw2[2 * (row * L + j)] = tw[2 * e];
                    tw2[2 * (row * L + j) + 1] = tw[2 * e + 1];
                }
        }
        if (tw2.empty()) tw2.assign(2, 0.0f);
    }
    // stft3's lane-major full stage-1 twiddles: [k1][j] = W_NC^{j*k1} (f64-rounded)
    std::vector<float> tw3;
    {
        int L = 0;
        if (stft_kernel_info((int)d.n_fft, nullptr, nullptr, &L) == 0 && L > 0 && p->NC >= (size_t)L) {
            const size_t P = p->NC / (size_t)L;
            tw3.resize(2 * P * (size_t)L);
            for (size_t k1 = 0; k1 < P; ++k1)
                for (size_t j = 0; j < (size_t)L; ++j) {
                    const size_t e = (j * k1) % p->NC;
                    tw3[2 * (k1 * L + j)] = tw[2 * e];
                    tw3[2 * (k1 * L + j) + 1] = tw[2 * e + 1];
                }
        }
        if (tw3.empty()) tw3.assign(2, 0.0f);
    }
    std::vector<float> sc = rfft_sin_cos(d.n_fft);
    const bool power = d.output == THESIA_OUT_POWER || d.output == THESIA_OUT_POWER_DB;
    p->log_amin = power ? log10f(1e-36f) : log10f(1e-18f);  // decibel.rs:7-8, :43
    int rc = p->wpad.upload(wpad.data(), wpad.size() * sizeof(float));
    if (!rc) rc = p->tw.upload(tw.data(), tw.size() * sizeof(float));
    if (!rc) rc = p->tw2.upload(tw2.data(), tw2.size() * sizeof(float));
    if (!rc) rc = p->tw3.upload(tw3.data(), tw3.size() * sizeof(float));
    if (!rc) rc = p->sincos.upload(sc.data(), sc.size() * sizeof(float));
    // the reference-order kernel: rustfft prepare_radix4 positions (oracle cfft_tab) and the
    // base butterfly_8 twiddles
    if (!rc) {
        const size_t NC = p->NC;
        std::vector<int> src(std::max<size_t>(NC, 1)), pos(std::max<size_t>(NC, 1));
        for (size_t i = 0; i < NC; ++i) src[i] = (int)i;
        if (NC > 4) {
            std::vector<int> idn(src);
            prepare_radix4_order(NC, idn.data(), src.data(), 1);
        }
        for (size_t jj = 0; jj < NC; ++jj) pos[(size_t)src[jj]] = (int)jj;
        rc = p->xpos.upload(pos.data(), pos.size() * sizeof(int));
        const double a1 = -2.0 * 3.14159265358979323846 * 1.0 / 8.0, a3 = -2.0 * 3.14159265358979323846 * 3.0 / 8.0;
        p->xw8[0] = (float)std::cos(a1); p->xw8[1] = (float)std::sin(a1);
        p->xw8[2] = (float)std::cos(a3); p->xw8[3] = (float)std::sin(a3);
    }
    if (!rc && (d.output == THESIA_OUT_MEL || d.output == THESIA_OUT_MEL_AMP_DB)) {
        const size_t F = p->NC + 1;
        if (d.mel_fb) {
            if (d.n_mels == 0) rc = set_error(THESIA_ERR_INVALID_ARG, "custom mel_fb needs n_mels");
            else { p->n_mels = d.n_mels; p->mel_fb.assign(d.mel_fb, d.mel_fb + F * d.n_mels); }
        } else if (d.n_mels == 0) {
            size_t nm = 0;
            p->mel_fb = calc_mel_fb_default(d.sr, d.n_fft, &nm);  // mel.rs:87-99
            p->n_mels = nm;
            if (nm == 0) rc = set_error(THESIA_ERR_INVALID_ARG, "no valid mel filterbank");
        } else {
            p->n_mels = d.n_mels;
            p->mel_fb = calc_mel_fb(d.sr, d.n_fft, d.n_mels, d.fmin, d.fmax, true);
        }
        if (!rc) rc = build_mel(p);
        if (!rc) rc = build_mel4(p);
        for (int i = 0; i < 2 && !rc; ++i) rc = build_melp(p, 2 + i, p->melp[i]);
        for (int i = 0; i < 2 && !rc; ++i) rc = build_melp(p, 2 + i, p->melr[i], 64, stftr_region_floats());
        if (!rc) {  // default: the fewest estimated instructions per chunk stream (5 + 6 S each)
            long bc = -1;
            for (int i = 0; i < 2; ++i)
                if (p->melp[i].chunks > 0) {
                    const long c = (long)p->melp[i].chunks * (5 + 6 * p->melp[i].steps);
                    if (bc < 0 || c < bc) { bc = c; p->melp_best = i; }
                }
            bc = -1;
            for (int i = 0; i < 2; ++i)
                if (p->melr[i].chunks > 0) {
                    const long c = (long)p->melr[i].chunks * (5 + 6 * p->melr[i].steps);
                    if (bc < 0 || c < bc) { bc = c; p->melr_best = i; }
                }
        }
        if (!rc) {  // the reference-order kernel: each mel's nonzero band, weights flat
            const size_t M = p->n_mels;
            std::vector<int4> band(std::max<size_t>(M, 1), int4{0, 0, 0, 0});
            std::vector<float> w;
            for (size_t m = 0; m < M; ++m) {
                long lo = -1, hi = -1;
                for (size_t k = 0; k < F; ++k)
                    if (p->mel_fb[k * M + m] != 0.0f) {
                        if (lo < 0) lo = (long)k;
                        hi = (long)k + 1;
                    }
                if (lo < 0) lo = hi = 0;
                band[m] = int4{(int)lo, (int)(hi - lo), (int)w.size(), 0};
                for (long k = lo; k < hi; ++k) w.push_back(p->mel_fb[(size_t)k * M + m]);
            }
            if (w.empty()) w.push_back(0.0f);
            rc = p->xmel_band.upload(band.data(), band.size() * sizeof(int4));
            if (!rc) rc = p->xmel_w.upload(w.data(), w.size() * sizeof(float));
        }
    }
    if (!rc) {
        p->use_v2 = stft2_supports((int)d.n_fft);
        if (p->use_v2) stft2_kernel_info((int)d.n_fft, &p->lds_bytes, &p->tile_frames, nullptr);
        else stft_kernel_info((int)d.n_fft, &p->lds_bytes, &p->tile_frames, nullptr);
    }
    if (rc) {
        delete p;
        return rc;
    }
    *out = p;
    return THESIA_OK;
}

// ------------------------------------------------------------------------------------
// batches
// ------------------------------------------------------------------------------------
Batch::~Batch() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
}

int batch_create(Plan* plan, const thesia_batch_desc& d, Batch** out) {
    *out = nullptr;
    if (!plan) return set_error(THESIA_ERR_INVALID_ARG, "null plan");
    if (d.channels == 0) return set_error(THESIA_ERR_INVALID_ARG, "channels must be > 0");
    if (d.input_format != THESIA_IN_F32 && d.input_format != THESIA_IN_S16)
        return set_error(THESIA_ERR_INVALID_ARG, "unknown input format");
    if (d.n_tracks == 0 || d.n_tracks > (size_t)0x7fffffff)
        return set_error(THESIA_ERR_INVALID_ARG, "n_tracks must be in [1, 2^31)");
    if (!d.d_input || !d.d_output || !d.track_offset || !d.track_len)
        return set_error(THESIA_ERR_INVALID_ARG, "null pointer in batch description");
    Batch* b = new Batch();
    b->plan = plan;
    b->desc = d;
    b->in_off.assign(d.track_offset, d.track_offset + d.n_tracks);
    b->len.assign(d.track_len, d.track_len + d.n_tracks);
    b->frame0.resize(d.n_tracks + 1);
    uint64_t acc = 0;
    for (size_t i = 0; i < d.n_tracks; ++i) {
        b->frame0[i] = acc;
        const uint64_t T = stft_n_frames(b->len[i], plan->win, plan->hop);
        if (T == 0) {
            delete b;
            return set_error(THESIA_ERR_TOO_SHORT,
                             "track " + std::to_string(i) + " is too short for win_length " +
                                 std::to_string(plan->win) + " (the reference panics, lib.rs:413)");
        }
        acc += T;
    }
    b->frame0[d.n_tracks] = acc;
    b->total_frames = acc;
    // the three per-track tables in one allocation (one hipMalloc / hipFree per batch)
    std::vector<uint64_t> tabs;
    tabs.reserve(3 * d.n_tracks + 1);
    tabs.insert(tabs.end(), b->in_off.begin(), b->in_off.end());
    tabs.insert(tabs.end(), b->len.begin(), b->len.end());
    tabs.insert(tabs.end(), b->frame0.begin(), b->frame0.end());
    int rc = b->d_tabs.upload(tabs.data(), tabs.size() * 8);
    if (rc) {
        delete b;
        return rc;
    }
    StftLaunch& L = b->launch;
    L.n_fft = (int)plan->n_fft;
    L.win = (int)plan->win;
    L.hop = (int)plan->hop;
    L.pad_left = (int)plan->pad_left;
    L.out_kind = plan->out_kind;
    L.in_format = d.input_format;
    L.channels = (int)d.channels;
    L.fold = (d.channels > 1 || d.fold_mono || d.input_format == THESIA_IN_S16) ? 1 : 0;
    L.in = d.d_input;
    L.trk_in_off = b->d_tabs.as<uint64_t>();
    L.trk_len = L.trk_in_off + d.n_tracks;
    L.trk_frame0 = L.trk_len + d.n_tracks;
    L.n_tracks = (int)d.n_tracks;
    L.total_frames = b->total_frames;
    L.wpad = plan->wpad.as<float>();
    L.tw1 = plan->tw.as<float2>();
    L.sincos = plan->sincos.as<float2>();
    L.tw2 = plan->tw2.as<float2>();
    L.tw3 = plan->tw3.as<float2>();
    L.log_amin = plan->log_amin;
    L.n_mels = (int)plan->n_mels;
    L.mel_rounds = plan->mel_rounds;
    L.mel_round = plan->mel_round.as<int2>();
    L.mel_k0 = plan->mel_k0.as<int>();
    L.mel_wt = plan->mel_wt.as<float>();
    L.mel4_rounds = plan->mel4_rounds;
    L.mel4_rows = (int)plan->mel4_wt_rows;
    L.mel4_round = plan->mel4_round.as<int2>();
    L.mel4_k0 = plan->mel4_k0.as<int>();
    L.mel4_wt = plan->mel4_wt.as<float4>();
    L.xpos = plan->xpos.as<int>();
    for (int i = 0; i < 4; ++i) L.xw8[i] = plan->xw8[i];
    L.xmel_band = plan->xmel_band.as<int4>();
    L.xmel_w = plan->xmel_w.as<float>();
    L.mel_chunks = plan->mel_chunks;
    L.mel_xo = plan->mel_xo.as<int>();
    L.out = d.d_output;
    b->apply_mel_path();
    // kernel choice: the streaming kernel for its geometry, else the 4-waves/SIMD kernel for
    // its sizes, else the general one (thesia_batch_set_option can force another one)
    b->k3_ok = plan->use_v2 && stft3_supports((int)plan->n_fft, (int)plan->win, (int)plan->hop,
                                              d.input_format, (int)d.channels) &&
               stft3_lds_bytes(L) <= 163840;  // the mel weights must fit LDS (else stft2)
    // (the viewer geometry runs stft5 for the mel and linear kinds only: complex rows stay on stft3)
    const bool view5 = !(plan->win == plan->n_fft && plan->hop * 4 == plan->n_fft);
    const bool k5_geo = b->k3_ok && stft5_supports((int)plan->n_fft, (int)plan->win, (int)plan->hop,
                                                   d.input_format, (int)d.channels) &&
                        !(view5 && L.out_kind == OUT_COMPLEX);
    if (k5_geo && L.melp_chunks && stft5_lds_bytes(L) > 163840) {  // packed stream too big: rounds
        b->mel_path = 1;
        b->apply_mel_path();
    }
    b->k5_ok = k5_geo && stft5_lds_bytes(L) <= 163840;
    // the reference-order streaming kernels (kernel 7): stftr at the canonical n_fft 2048
    // geometry (mel kinds need its packed stream, 64 lanes per frame), stftq at n_fft 256 / 512 /
    // 1024
    if (plan->melr_best >= 0) {
        const Plan::Melp& m = plan->melr[plan->melr_best];
        L.melr_chunks = m.chunks;
        L.melr_steps = m.steps;
        L.melr_meta = m.meta.as<int4>();
        L.melr_wt = m.wt.as<float4>();
    }
    const bool mel_kind = L.out_kind == OUT_MEL || L.out_kind == OUT_MEL_AMP_DB;
    b->kr_ok = (stftr_supports((int)plan->n_fft, (int)plan->win, (int)plan->hop, d.input_format, (int)d.channels) &&
                (!mel_kind || L.melr_chunks > 0) && stftr_lds_bytes(L) <= 163840) ||
               (stftq_supports((int)plan->n_fft, (int)plan->win, (int)plan->hop, d.input_format, (int)d.channels) &&
                stftq_lds_bytes(L) <= 163840);
    b->k5_view = view5;
    b->kernel = b->auto_kernel();
    if (hipEventCreate(&b->ev0) != hipSuccess || hipEventCreate(&b->ev1) != hipSuccess) {
        delete b;
        return set_error(THESIA_ERR_DEVICE, "hipEventCreate failed");
    }
    *out = b;
    return THESIA_OK;
}

void Batch::apply_mel_path() {
    StftLaunch& L = launch;
    L.melp_chunks = L.melp_steps = L.melp_v4 = 0;
    L.melp_meta = nullptr;
    L.melp_wt = nullptr;
    const int idx = mel_path == 0 ? plan->melp_best : mel_path >= 2 ? mel_path - 2 : -1;
    if (idx < 0 || plan->melp[idx].chunks == 0) return;
    const Plan::Melp& m = plan->melp[idx];
    L.melp_chunks = m.chunks;
    L.melp_steps = m.steps;
    L.melp_meta = m.meta.as<int4>();
    L.melp_wt = m.wt.as<float4>();
    L.melp_v4 = plan->n_mels % 4 == 0 && plan->n_mels <= 128 &&
                (reinterpret_cast<uintptr_t>(L.out) & 15) == 0;
}

int batch_set_option(Batch* b, int option, int64_t value) {
    switch (option) {
        case THESIA_BATCH_OPT_KERNEL:
            if (value == 0) b->kernel = b->auto_kernel();
            else if (value == 1) b->kernel = 1;
            else if (value == 2 && stft2_supports((int)b->plan->n_fft)) b->kernel = 2;
            else if (value == 3 && b->k3_ok) b->kernel = 3;
            else if (value == 5 && b->k5_ok) b->kernel = 5;
            else if (value == 7 && b->kr_ok) b->kernel = 7;
            else if (value == 9 && stftx_lds_bytes((int)b->plan->n_fft, true) <= 163840) b->kernel = 9;
            else return set_error(THESIA_ERR_UNSUPPORTED, "kernel " + std::to_string(value) +
                                                             " does not run this batch's geometry");
            b->kernel_forced = value != 0;
            return THESIA_OK;
        case THESIA_BATCH_OPT_MAX_BLOCKS:
            if (value < 0 || value > (1 << 30)) return set_error(THESIA_ERR_INVALID_ARG, "max_blocks out of range");
            b->launch.grid = (int)value;
            return THESIA_OK;
#ifdef THESIA_STAMPS
        case 100:  // diagnostic build: device buffer for the stft5 phase stamps (scripts/stamps.py)
            b->launch.stamps = reinterpret_cast<unsigned long long*>(value);
            return THESIA_OK;
#endif
        case THESIA_BATCH_OPT_RANGE:
            if (value != 0 && b->launch.out_kind == OUT_COMPLEX)
                return set_error(THESIA_ERR_INVALID_ARG, "ranges need real output rows");
            b->range = reinterpret_cast<int*>(value);
            if (!b->kernel_forced) b->kernel = b->auto_kernel();  // the range decides stft3 vs stft5
            return THESIA_OK;
        case THESIA_BATCH_OPT_MEL_PATH: {
            if (value < 0 || value > 3) return set_error(THESIA_ERR_INVALID_ARG, "mel_path must be 0..3");
            if (value >= 2 && b->plan->melp[value - 2].chunks == 0)
                return set_error(THESIA_ERR_UNSUPPORTED, "no packed mel stream for this plan");
            const int prev = b->mel_path;
            b->mel_path = (int)value;
            b->apply_mel_path();
            if (b->k5_ok && stft5_lds_bytes(b->launch) > 163840) {
                b->mel_path = prev;
                b->apply_mel_path();
                return set_error(THESIA_ERR_UNSUPPORTED, "the mel tables of that path do not fit LDS");
            }
            return THESIA_OK;
        }
        case THESIA_BATCH_OPT_ROW_STORE:
            if (value < 0 || value > 3) return set_error(THESIA_ERR_INVALID_ARG, "row_store must be 0..3");
            // 2 and 3 name complex-row methods: on real rows they would change nothing but turn
            // the in-epilogue range fold off
            if (value >= 2 && b->launch.out_kind != OUT_COMPLEX)
                return set_error(THESIA_ERR_INVALID_ARG, "row_store 2 / 3 apply to complex rows only");
            b->launch.row_alt = (int)value;
            return THESIA_OK;
        default:
            return set_error(THESIA_ERR_INVALID_ARG, "unknown batch option");
    }
}

int batch_run(Batch* b, hipStream_t s) {
    if (!s) s = default_stream();
    // per-track output ranges: folded into stft3's staged-row epilogue (linear kinds) and into
    // kernel 7's (amp dB), else one reduction pass over the rows after the spectrogram launch
    const uint64_t n_tr = b->frame0.empty() ? 0 : b->frame0.size() - 1;
    const bool lin = b->launch.out_kind != OUT_COMPLEX && b->launch.out_kind != OUT_MEL &&
                     b->launch.out_kind != OUT_MEL_AMP_DB;
    bool in_kernel = false;
    if (b->range && launch_range_init(b->range, n_tr, s))
        return set_error(THESIA_ERR_DEVICE, "range init launch failed");
    int rc = -2;
    if (b->kernel == 9) {
        rc = launch_stftx(b->launch, s);
        if (rc) return set_error(rc == -2 ? THESIA_ERR_UNSUPPORTED : THESIA_ERR_DEVICE, "stftx launch failed");
    } else if (b->kernel == 7) {
        const bool r = b->plan->n_fft == 2048;
        // amp dB rows fold their range into the epilogue (stftq / stftr RG instances)
        const bool fold = b->range && b->launch.out_kind == OUT_AMP_DB;
        b->launch.trk_range = fold ? b->range : nullptr;
        rc = r ? launch_stftr(b->launch, s) : launch_stftq(b->launch, s);
        in_kernel = fold && rc == 0;
        b->launch.trk_range = nullptr;
        if (rc)
            return set_error(rc == -2 ? THESIA_ERR_UNSUPPORTED : THESIA_ERR_DEVICE,
                             r ? "stftr launch failed" : "stftq launch failed");
    } else {
        if (b->kernel == 5) rc = launch_stft5(b->launch, s);
        if (rc == -2 && b->kernel >= 3) {
            const bool fold = b->range && lin && b->launch.row_alt == 0;
            b->launch.trk_range = fold ? b->range : nullptr;
            rc = launch_stft3(b->launch, s);
            in_kernel = fold && rc == 0;
            b->launch.trk_range = nullptr;
        }
        if (rc == -2 && b->kernel >= 2) rc = launch_stft2(b->launch, s);
        if (rc == -2) rc = launch_stft(b->launch, s);
        if (rc == -2) return set_error(THESIA_ERR_UNSUPPORTED, "unsupported n_fft");
        if (rc) return set_error(THESIA_ERR_DEVICE, std::string("stft launch failed: ") +
                                                        hipGetErrorString(hipGetLastError()));
    }
    if (b->range && !in_kernel &&
        launch_range_rows(static_cast<const float*>(b->desc.d_output), b->launch.trk_frame0, n_tr,
                          (uint32_t)b->plan->row_bins(), b->range, s))
        return set_error(THESIA_ERR_DEVICE, "range launch failed");
#ifndef THESIA_DIAG_NO_LAST_USE  // (diagnostic build: the round-5 cache, for the test's control)
    b->d_tabs.used_on(s);  // the kernels just enqueued on s read the track tables
#endif
    return THESIA_OK;
}

// Library streams of the device (created once, kept), forked from and joined back to a caller's
// stream: the work of independent launches (batches_run's batches, render_rgb_fused's groups)
// overlaps, so one launch's ramp and tail fill with another's blocks. Callers hold
// run_pool_mutex() from the fork to the join (the events are shared).
struct RunPool {
    static constexpr int kStreams = 4;
    hipStream_t st[kStreams] = {};
    hipEvent_t fork = nullptr, join[kStreams] = {};
    hipError_t fork_from(hipStream_t s, int k) {
        hipError_t e = hipEventRecord(fork, s);
        for (int i = 0; i < k && e == hipSuccess; ++i) e = hipStreamWaitEvent(st[i], fork, 0);
        return e;
    }
    int join_into(hipStream_t s, int k) {
        hipError_t e = hipSuccess;
        for (int i = 0; i < k; ++i) {
            hipError_t e1 = hipEventRecord(join[i], st[i]);
            if (e1 == hipSuccess) e1 = hipStreamWaitEvent(s, join[i], 0);
            if (e == hipSuccess) e = e1;
        }
        return e == hipSuccess ? THESIA_OK : set_error(THESIA_ERR_DEVICE, hipGetErrorString(e));
    }
};
static std::mutex& run_pool_mutex() {
    static auto& mu = *new std::mutex();  // leaked, see dev_taps
    return mu;
}
static int run_pool(RunPool** out) {  // caller holds run_pool_mutex()
    static auto& pools = *new std::map<int, RunPool>();  // leaked, see dev_taps
    int dev = 0;
    (void)hipGetDevice(&dev);
    RunPool& p = pools[dev];
    if (!p.fork) {
        for (int i = 0; i < RunPool::kStreams; ++i) {
            THESIA_HIP(hipStreamCreateWithFlags(&p.st[i], hipStreamNonBlocking));
            THESIA_HIP(hipEventCreateWithFlags(&p.join[i], hipEventDisableTiming));
        }
        THESIA_HIP(hipEventCreateWithFlags(&p.fork, hipEventDisableTiming));
    }
    *out = &p;
    return THESIA_OK;
}

// Several batches (e.g. one per geometry group) on up to kRunStreams library streams of the
// device, forked from and joined back to `s`: a small launch's ramp (the first frame of every
// stream loaded without prefetch, the tables staged into LDS) overlaps the others' work.
// Stream-ordered on `s` like batch_run.
int batches_policy();
int batches_run(Batch* const* b, size_t n, hipStream_t s) {
    if (!s) s = default_stream();
    if (n <= 1) return n ? batch_run(b[0], s) : THESIA_OK;
    {  // the batches run concurrently: the same batch twice would race on its output and ranges
        std::vector<const Batch*> seen(b, b + n);
        std::sort(seen.begin(), seen.end());
        if (std::adjacent_find(seen.begin(), seen.end()) != seen.end() || seen.front() == nullptr)
            return set_error(THESIA_ERR_INVALID_ARG, "batches_run: a batch handle appears twice (or is null)");
    }
    if (batches_policy() == 2) {  // one after another on the caller's stream
        for (size_t i = 0; i < n; ++i) {
            const int rc = batch_run(b[i], s);
            if (rc) return rc;
        }
        return THESIA_OK;
    }
    std::lock_guard<std::mutex> lk(run_pool_mutex());
    RunPool* p = nullptr;
    int rc = run_pool(&p);
    if (rc) return rc;
    const int k = (int)std::min<size_t>(RunPool::kStreams, n);
    // policy 1: every batch whose block count the caller left automatic gets a share of one
    // occupancy wave proportional to its work (frames x n_fft log2 n_fft), so the concurrent
    // batches sit on disjoint CUs and each frame stream walks more frames (a stream's ring
    // prologue reads 4 hops to produce its first frame); policy 0: each batch takes a whole wave
    std::vector<float> share(n, 0.f);
    if (batches_policy() == 1 && n <= (size_t)k) {
        double tot = 0;
        std::vector<double> w(n, 0.0);
        for (size_t i = 0; i < n; ++i) {
            const double nf = (double)b[i]->plan->n_fft;
            w[i] = (double)b[i]->total_frames * nf * std::log2(std::max(nf, 2.0));
            tot += w[i];
        }
        for (size_t i = 0; i < n && tot > 0; ++i) share[i] = (float)(w[i] / tot);
    }
    THESIA_HIP(p->fork_from(s, k));
    for (size_t i = 0; i < n && !rc; ++i) {
        const float keep = b[i]->launch.grid_share;
        b[i]->launch.grid_share = share[i];
        rc = batch_run(b[i], p->st[i % k]);
        b[i]->launch.grid_share = keep;
    }
    const int jrc = p->join_into(s, k);  // join even after an error: `s` never runs ahead of them
    for (size_t i = 0; i < n; ++i) b[i]->d_tabs.used_on(s);  // the forks are joined into s
    return rc ? rc : jrc;
}

static int g_batches_policy = 0;  // thesia_set_batches_policy
int batches_policy() { return __atomic_load_n(&g_batches_policy, __ATOMIC_RELAXED); }
int set_batches_policy(int policy) {
    if (policy < 0 || policy > 2) return set_error(THESIA_ERR_INVALID_ARG, "batches policy must be 0, 1 or 2");
    __atomic_store_n(&g_batches_policy, policy, __ATOMIC_RELAXED);
    return THESIA_OK;
}

// host side of Batch::range: {ord max, ord min, NaN} -> (max, min, NaN) per track
int ranges_read(const int* d_range, size_t n, float* mx, float* mn, int* nan, hipStream_t s) {
    if (n == 0) return THESIA_OK;
    std::vector<int> h(3 * n);
    THESIA_HIP(copy_on(h.data(), d_range, h.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    THESIA_HIP(hipStreamSynchronize(s));
    for (size_t i = 0; i < n; ++i) {
        mx[i] = range_unord(h[3 * i]);
        mn[i] = range_unord(h[3 * i + 1]);
        nan[i] = h[3 * i + 2];
    }
    return THESIA_OK;
}

// ------------------------------------------------------------------------------------
// display helpers
// ------------------------------------------------------------------------------------
int minmax_device(const float* d_x, uint64_t n, float* mx, float* mn, bool* nan, hipStream_t s) {
    if (n == 0) {  // ndarray-stats EmptyInput -> unwrap_or(-inf / +inf), lib.rs:198-199
        *mx = -INFINITY;
        *mn = INFINITY;
        *nan = false;
        return THESIA_OK;
    }
    int nblk = (int)std::min<uint64_t>((n + 255) / 256, 1024);
    DevBuf part, flag;
    int rc = part.alloc((size_t)nblk * 2 * sizeof(float));
    if (!rc) rc = flag.alloc(sizeof(int));
    if (rc) return rc;
    THESIA_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    if (launch_minmax(d_x, n, part.as<float>(), flag.as<int>(), nblk, s))
        return set_error(THESIA_ERR_DEVICE, "minmax launch failed");
    std::vector<float> h((size_t)nblk * 2);
    int hf = 0;
    THESIA_HIP(copy_on(h.data(), part.p, h.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    THESIA_HIP(copy_on(&hf, flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    THESIA_HIP(hipStreamSynchronize(s));
    float a = -INFINITY, b = INFINITY;
    for (int i = 0; i < nblk; ++i) {
        a = fmaxf(a, h[2 * i]);
        b = fminf(b, h[2 * i + 1]);
    }
    *mx = a;
    *mn = b;
    *nan = hf != 0;
    return THESIA_OK;
}

static int g_render_path = 0;  // thesia_set_render_path

int render_path() { return __atomic_load_n(&g_render_path, __ATOMIC_RELAXED); }
int set_render_path(int path) {
    if (path < 0 || path > 5) return set_error(THESIA_ERR_INVALID_ARG, "render path must be 0 .. 5");
    __atomic_store_n(&g_render_path, path, __ATOMIC_RELAXED);
    return THESIA_OK;
}

static std::vector<uint8_t> colormap_bytes() {
    std::vector<uint8_t> c(30);
    for (int i = 0; i < 10; ++i)
        for (int k = 0; k < 3; ++k) c[i * 3 + k] = kColormap[i][k];
    return c;
}

// Lanczos3 tap tables of one (size -> new size) resample, resident in HBM. Cached per
// (device, size, new size): a batch of same-geometry images uploads them once.
struct DevTaps {
    DevBuf left, count, offset, weights;
    int max_taps = 0;
    std::vector<int32_t> h_left, h_count;  // host copies (block spans of the fused render)
    // the taps regrouped by 8-frame step for render_stripe_kernel (RenderDesc::hst / hsw), built
    // on first use per slot count A (8, 12, 16): per step its first column ca, and the weights
    // [step][frame u][slot a] of columns ca + a (+0 outside a column's support and past na)
    int st_maxna = -1;  // most columns meeting one step (-1: not computed yet)
    std::vector<int32_t> h_st_ca;
    DevBuf st_ca[3], st_w[3];
};

static int dev_taps(uint32_t n, uint32_t nn, const DevTaps** out) {
    static std::mutex mu;
    // intentionally leaked: freeing HBM from a static destructor would race HIP's teardown
    static auto& cache = *new std::map<std::tuple<int, uint32_t, uint32_t>, std::unique_ptr<DevTaps>>();
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(dev, n, nn);
    auto it = cache.find(key);
    if (it == cache.end()) {
        Taps t = lanczos3_taps(n, nn);
        auto d = std::make_unique<DevTaps>();
        int rc = d->left.upload(t.left.data(), t.left.size() * 4);
        if (!rc) rc = d->count.upload(t.count.data(), t.count.size() * 4);
        if (!rc) rc = d->offset.upload(t.offset.data(), t.offset.size() * 4);
        if (!rc) rc = d->weights.upload(t.weights.data(), t.weights.size() * 4);
        if (rc) return rc;
        d->max_taps = t.max_taps;
        d->h_left.assign(t.left.begin(), t.left.end());
        d->h_count.assign(t.count.begin(), t.count.end());
        it = cache.emplace(key, std::move(d)).first;
    }
    *out = it->second.get();
    return THESIA_OK;
}

// The stepped form of an (n -> nn) tap table: step s covers frames [8s, 8s + 8); its columns are
// those whose support [l, l + cnt) meets the step, ca .. ca + na - 1 (supports are monotone in
// the column); render_stripe_kernel's slot a of the step holds column ca + a, with the 8 weights
// of the step's frames (the column's weight where the frame is inside its support, +0 elsewhere
// and for a >= na), laid out [step][frame][slot].
static void stepped_cols(const DevTaps& t, uint32_t n, uint32_t nn, std::vector<int32_t>* ca_out, int* maxna) {
    const int nsteps = (int)((n + 7) / 8);
    ca_out->assign(nsteps, 0);
    int ca = 0, cb = -1, mx = 0;
    for (int s = 0; s < nsteps; ++s) {
        while (ca < (int)nn && ((t.h_left[ca] + t.h_count[ca] - 1) >> 3) < s) ++ca;
        while (cb + 1 < (int)nn && (t.h_left[cb + 1] >> 3) <= s) ++cb;
        (*ca_out)[s] = ca;
        mx = std::max(mx, cb >= ca ? cb - ca + 1 : 0);
    }
    *maxna = mx;
}

static int dev_taps_stepped(uint32_t n, uint32_t nn, int slots, const DevTaps** out) {
    const DevTaps* t = nullptr;
    int rc = dev_taps(n, nn, &t);
    if (rc) return rc;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    DevTaps* d = const_cast<DevTaps*>(t);  // the cache owns it; only this function adds the steps
    if (d->st_maxna < 0) stepped_cols(*d, n, nn, &d->h_st_ca, &d->st_maxna);
    const int k = slots / 4 - 2;
    if (slots > 0 && (k < 0 || k > 2 || slots % 4)) return set_error(THESIA_ERR_INVALID_ARG, "stepped taps: 8, 12 or 16 slots");
    if (slots > 0 && !d->st_w[k].p) {
        const Taps tp = lanczos3_taps(n, nn);
        const int nsteps = (int)d->h_st_ca.size();
        std::vector<float> w((size_t)nsteps * 8 * slots, 0.0f);
        for (int s = 0; s < nsteps; ++s)
            for (int a = 0; a < slots; ++a) {
                const int c = d->h_st_ca[s] + a;
                if (c >= (int)nn) break;
                const int l = tp.left[c], cnt = tp.count[c];
                for (int u = 0; u < 8; ++u) {
                    const int f = 8 * s + u;
                    if (f >= l && f < l + cnt) w[((size_t)s * 8 + u) * slots + a] = tp.weights[tp.offset[c] + (f - l)];
                }
            }
        if (w.empty()) w.push_back(0.0f);
        rc = d->st_ca[k].upload(d->h_st_ca.data(), std::max<size_t>(d->h_st_ca.size(), 1) * 4);
        if (!rc) rc = d->st_w[k].upload(w.data(), w.size() * 4);
        if (rc) return rc;
    }
    *out = d;
    return THESIA_OK;
}

int grey_to_rgb_device(const float* d_grey, uint32_t w, uint32_t h, uint32_t nw, uint32_t nh,
                       uint8_t* d_rgb, hipStream_t s) {
    if (nw == 0 || nh == 0) return THESIA_OK;
    if (w == 0 || h == 0) return set_error(THESIA_ERR_INVALID_ARG, "empty grey image");
    // image 0.23.12 resize: vertical_sample (h -> nh) into f32, then horizontal (w -> nw)
    const DevTaps *vt = nullptr, *ht = nullptr;
    const uint8_t* cmap_ptr = nullptr;
    int rc = dev_taps(h, nh, &vt);
    if (!rc) rc = dev_taps(w, nw, &ht);
    if (rc) return rc;
    {  // the colormap LUT, once per device
        static std::mutex mu;
        static auto& cmaps = *new std::map<int, DevBuf>();  // leaked, see dev_taps
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> lk(mu);
        DevBuf& cm = cmaps[dev];
        if (!cm.p) {
            std::vector<uint8_t> bytes = colormap_bytes();
            rc = cm.upload(bytes.data(), bytes.size());
            if (rc) return rc;
        }
        cmap_ptr = cm.as<uint8_t>();
    }
    DevBuf tmp;
    rc = tmp.alloc((size_t)w * nh * sizeof(float));
    if (rc) return rc;
    if (launch_resize_v(d_grey, w, h, nh, vt->left.as<int32_t>(), vt->count.as<int32_t>(),
                        vt->offset.as<int32_t>(), vt->weights.as<float>(), vt->max_taps,
                        tmp.as<float>(), s))
        return set_error(THESIA_ERR_DEVICE, "resize_v launch failed");
    if (launch_resize_h_rgb(tmp.as<float>(), w, nh, nw, ht->left.as<int32_t>(),
                            ht->count.as<int32_t>(), ht->offset.as<int32_t>(),
                            ht->weights.as<float>(), ht->max_taps, cmap_ptr, d_rgb, s))
        return set_error(THESIA_ERR_DEVICE, "resize_h launch failed");
    THESIA_HIP(hipStreamSynchronize(s));
    return THESIA_OK;
}

static int minmax_segments_core(size_t n_groups, const float* const* d_x, const uint64_t* const* row0,
                                const size_t* bins, const size_t* ns, float* mx, float* mn, int* nan,
                                hipStream_t s);

// Calls of more than 65535 tracks (the launch's grid.y limit) run as consecutive pieces of at
// most that many tracks (a group's track range is cut where needed: row0 + i0 is the row table of
// its tracks i0.. as it stands); the outputs stay in the concatenated group order.
int minmax_segments_multi(size_t n_groups, const float* const* d_x, const uint64_t* const* row0,
                          const size_t* bins, const size_t* ns, float* mx, float* mn, int* nan,
                          hipStream_t s) {
    constexpr size_t kMax = 65535;
    size_t ntr = 0;
    for (size_t k = 0; k < n_groups; ++k) ntr += ns[k];
    if (ntr <= kMax) return minmax_segments_core(n_groups, d_x, row0, bins, ns, mx, mn, nan, s);
    std::vector<const float*> px;
    std::vector<const uint64_t*> pr;
    std::vector<size_t> pb, pn;
    size_t in_piece = 0, done = 0;
    auto flush = [&]() -> int {
        if (px.empty()) return THESIA_OK;
        const int rc = minmax_segments_core(px.size(), px.data(), pr.data(), pb.data(), pn.data(), mx + done,
                                            mn + done, nan + done, s);
        done += in_piece;
        in_piece = 0;
        px.clear(); pr.clear(); pb.clear(); pn.clear();
        return rc;
    };
    for (size_t k = 0; k < n_groups; ++k) {
        for (size_t i0 = 0; i0 < ns[k];) {
            const size_t c = std::min(ns[k] - i0, kMax - in_piece);
            px.push_back(d_x[k]);
            pr.push_back(row0[k] + i0);
            pb.push_back(bins[k]);
            pn.push_back(c);
            in_piece += c;
            i0 += c;
            if (in_piece == kMax) {
                const int rc = flush();
                if (rc) return rc;
            }
        }
    }
    return flush();
}

static int minmax_segments_core(size_t n_groups, const float* const* d_x, const uint64_t* const* row0,
                                const size_t* bins, const size_t* ns, float* mx, float* mn, int* nan,
                                hipStream_t s) {
    // one launch over every group's tracks: segment bounds are element offsets from the lowest
    // group buffer (one flat device address space), one table upload, one readback
    const float* base = nullptr;
    size_t ntr = 0;
    uint64_t tot = 0;
    for (size_t k = 0; k < n_groups; ++k) {
        if (ns[k] == 0) continue;
        if (!base || d_x[k] < base) base = d_x[k];
        ntr += ns[k];
        tot += (row0[k][ns[k]] - row0[k][0]) * bins[k];
    }
    if (ntr == 0) return THESIA_OK;
    // [lo, hi) per track: each track closed by its own end, so no segment spans the gap
    // between two groups' buffers
    std::vector<uint64_t> lo(ntr), hi(ntr);
    size_t t = 0;
    for (size_t k = 0; k < n_groups; ++k) {
        const uint64_t off = ns[k] ? (uint64_t)(d_x[k] - base) : 0;
        for (size_t i = 0; i < ns[k]; ++i, ++t) {
            lo[t] = off + row0[k][i] * bins[k];
            hi[t] = off + row0[k][i + 1] * bins[k];
        }
    }
    // blocks per track: enough to fill the device at the call's total size
    const int nper = (int)std::min<uint64_t>(64, std::max<uint64_t>(1, (tot / ntr) / (256 * 4 * 8)));
    // grow-only per-device workspace (a hipMalloc per call cost more than the reduction)
    struct Ws { DevBuf seg, part, flag; };
    static std::mutex ws_mu;
    static auto& ws_map = *new std::map<int, Ws>();  // leaked, see dev_taps
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(ws_mu);
    Ws& ws = ws_map[dev];
    auto grow = [](DevBuf& b, size_t bytes) {
        if (b.bytes >= bytes && b.p) return 0;
        b.release();
        return b.alloc(bytes + bytes / 8);
    };
    std::vector<uint64_t> bounds(2 * ntr);
    for (size_t i = 0; i < ntr; ++i) {
        bounds[2 * i] = lo[i];
        bounds[2 * i + 1] = hi[i];
    }
    int rc = grow(ws.seg, bounds.size() * 8);
    if (!rc) rc = grow(ws.part, ntr * nper * 2 * sizeof(float));
    if (!rc) rc = grow(ws.flag, ntr * sizeof(int));
    if (rc) return rc;
    THESIA_HIP(copy_on(ws.seg.p, bounds.data(), bounds.size() * 8, hipMemcpyHostToDevice, s));
    THESIA_HIP(hipMemsetAsync(ws.flag.p, 0, ntr * sizeof(int), s));
    if (launch_minmax_seg(base, ws.seg.as<uint64_t>(), (int)ntr, nper, ws.part.as<float>(), ws.flag.as<int>(), s))
        return set_error(THESIA_ERR_DEVICE, "minmax_seg launch failed");
    std::vector<float> h(ntr * nper * 2);
    std::vector<int> hf(ntr);
    THESIA_HIP(copy_on(h.data(), ws.part.p, h.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    THESIA_HIP(copy_on(hf.data(), ws.flag.p, ntr * sizeof(int), hipMemcpyDeviceToHost, s));
    THESIA_HIP(hipStreamSynchronize(s));
    for (size_t i = 0; i < ntr; ++i) {
        float a = -INFINITY, b = INFINITY;  // empty track: ndarray-stats EmptyInput -> -inf / +inf
        for (int q = 0; q < nper; ++q) {
            a = fmaxf(a, h[(i * nper + q) * 2]);
            b = fminf(b, h[(i * nper + q) * 2 + 1]);
        }
        mx[i] = a;
        mn[i] = b;
        nan[i] = hf[i];
    }
    return THESIA_OK;
}

int minmax_segments_device(const float* d_x, const uint64_t* row0, size_t bins, size_t n,
                           float* mx, float* mn, int* nan, hipStream_t s) {
    return minmax_segments_multi(1, &d_x, &row0, &bins, &n, mx, mn, nan, s);
}

#ifndef THESIA_VBAND
#define THESIA_VBAND 64  // widest vertical band tried (64 beat 128-512 on C5: more blocks)
#endif
#ifndef THESIA_STRIP
#define THESIA_STRIP 64  // output columns per stripe block (a multiple of 16)
#endif
#ifndef THESIA_VROWS
#define THESIA_VROWS 128  // grey rows per vertical tile (<= 256; A/B via scripts/build_variant.sh)
#endif

namespace {

const uint8_t* colormap_device(int* rc) {  // the colormap LUT, once per device
    static std::mutex mu;
    static auto& cmaps = *new std::map<int, DevBuf>();  // leaked, see dev_taps
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    DevBuf& cm = cmaps[dev];
    *rc = 0;
    if (!cm.p) {
        std::vector<uint8_t> bytes = colormap_bytes();
        *rc = cm.upload(bytes.data(), bytes.size());
        if (*rc) return nullptr;
    }
    return cm.as<uint8_t>();
}

// One group of the fused display path: tracks sharing one spectrogram buffer and bin count.
struct FusedGroup {
    const float* spec = nullptr;
    uint32_t bins = 0;
    size_t desc0 = 0, ndesc = 0;  // its RenderDesc range in the call's table
    uint64_t tmp_tot = 0;         // intermediate floats ([nheight][T] per track)
    uint32_t T_max = 0, H_max = 0, nw_max = 0, v_band = 1;
    int h_taps = 0, h_span = 0, v_rows = 1, v_kv = 4;
    int v_fpl = 1;  // frames per lane of the vertical pass (4: grey_vert_wide_kernel)
    uint64_t cost = 0;  // HBM floats its two passes move (spectrogram, intermediate twice, RGB / 4)
    int stream = 0;     // render_rgb_fused: the library stream it runs on
    // the single-pass display (render_stripe_kernel) where its instances cover the group's
    // geometry (plan_stripe); then no intermediate is formed
    bool stripe = false;
    uint32_t st_strip = THESIA_STRIP;
    int st_kv = 0, st_slots = 0, st_acc = 0, st_fc = 0, st_npf = 0, st_waves = 4, st_tile = 0, st_hdr = 0,
        st_wts = 0;
    int st_ring = 0, st_hg = 0;  // ring mode (render path 5): ring frames, tap groups of 4
    bool st_dword = false;
};

// Host planning of one group: a RenderDesc per non-empty track (appended to `desc`), the
// single-pass display where `stripe` asks for it (1 the automatic choice, 2 wherever covered), the
// vertical band (the widest whose grey rows <= THESIA_VROWS and weights <= 4096 fit the LDS
// tile for every track of the group) and the horizontal pass's tap / span bounds.
// The single-pass display for a group (render_stripe_kernel): the instance (KV vertical taps,
// A accumulator slots, FC frames per chunk) and the LDS bounds over every track, strip and row
// block; g.stripe stays false where no instance covers the group (more than 16 vertical taps, more
// than 16 columns meeting an 8-frame step, a chunk that does not fit the staging registers).
struct StripeTrack {
    const DevTaps *vt, *ht;
    uint32_t T, H, nw, oz;
    uint64_t rgb_off;
};
void plan_stripe_ring(const std::vector<StripeTrack>& trk, uint32_t bins, uint32_t nheight, FusedGroup& g) {
    int kvmax = 0, hcmax = 0;
    bool dword = true;
    for (const StripeTrack& t : trk) {
        if ((uint64_t)t.T * bins >= (1ull << 30)) return;  // the kernel's 32-bit byte offsets
        kvmax = std::max(kvmax, t.vt->max_taps);
        hcmax = std::max(hcmax, t.ht->max_taps);
        dword = dword && t.nw % 4 == 0 && t.rgb_off % 4 == 0;
    }
    const int kv = kvmax <= 7 ? 7 : kvmax <= 8 ? 8 : kvmax <= 12 ? 12 : kvmax <= 16 ? 16 : 0;
    const int hg = hcmax <= 8 ? 2 : hcmax <= 12 ? 3 : hcmax <= 16 ? 4 : hcmax <= 24 ? 6 : 0;
    if (!kv || !hg) return;
    int ring = 8;
    while (ring < hcmax + 7) ring *= 2;
    constexpr int kWaveRows = 64;
    const uint32_t strip = g.st_strip;
    int tile = 1, nbmax = 0;
    for (const StripeTrack& t : trk) {
        const int top = (int)t.H - (int)bins;
        for (uint32_t R0 = 0; R0 < nheight; R0 += kWaveRows) {
            const uint32_t rlo = std::max(R0, t.oz), rhi = std::min(R0 + kWaveRows, nheight);
            if (rlo >= rhi) continue;
            const int ya = t.vt->h_left[rlo], nt = t.vt->h_left[rhi - 1] + kv - ya;
            tile = std::max(tile, nt);
            nbmax = std::max(nbmax, std::min(ya + nt, (int)t.H) - std::max(ya, top));
        }
    }
    const int hdr = 2 * (int)strip, wts = (int)strip * 4 * hg, slots = ring + 4 * hg + 1;
    int fc = 16, npf = 16, waves = nheight > 256 ? 8 : 4;
    auto lds = [&]() { return render_stripe_lds_bytes(fc, tile, hdr, wts, waves, slots); };
    if (fc * nbmax > 64 * npf || lds() > (waves == 8 ? 81920 : 54613)) fc = 8;
    if (waves == 8 && lds() > 81920) waves = 4;
    if (fc * nbmax > 64 * npf || lds() > 163840) return;
    if (fc * (int)bins >= 65536 || tile * (fc + 4) >= 65536) return;
    g.stripe = true;
    g.st_kv = kv;
    g.st_slots = 4;
    g.st_acc = 1;
    g.st_fc = fc;
    g.st_npf = npf;
    g.st_waves = waves;
    g.st_tile = tile;
    g.st_hdr = hdr;
    g.st_wts = wts;
    g.st_dword = dword;
    g.st_ring = ring;
    g.st_hg = hg;
}

// Automatic choice (render path 0): only groups whose frames outnumber their image columns at
// least 3 to 1. There the two-kernel path's intermediate ([nheight][T] f32, written and read
// back) dominates its traffic, and the stripe kernel's fixed 8-frame steps waste few slots
// (about 8 + 6 T/nw columns meet a step, 6 of them with work per frame). Measured per C5 group
// alone (profiles/r04_display): 44.1 kHz / 256 (T/nw 6.9) 846 -> 575 us, 48 kHz / 512 (3.8)
// 604 -> 504, 22.05 kHz / 256 (3.4) 478 -> 419; slower at T/nw 1.25 .. 1.9 (8 kHz / 256 265 ->
// 291, 16 kHz / 512 293 -> 317, 24 kHz / 512 341 -> 349, 44.1 kHz / 1024 359 -> 394) and even
// below 1. Path 4 takes it wherever an instance covers the geometry.
// Ring mode (render path 5, round 6; `ring`): the groups below 3 frames per column, where the slot
// mode is not taken, run the stripe kernel with the horizontal sums over each column's exact taps
// from a per-lane LDS ring of the recent frames' vertical sums (render_stripe.hip): at most 24 taps
// per column (6 float4 groups), a ring of the next power of 2 >= taps + 7 frames.
void plan_stripe(const std::vector<StripeTrack>& trk, uint32_t bins, uint32_t nheight, FusedGroup& g,
                 bool force, bool ring = false) {
    g.stripe = false;
    g.st_ring = g.st_hg = 0;
    if (trk.empty()) return;
    if (!force) {
        uint64_t frames = 0, cols = 0;
        for (const StripeTrack& t : trk) {
            frames += t.T;
            cols += t.nw;
        }
        if (frames < 3 * cols) {
            if (ring) plan_stripe_ring(trk, bins, nheight, g);
            return;
        }
    }
    int kvmax = 0, amax = 0;
    bool dword = true;
    for (const StripeTrack& t : trk) {
        if ((uint64_t)t.T * bins >= (1ull << 30)) return;  // the kernel's 32-bit byte offsets
        kvmax = std::max(kvmax, t.vt->max_taps);
        amax = std::max(amax, t.ht->st_maxna);
        dword = dword && t.nw % 4 == 0 && t.rgb_off % 4 == 0;
    }
    const int slots = amax <= 8 ? 8 : amax <= 12 ? 12 : amax <= 16 ? 16 : 0;
    // 7 taps (no padded tap for the upsampling rows' 6-7) where an instance has the step table
    const int kv = kvmax <= 7 && slots <= 12 ? 7 : kvmax <= 8 ? 8 : kvmax <= 12 ? 12 : kvmax <= 16 ? 16 : 0;
    if (!kv || !slots) return;
    constexpr int kWaveRows = 64;  // render_stripe.hip: lane = row, a wave's rows stage their own tile
    const uint32_t strip = g.st_strip;
    int tile = 1, nbmax = 0, hdr = 1;
    for (const StripeTrack& t : trk) {
        const int top = (int)t.H - (int)bins;
        for (uint32_t R0 = 0; R0 < nheight; R0 += kWaveRows) {
            const uint32_t rlo = std::max(R0, t.oz), rhi = std::min(R0 + kWaveRows, nheight);
            if (rlo >= rhi) continue;
            const int ya = t.vt->h_left[rlo], nt = t.vt->h_left[rhi - 1] + kv - ya;
            tile = std::max(tile, nt);
            nbmax = std::max(nbmax, std::min(ya + nt, (int)t.H) - std::max(ya, top));
        }
        for (uint32_t c0 = 0; c0 < t.nw; c0 += strip) {
            const uint32_t c1 = std::min(c0 + strip, t.nw);
            const int s_lo = t.ht->h_left[c0] >> 3;
            const int s_hi = (t.ht->h_left[c1 - 1] + t.ht->h_count[c1 - 1] - 1) >> 3;
            hdr = std::max(hdr, s_hi - s_lo + 1);
        }
    }
    const int wts = hdr * 8 * (kv > 8 ? 16 : slots);
    // staged values per lane and chunk: fc x (bins per frame) <= 64 x npf; 8 waves per block
    // (the strip's step table staged once for 512 rows) where two such blocks fit a CU's LDS,
    // else 4
    int fc = 16, npf = 8, waves = nheight > 256 ? 8 : 4;
    if (fc * nbmax > 64 * npf) npf = 16;
    auto lds = [&]() { return render_stripe_lds_bytes(fc, tile, hdr, wts, waves); };
    if (fc * nbmax > 64 * npf || lds() > (waves == 8 ? 81920 : 54613)) fc = 8;
    if (waves == 8 && lds() > 81920) waves = 4;
    if (fc * nbmax > 64 * npf || lds() > 163840) return;
    // the kept element places (render_stripe.hip pk): a chunk's row offsets and the tile's float
    // indices below 2^16
    if (fc * (int)bins >= 65536 || tile * (fc + 4) >= 65536) return;
    // the instances compiled (render_stripe.hip launch_render_stripe)
    if (kv > 8) npf = 16;
    const int slots_run = kv > 8 ? 16 : slots;
    // accumulators: the exact count where an instance has it (9, 10 on the 12-wide table)
    const int acc_run = kv > 8 ? 16 : (slots == 12 && amax <= 10) ? std::max(9, amax) : slots;
    if (fc == 8) npf = 16;
    g.stripe = true;
    g.st_kv = kv;
    g.st_slots = slots_run;
    g.st_acc = acc_run;
    g.st_fc = fc;
    g.st_npf = npf;
    g.st_waves = waves;
    g.st_tile = tile;
    g.st_hdr = hdr;
    g.st_wts = wts;
    g.st_dword = dword;
}

int plan_fused_group(const float* d_spec, const uint64_t* row0, size_t bins, size_t n,
                     const float* up_ratio, const uint32_t* nwidth, uint32_t nheight,
                     const uint64_t* rgb_off, std::vector<RenderDesc>& desc, FusedGroup& g, bool wide,
                     int stripe) {
    g.spec = d_spec;
    g.bins = (uint32_t)bins;
    g.desc0 = desc.size();
    std::vector<std::pair<const DevTaps*, uint32_t>> vts;  // (vertical taps, oz)
    std::vector<StripeTrack> strk;
    for (size_t i = 0; i < n; ++i) {
        const float hf = roundf((float)bins * up_ratio[i]);  // display.rs:46
        const uint32_t H = hf > 0.f ? (uint32_t)hf : 0u;
        if (H < bins) return set_error(THESIA_ERR_INVALID_ARG, "up_ratio < 1 (display.rs:47 underflows)");
        const uint32_t T = (uint32_t)(row0[i + 1] - row0[i]);
        if (T == 0 || nwidth[i] == 0) continue;
        const DevTaps *vt = nullptr, *ht = nullptr;
        int rc = dev_taps(H, nheight, &vt);
        if (!rc) rc = stripe ? dev_taps_stepped(T, nwidth[i], 0, &ht) : dev_taps(T, nwidth[i], &ht);
        if (rc) return rc;
        RenderDesc r{};
        r.spec_off = row0[i] * bins;
        r.tmp_off = g.tmp_tot;
        r.ts = (T + 15) & ~15u;  // 64-byte aligned intermediate rows
        r.rgb_off = rgb_off[i];
        r.T = T;
        r.H = H;
        r.nw = nwidth[i];
        r.vl = vt->left.as<int32_t>(); r.vc = vt->count.as<int32_t>();
        r.vo = vt->offset.as<int32_t>(); r.vw = vt->weights.as<float>();
        r.hl = ht->left.as<int32_t>(); r.hc = ht->count.as<int32_t>();
        r.ho = ht->offset.as<int32_t>(); r.hw = ht->weights.as<float>();
        // oz: output rows whose taps end at or above the band's top row H - bins
        const int32_t top = (int32_t)H - (int32_t)bins;
        uint32_t oz = 0;
        while (oz < nheight && vt->h_left[oz] + vt->h_count[oz] <= top) ++oz;
        r.oz = oz;
        if (stripe) strk.push_back(StripeTrack{vt, ht, T, H, nwidth[i], oz, rgb_off[i]});
        if (std::find(vts.begin(), vts.end(), std::make_pair(vt, oz)) == vts.end()) vts.emplace_back(vt, oz);
        g.tmp_tot += (uint64_t)r.ts * nheight;
        g.cost += (uint64_t)T * bins + 2ull * r.ts * nheight + (3ull * nwidth[i] * nheight) / 4;
        g.h_taps = std::max(g.h_taps, ht->max_taps);
        g.h_span = std::max<int>(g.h_span, (int)((256.0 * T + nwidth[i] - 1) / nwidth[i]) + ht->max_taps + 8);
        g.T_max = std::max(g.T_max, T);
        g.H_max = std::max(g.H_max, H);
        g.nw_max = std::max(g.nw_max, nwidth[i]);
        desc.push_back(r);
    }
    g.ndesc = desc.size() - g.desc0;
    if (stripe) {
        plan_stripe(strk, (uint32_t)bins, nheight, g, stripe == 2, stripe == 3);
        if (g.stripe && g.st_hg) {  // ring mode: the plain tap tables (hl / hc / ho / hw), no step tables
            uint64_t cost = 0;
            for (size_t i = g.desc0; i < g.desc0 + g.ndesc; ++i) {
                desc[i].tmp_off = 0;
                cost += (uint64_t)desc[i].T * bins + (3ull * desc[i].nw * nheight) / 4;
            }
            g.tmp_tot = 0;
            g.cost = cost * 3;  // compute-bound like the slot mode (see below)
        } else if (g.stripe) {  // no intermediate: the group's workspace share and its cost change
            uint64_t cost = 0;
            for (size_t i = g.desc0; i < g.desc0 + g.ndesc; ++i) {
                const DevTaps* ht = nullptr;  // the step tables for the group's slot count
                const int rc = dev_taps_stepped(desc[i].T, desc[i].nw, g.st_slots, &ht);
                if (rc) return rc;
                const int k = g.st_slots / 4 - 2;
                desc[i].hst = ht->st_ca[k].as<int32_t>();
                desc[i].hsw = ht->st_w[k].as<float>();
                desc[i].tmp_off = 0;
                cost += (uint64_t)desc[i].T * bins + (3ull * desc[i].nw * nheight) / 4;
            }
            g.tmp_tot = 0;
            // the stream scheduling's cost is in HBM floats moved; the single-pass kernel is
            // compute-bound (VALU and latency: per track ~1.8x the time of a two-kernel group of the
            // same floats on C5), so its floats count 3 times (C5 display 2.52 / 2.51 -> 2.50 /
            // 2.48 ms vs 1x; 5x 2.50 / 2.50, profiles/r04_display/ab_experiments.txt;
            // THESIA_STRIPE_COST in the experiment build)
            uint64_t factor = 3;
#ifdef THESIA_EXPERIMENTS
            if (const char* e = std::getenv("THESIA_STRIPE_COST")) factor = (uint64_t)std::max(1, std::atoi(e));
#endif
            g.cost = cost * factor;
        }
    }
    // taps per row padded to kv (a multiple of 4, zero weights): the tile holds the band's
    // supports plus kv rows, the weight table band x kv floats
    int kv = 4;
    for (const auto& [vt, oz] : vts) kv = std::max(kv, (vt->max_taps + 3) & ~3);
    g.v_kv = kv;
    auto band_need = [&](uint32_t band, int* rows_out, int cap) {
        int rows = 1;
        for (const auto& [vt, oz] : vts)
            for (uint32_t ob = 0; ob < nheight; ob += band) {
                const uint32_t o0 = std::max(ob, oz), o1 = std::min(nheight, ob + band) - 1;
                if (o0 > o1) continue;
                rows = std::max(rows, vt->h_left[o1] - vt->h_left[o0] + kv);
            }
        *rows_out = rows;
        return rows <= cap && (int)band * kv <= 4096;
    };
    g.v_band = THESIA_VBAND;
    while (!band_need(g.v_band, &g.v_rows, THESIA_VROWS) && g.v_band > 1) g.v_band /= 2;
    g.v_fpl = 1;
    if (wide && g.H_max <= nheight) {
        // the wide vertical pass (4 frames per lane; its tile rows are 260 floats, so it holds
        // at most 40 of them, ~42 KiB) for groups that upsample vertically (H <= nheight: few
        // grey rows per band) where a band of at least 16 output rows fits. Measured per group
        // (C5, profiles/r03_s2_display): 44.1 kHz / n_fft 256 470 -> 381 us, 22.05 kHz / 256
        // 176 -> 159, 48 kHz / 512 310 -> 295; the downsampling groups ran slower (their bands
        // shrink to 16 rows of 40 tile rows). Display per C5 step 3.285 -> 3.232 ms (in process).
        uint32_t band = THESIA_VBAND;
        int rows = 1;
        while (!band_need(band, &rows, 40) && band > 1) band /= 2;
        if (band >= 16 && band_need(band, &rows, 40)) {
            g.v_fpl = 4;
            g.v_band = band;
            g.v_rows = rows;
        }
    }
    return THESIA_OK;
}

}  // namespace

int render_rgb_fused(size_t n_groups, const float* const* d_specs, const uint64_t* const* row0s,
                     const size_t* bins, const size_t* ns, const float* up_ratio,
                     const uint32_t* nwidth, uint32_t nheight, float max, float min, uint8_t* d_rgb,
                     const uint64_t* rgb_off, hipStream_t s, const float* d_grange) {
    if (nheight == 0) return THESIA_OK;
    int rc = 0;
    const uint8_t* cmap_ptr = colormap_device(&rc);
    if (rc) return rc;
    // the plan (descriptor table, bands, tap tables) depends only on the call's geometry: a
    // call repeating the previous one's geometry (every step of a render loop) reuses the
    // table already on the device and skips the planning and the upload
    std::vector<uint8_t> key;
    auto put = [&key](const void* p, size_t bytes) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        key.insert(key.end(), b, b + bytes);
    };
    size_t ntr = 0;
    const int rpath = render_path();
    put(&rpath, sizeof rpath);
    // groups in flight at once (THESIA_RENDER_STREAMS, 1..4; default 4)
    static const int nst = [] {
        const char* e = std::getenv("THESIA_RENDER_STREAMS");
        const int v = e ? std::atoi(e) : RunPool::kStreams;
        return v < 1 ? 1 : v > RunPool::kStreams ? RunPool::kStreams : v;
    }();
    put(&n_groups, sizeof n_groups);
    put(&nheight, sizeof nheight);
    put(&d_rgb, sizeof d_rgb);
    put(&d_grange, sizeof d_grange);
    for (size_t k = 0; k < n_groups; ++k) {
        put(&d_specs[k], sizeof(void*));
        put(&bins[k], sizeof(size_t));
        put(&ns[k], sizeof(size_t));
        if (ns[k]) put(row0s[k], (ns[k] + 1) * sizeof(uint64_t));
        ntr += ns[k];
    }
    put(up_ratio, ntr * sizeof(float));
    put(nwidth, ntr * sizeof(uint32_t));
    put(rgb_off, ntr * sizeof(uint64_t));
    struct Ws {
        DevBuf tmp, desc;
        std::vector<uint8_t> key;  // geometry of the table in `desc`
        std::vector<FusedGroup> groups;
    };
    static std::mutex ws_mu;
    static auto& ws_map = *new std::map<int, Ws>();  // leaked, see dev_taps
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(ws_mu);
    Ws& ws = ws_map[dev];
    if (ws.key != key) {
        ws.key.clear();
        {  // the tracks' RGB ranges are written concurrently: they must not overlap
            std::vector<std::pair<uint64_t, uint64_t>> rr;
            for (size_t i = 0; i < ntr; ++i)
                if (nwidth[i]) rr.emplace_back(rgb_off[i], rgb_off[i] + (uint64_t)nwidth[i] * nheight * 3);
            std::sort(rr.begin(), rr.end());
            for (size_t i = 1; i < rr.size(); ++i)
                if (rr[i].first < rr[i - 1].second)
                    return set_error(THESIA_ERR_INVALID_ARG, "render: two tracks' RGB ranges overlap");
        }
        std::vector<RenderDesc> desc;
        std::vector<FusedGroup> groups(n_groups);
        size_t t0 = 0;
        for (size_t k = 0; k < n_groups; ++k) {
            rc = plan_fused_group(d_specs[k], row0s[k], bins[k], ns[k], up_ratio + t0, nwidth + t0, nheight,
                                  rgb_off + t0, desc, groups[k], true,
                                  rpath == 0 ? 1 : rpath == 4 ? 2 : rpath == 5 ? 3 : 0);
            if (rc) return rc;
            t0 += ns[k];
        }
        // the groups run on nst streams, the largest first, each to the least loaded stream
        // (by the HBM floats it moves); a stream's groups share an intermediate region of the
        // largest of them, the regions side by side; ws.groups in launch order
        std::vector<size_t> ord(n_groups);
        for (size_t k = 0; k < n_groups; ++k) ord[k] = k;
        std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return groups[a].cost > groups[b].cost; });
        std::vector<uint64_t> load(nst, 0), slot(nst, 0), slot0(nst, 0);
        for (size_t k : ord) {
            const int i = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            groups[k].stream = i;
            load[i] += groups[k].cost;
            slot[i] = std::max(slot[i], groups[k].tmp_tot);
        }
        for (int i = 1; i < nst; ++i) slot0[i] = slot0[i - 1] + slot[i - 1];
        const uint64_t tmp_max = std::max<uint64_t>(1, slot0[nst - 1] + slot[nst - 1]);
        for (const FusedGroup& g : groups)
            for (size_t i = g.desc0; i < g.desc0 + g.ndesc; ++i) desc[i].tmp_off += slot0[g.stream];
        std::vector<FusedGroup> sorted;
        for (size_t k : ord) sorted.push_back(groups[k]);
        groups = std::move(sorted);
        auto grow = [](DevBuf& b, size_t bytes) {
            if (b.bytes >= bytes && b.p) return 0;
            b.release();
            return b.alloc(bytes + bytes / 8);
        };
        const void* tmp_before = ws.tmp.p;
        rc = grow(ws.tmp, tmp_max * sizeof(float));
        if (!rc) rc = grow(ws.desc, std::max<size_t>(desc.size(), 1) * sizeof(RenderDesc));
        if (rc) return rc;
        // the intermediate rows' padding [T, ts) is never written by the vertical pass: zero it
        // once per allocation, so every float a horizontal pass may stage is finite
        if (ws.tmp.p != tmp_before) THESIA_HIP(hipMemsetAsync(ws.tmp.p, 0, ws.tmp.bytes, s));
        if (!desc.empty()) {
            for (RenderDesc& r : desc) r.grange = d_grange;  // (part of the cache key)
            THESIA_HIP(copy_ordered(ws.desc.p, desc.data(), desc.size() * sizeof(RenderDesc), hipMemcpyHostToDevice));
        }
        ws.groups = std::move(groups);
        ws.key = std::move(key);
    }
    const std::vector<FusedGroup>& groups = ws.groups;
    // the horizontal pass: LDS-DMA row staging (display_kernels.hip resize_h_dma_kernel; the
    // register-staged pass of the three-stage path where a span does not fit)
    const bool h_dma = true;
    auto launch_group = [&](const FusedGroup& g, hipStream_t st) {
        for (size_t b = 0; b < g.ndesc; b += 65535) {  // grid.z limit
            const uint32_t nb = (uint32_t)std::min<size_t>(65535, g.ndesc - b);
            if (g.stripe) {
                StripeLaunch L{};
                L.spec = g.spec;
                L.bins = g.bins;
                L.max = max;
                L.min = min;
                L.nh = nheight;
                L.desc = ws.desc.as<RenderDesc>() + g.desc0 + b;
                L.n = nb;
                L.nw_max = g.nw_max;
                L.strip = g.st_strip;
                L.kv = g.st_kv;
                L.slots = g.st_slots;
                L.acc = g.st_acc;
                L.abl = 0;
#ifdef THESIA_EXPERIMENTS
                if (const char* e = std::getenv("THESIA_STRIPE_ABL")) L.abl = std::atoi(e);
#endif
                L.fc = g.st_fc;
                L.npf = g.st_npf;
                L.waves = g.st_waves;
                L.tile_cap = g.st_tile;
                L.hdr_cap = g.st_hdr;
                L.wts_cap = g.st_wts;
                L.dword_rgb = g.st_dword;
                L.ring = g.st_ring;
                L.hg = g.st_hg;
                L.cmap = cmap_ptr;
                L.rgb = d_rgb;
                if (launch_render_stripe(L, st)) return set_error(THESIA_ERR_DEVICE, "render stripe launch failed");
                continue;
            }
            if (launch_render_batch2(g.spec, g.bins, max, min, ws.desc.as<RenderDesc>() + g.desc0 + b, nb,
                                     g.T_max, g.H_max, g.nw_max, nheight, g.h_taps, g.h_span, g.v_band,
                                     g.v_rows, g.v_kv, ws.tmp.as<float>(), cmap_ptr, d_rgb, st, h_dma,
                                     g.v_fpl))
                return set_error(THESIA_ERR_DEVICE, "render batch launch failed");
        }
        return THESIA_OK;
    };
    const int k = (int)std::min<size_t>(nst, groups.size());
    if (k <= 1) {
        for (const FusedGroup& g : groups)
            if ((rc = launch_group(g, s))) return rc;
        return THESIA_OK;
    }
    std::lock_guard<std::mutex> plk(run_pool_mutex());
    RunPool* p = nullptr;
    if ((rc = run_pool(&p))) return rc;
    THESIA_HIP(p->fork_from(s, k));
    for (size_t i = 0; i < groups.size() && !rc; ++i) rc = launch_group(groups[i], p->st[groups[i].stream]);
    const int jrc = p->join_into(s, k);
    // stream-ordered: the images are complete for every later library call (copies included)
    return rc ? rc : jrc;
}

// InvRealFFT (realfft.rs:167-241) over device buffers: the length's tables come from a Plan
// of n_fft = length, built once per (device, length) and kept
int inv_real_fft_device(const float* d_in, size_t n_frames, size_t length, float* d_out, hipStream_t s) {
    if (length % 2) return set_error(THESIA_ERR_INVALID_ARG, "Length must be even (realfft.rs:171)");
    if (length < 2 || (length & (length - 1)))
        return set_error(THESIA_ERR_UNSUPPORTED, "Radix4 needs a power-of-two length/2 (the reference panics)");
    if (length > 4096) return set_error(THESIA_ERR_UNSUPPORTED, "length above 4096 (the engine's n_fft range)");
    static std::mutex mu;
    static auto& plans = *new std::map<std::pair<int, size_t>, Plan*>();  // leaked, see dev_taps
    int dev = 0;
    (void)hipGetDevice(&dev);
    Plan* p = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = plans.find({dev, length});
        if (it != plans.end()) {
            p = it->second;
        } else {
            thesia_plan_desc d{};
            d.sr = 48000;
            d.n_fft = length;
            d.win_length = length;
            d.hop_length = std::max<size_t>(1, length / 4);
            d.output = THESIA_OUT_COMPLEX;
            int rc = plan_create(d, &p);
            if (rc) return rc;
            plans[{dev, length}] = p;
        }
    }
    if (launch_irfftx(d_in, n_frames, (int)length, p->xpos.as<int>(), p->tw.as<float>(),
                      p->sincos.as<float>(), p->xw8, d_out, s))
        return set_error(THESIA_ERR_DEVICE, "irfft launch failed");
    return THESIA_OK;
}

int render_rgb_batch_device(const float* d_spec, const uint64_t* row0, size_t bins, size_t n,
                            const float* up_ratio, const uint32_t* nwidth, uint32_t nheight,
                            float max, float min, uint8_t* d_rgb, const uint64_t* rgb_off,
                            hipStream_t s) {
    if (n == 0 || nheight == 0) return THESIA_OK;
    // workspaces sized for the largest track; launches are stream-ordered, so reusing them
    // track after track is race-free
    size_t grey_max = 1, tmp_max = 1;
    std::vector<uint32_t> H(n);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t T = row0[i + 1] - row0[i];
        const float h = roundf((float)bins * up_ratio[i]);  // display.rs:46
        H[i] = h > 0.f ? (uint32_t)h : 0u;
        if (H[i] < bins) return set_error(THESIA_ERR_INVALID_ARG, "up_ratio < 1 (display.rs:47 underflows)");
        grey_max = std::max<size_t>(grey_max, (size_t)H[i] * T);
        tmp_max = std::max<size_t>(tmp_max, (size_t)T * nheight);
    }
    int crc = 0;
    const uint8_t* cmap_ptr = colormap_device(&crc);
    if (crc) return crc;
    if (render_path() == 0 || render_path() >= 3) {
        const size_t ns[1] = {n};
        const size_t bs[1] = {bins};
        return render_rgb_fused(1, &d_spec, &row0, bs, ns, up_ratio, nwidth, nheight, max, min, d_rgb,
                                rgb_off, s);
    }
    if (render_path() == 2) {
        // every track in one launch per stage (launch_render_batch); workspaces for all tracks
        std::vector<RenderDesc> desc;
        desc.reserve(n);
        uint64_t grey_tot = 0, tmp_tot = 0;
        uint32_t T_max = 0, H_max = 0, nw_max = 0;
        int h_taps = 0, h_span = 0;  // horizontal pass: max taps, max input span of 256 columns
        for (size_t i = 0; i < n; ++i) {
            const uint32_t T = (uint32_t)(row0[i + 1] - row0[i]);
            if (T == 0 || nwidth[i] == 0) continue;
            const DevTaps *vt = nullptr, *ht = nullptr;
            int rc = dev_taps(H[i], nheight, &vt);
            if (!rc) rc = dev_taps(T, nwidth[i], &ht);
            if (rc) return rc;
            RenderDesc r{};
            r.spec_off = row0[i] * bins;
            r.grey_off = grey_tot;
            r.tmp_off = tmp_tot;
            r.ts = T;
            r.rgb_off = rgb_off[i];
            r.T = T;
            r.H = H[i];
            r.nw = nwidth[i];
            r.vl = vt->left.as<int32_t>(); r.vc = vt->count.as<int32_t>();
            r.vo = vt->offset.as<int32_t>(); r.vw = vt->weights.as<float>();
            r.hl = ht->left.as<int32_t>(); r.hc = ht->count.as<int32_t>();
            r.ho = ht->offset.as<int32_t>(); r.hw = ht->weights.as<float>();
            grey_tot += (uint64_t)H[i] * T;
            tmp_tot += (uint64_t)T * nheight;
            h_taps = std::max(h_taps, ht->max_taps);
            h_span = std::max<int>(h_span, (int)((256.0 * T + nwidth[i] - 1) / nwidth[i]) + ht->max_taps + 8);
            T_max = std::max(T_max, T);
            H_max = std::max(H_max, H[i]);
            nw_max = std::max(nw_max, nwidth[i]);
            desc.push_back(r);
        }
        if (desc.empty()) return THESIA_OK;
        // grow-only workspaces per device, held for the call (hipMalloc / hipFree of a few
        // hundred MB per call measured as multi-ms stalls in the C5 step)
        struct Ws { DevBuf grey, tmp, desc; };
        static std::mutex ws_mu;
        static auto& ws_map = *new std::map<int, Ws>();  // leaked, see dev_taps
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> lk(ws_mu);
        Ws& ws = ws_map[dev];
        auto grow = [](DevBuf& b, size_t bytes) {
            if (b.bytes >= bytes && b.p) return 0;
            b.release();
            return b.alloc(bytes + bytes / 8);
        };
        int rc = grow(ws.grey, grey_tot * sizeof(float));
        if (!rc) rc = grow(ws.tmp, tmp_tot * sizeof(float));
        if (!rc) rc = grow(ws.desc, desc.size() * sizeof(RenderDesc));
        if (rc) return rc;
        THESIA_HIP(copy_on(ws.desc.p, desc.data(), desc.size() * sizeof(RenderDesc), hipMemcpyHostToDevice, s));
        DevBuf& grey = ws.grey;
        DevBuf& tmp = ws.tmp;
        DevBuf& ddesc = ws.desc;
        for (size_t b = 0; b < desc.size(); b += 65535) {  // grid.z limit
            const uint32_t nb = (uint32_t)std::min<size_t>(65535, desc.size() - b);
            if (launch_render_batch(d_spec, (uint32_t)bins, max, min, ddesc.as<RenderDesc>() + b, nb,
                                    T_max, H_max, nw_max, nheight, h_taps, h_span, grey.as<float>(), tmp.as<float>(),
                                    cmap_ptr, d_rgb, s))
                return set_error(THESIA_ERR_DEVICE, "render batch launch failed");
        }
        THESIA_HIP(hipStreamSynchronize(s));
        return THESIA_OK;
    }
    DevBuf grey, tmp;
    int rc = grey.alloc(grey_max * sizeof(float));
    if (!rc) rc = tmp.alloc(tmp_max * sizeof(float));
    if (rc) return rc;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t T = (uint32_t)(row0[i + 1] - row0[i]);
        if (T == 0 || nwidth[i] == 0) continue;
        const DevTaps *vt = nullptr, *ht = nullptr;
        rc = dev_taps(H[i], nheight, &vt);
        if (!rc) rc = dev_taps(T, nwidth[i], &ht);
        if (rc) return rc;
        if (launch_spec_to_grey(d_spec + row0[i] * bins, T, (uint32_t)bins, H[i], max, min,
                                grey.as<float>(), s) ||
            launch_resize_v(grey.as<float>(), T, H[i], nheight, vt->left.as<int32_t>(),
                            vt->count.as<int32_t>(), vt->offset.as<int32_t>(),
                            vt->weights.as<float>(), vt->max_taps, tmp.as<float>(), s) ||
            launch_resize_h_rgb(tmp.as<float>(), T, nheight, nwidth[i], ht->left.as<int32_t>(),
                                ht->count.as<int32_t>(), ht->offset.as<int32_t>(),
                                ht->weights.as<float>(), ht->max_taps, cmap_ptr,
                                d_rgb + rgb_off[i], s))
            return set_error(THESIA_ERR_DEVICE, "render launch failed");
    }
    THESIA_HIP(hipStreamSynchronize(s));
    return THESIA_OK;
}

int wav_to_image_device(const float* d_wav, uint64_t n, uint32_t nwidth, uint32_t nheight,
                        float amp_min, float amp_max, uint8_t* d_out, int* panicked,
                        hipStream_t s) {
    *panicked = 0;
    if (nwidth == 0 || nheight == 0) return THESIA_OK;
    const float spp = (float)n / (float)nwidth;  // display.rs:74
    DevBuf up, flag;
    uint64_t n_up = 0;
    int rc = flag.alloc(sizeof(int));
    if (rc) return rc;
    THESIA_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    if (spp < 1.0f) {  // display.rs:76-91 linear upsampling by factor
        const uint32_t factor = (uint32_t)ceilf(1.0f / spp);
        n_up = (uint64_t)factor * n;
        rc = up.alloc(n_up * sizeof(float));
        if (rc) return rc;
        if (launch_wav_upsample(d_wav, n, factor, up.as<float>(), s))
            return set_error(THESIA_ERR_DEVICE, "wav upsample launch failed");
    }
    if (launch_wav_image(d_wav, n, up.p ? up.as<float>() : nullptr, n_up, nwidth, nheight, spp,
                         amp_min, amp_max, d_out, flag.as<int>(), s))
        return set_error(THESIA_ERR_DEVICE, "wav image launch failed");
    THESIA_HIP(copy_on(panicked, flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    THESIA_HIP(hipStreamSynchronize(s));
    return THESIA_OK;
}

const int16_t* synth_lut_host() {
    static std::vector<int16_t> lut;
    static std::once_flag once;
    std::call_once(once, [] {
        lut.resize(4096);
        for (int i = 0; i < 4096; ++i)
            lut[i] = (int16_t)std::lround(32767.0 * std::sin(2.0 * 3.14159265358979323846 * i / 4096.0));
    });
    return lut.data();
}

}  // namespace thesia
