// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access shapes of the incremental
// and merge kernels (MI355X_MICROARCH.md §HBM: only 16-B-per-lane streaming reads and stores are
// calibrated; "calibrate on a known byte count in your own access pattern").  Dev tool, not
// product code: tools/calib/run.sh builds it and runs one PMC pass per counter.
//
// Every kernel touches distinct 128-B lines of a 2 GiB buffer (far past the 256 MiB Infinity
// Cache; a line is touched by one kernel only, in a random order), L lanes per line, W bytes per
// lane at the line's start, so the kernel's algorithmic bytes are lines x L x W.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr size_t LINE = 128, NLINES = (size_t)16 << 20;   // 2 GiB

template <int L, int W>
__global__ void rd_lines(const uint8_t *buf, const uint32_t *perm, uint32_t n_groups, uint32_t *sink) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, g = t / L, k = t % L;
    if (g >= n_groups) return;
    const uint8_t *p = buf + (size_t)perm[g] * LINE + (size_t)k * W;
    uint32_t v;
    if constexpr (W == 16) { const uint4 x = *reinterpret_cast<const uint4 *>(p); v = x.x ^ x.y ^ x.z ^ x.w; }
    else if constexpr (W == 8) { const uint2 x = *reinterpret_cast<const uint2 *>(p); v = x.x ^ x.y; }
    else v = *reinterpret_cast<const uint32_t *>(p);
    if (v == 0x9E3779B9u) sink[0] = t;                       // (keeps the load; never true on zeros)
}

template <int L, int W>
__global__ void wr_lines(uint8_t *buf, const uint32_t *perm, uint32_t n_groups) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, g = t / L, k = t % L;
    if (g >= n_groups) return;
    uint8_t *p = buf + (size_t)perm[g] * LINE + (size_t)k * W;
    if constexpr (W == 16) *reinterpret_cast<uint4 *>(p) = make_uint4(t, t, t, t);
    else if constexpr (W == 8) *reinterpret_cast<uint2 *>(p) = make_uint2(t, t);
    else *reinterpret_cast<uint32_t *>(p) = t;
}

__global__ void rd_stream(const uint4 *buf, size_t n, uint32_t *sink) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint4 x = buf[t];
    if ((x.x ^ x.y ^ x.z ^ x.w) == 0x9E3779B9u) sink[0] = (uint32_t)t;
}

struct Case { const char *name; int L, W; bool write; };

int main() {
    uint8_t *buf; uint32_t *perm_d, *sink;
    CK(hipMalloc(&buf, NLINES * LINE));
    CK(hipMemset(buf, 0, NLINES * LINE));
    CK(hipMalloc(&sink, 64));
    std::vector<uint32_t> perm(NLINES);
    std::iota(perm.begin(), perm.end(), 0u);
    std::mt19937 rng(7);
    std::shuffle(perm.begin(), perm.end(), rng);
    CK(hipMalloc(&perm_d, NLINES * 4));
    CK(hipMemcpy(perm_d, perm.data(), NLINES * 4, hipMemcpyHostToDevice));
    // the stream reads the first 256 MiB twice over distinct halves; the line kernels each take
    // a disjoint 1M-line slice of the permutation (none overlaps the streamed range's reuse)
    const uint32_t G = 1u << 20;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timed = [&](const char *nm, size_t bytes, auto launch) -> int {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-22s algorithmic %12zu B  %.3f ms\n", nm, bytes, ms);
        return 0;
    };
    const size_t SN = ((size_t)512 << 20) / 16;                // 512 MiB streamed
    if (timed("rd_stream_16B", SN * 16, [&] { rd_stream<<<(unsigned)((SN + 255) / 256), 256>>>((const uint4 *)buf, SN, sink); })) return 1;
    uint32_t slice = 8;                                        // lines 0..8M-1 of perm may hold streamed lines: skip
#define RD(L_, W_) do { const uint32_t *pp = perm_d + (size_t)slice++ * G; \
        if (timed("rd_" #L_ "x" #W_ "B", (size_t)G * L_ * W_, [&] { rd_lines<L_, W_><<<(G * L_ + 255) / 256, 256>>>(buf, pp, G, sink); })) return 1; } while (0)
#define WR(L_, W_) do { const uint32_t *pp = perm_d + (size_t)slice++ * G; \
        if (timed("wr_" #L_ "x" #W_ "B", (size_t)G * L_ * W_, [&] { wr_lines<L_, W_><<<(G * L_ + 255) / 256, 256>>>(buf, pp, G); })) return 1; } while (0)
    RD(8, 16);   // a whole 128-B line
    RD(4, 16);   // 64 B
    RD(2, 16);   // 32 B (a clock / result / state row)
    RD(1, 16);   // 16 B (a register row)
    RD(1, 8);    // 8 B (a survivor slot's metadata)
    RD(1, 4);    // 4 B (a packed change key)
    WR(2, 16);   // 32 B rows
    WR(1, 4);    // 4 B
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
