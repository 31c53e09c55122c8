// microbench_bucket.hip -- the bucketed first round's local sort in
// isolation: n synthetic key1-like keys already in bucket order (bucket =
// top 16 bits, rising with the position; low bits random), the window
// kernels of sa_bucket.h, then k_bucket_sort against a streaming
// copy of the same 12 bytes per suffix in and out.  Not part of libsa_hip.
//   build: make -C hpc_suffix_array_amd/csrc microbench_bucket
//   run:   hpc_suffix_array_amd/csrc/build/microbench_bucket [log2 n] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sa_bucket.h"

using namespace sa;

// per-phase clock64() spans of each workgroup's thread 0 (k_bucket_sort's
// Probe hook), summed into words[32 ..] as 7 u64
struct ClockProbe {
    uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0}, last = 0;
    __device__ __forceinline__ void mark(int k) {
        const uint64_t now = clock64();
        if (k >= 0) acc[k] += now - last;
        last = now;
    }
    __device__ __forceinline__ void flush(uint32_t* words) {
        if (threadIdx.x == 0)
            for (int k = 0; k < 7; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(words + 32) + k, acc[k]);
    }
};

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

// key = bucket << rb | random rbits bits, bucket = (i << 17) / n (rb = 28;
// fewer random bits make equal keys: unsorted groups for the segments)
// key1 = bucket << rb | random rbits bits, bucket = (i << 17) / n; as the
// second bucket pass writes them: bucket-relative items (key1 - (Dmin(b) <<
// rb)) << ib | idx with Dmin(b) = b (cmul = 1, bsh = 0); keys[] keeps key1
// for the copy baseline and the check
__global__ void k_keys(uint64_t* keys, uint32_t* vals, uint64_t* items, uint64_t n, uint32_t rb, uint32_t rbits,
                       uint32_t ib) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const uint64_t low = (z & ((1ull << rbits) - 1)) << (rb - rbits);
        keys[i] = ((i << 17) / n << rb) | low;
        vals[i] = (uint32_t)(z >> 32) & ((1u << ib) - 1u);
        items[i] = (low << ib) | vals[i];
    }
}

__global__ void k_tables(uint64_t n, uint32_t* bstart, uint32_t* bdmin) {
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b <= (1u << 17); b += gridDim.x * blockDim.x) {
        bstart[b] = b == (1u << 17) ? (uint32_t)n : (uint32_t)(((uint64_t)b * n + (1u << 17) - 1) >> 17);
        bdmin[b] = b;
    }
}

__global__ void k_copy12(const uint64_t* __restrict__ a, const uint32_t* __restrict__ av, uint64_t n,
                         uint64_t* __restrict__ b, uint32_t* __restrict__ bv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        b[i] = a[i];
        bv[i] = av[i];
    }
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? std::atoi(argv[1]) : 30;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    const uint32_t rbits = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 28;
    const uint64_t n = 1ull << lg;
    const uint32_t rb = 28, ib = lg;
    uint64_t *keys, *okeys;
    uint32_t *vals, *ovals, *ws, *words, *tab;
    uint64_t* items;
    CK(hipMalloc(&keys, n * 8));
    CK(hipMalloc(&items, n * 8));
    CK(hipMalloc(&tab, ((1u << 17) + 1) * 8));
    CK(hipMalloc(&okeys, n * 8));
    CK(hipMalloc(&vals, n * 4));
    CK(hipMalloc(&ovals, n * 4));
    const uint64_t nw = (n + kWinStride - 1) / kWinStride;
    CK(hipMalloc(&ws, (4 * nw + 3) * 4));
    uint32_t* retry;
    uint4* hdr;
    CK(hipMalloc(&retry, (nw + 1) * 4));
    CK(hipMalloc(&hdr, (nw + 1) * 16));
    CK(hipMalloc(&words, 256));
    uint32_t* list = ws + nw + 1;
    uint32_t* skew = list + nw;
    uint32_t* wbk = skew + nw;   // each window's first bucket
    uint32_t* bstart = tab;
    uint32_t* bdmin = tab + (1u << 17) + 1;
    hipLaunchKernelGGL(k_keys, dim3(8192), dim3(256), 0, 0, keys, vals, items, n, rb, rbits, ib);
    hipLaunchKernelGGL(k_tables, dim3(512), dim3(256), 0, 0, n, bstart, bdmin);
    const BucketRel br{wbk, bstart, bdmin, rb};
    BucketRel brf = br;   // fixed span: the keys fill rb bits of their bucket
    brf.bits1 = rb;
    // segments outputs (as round1_bucketed lays them out)
    uint32_t *rank, *member, *tmp;
    CK(hipMalloc(&rank, n * 4));
    CK(hipMalloc(&member, n / 8 + 64));
    CK(hipMalloc(&tmp, n * 12));
    uint32_t* cnt;
    CK(hipMalloc(&cnt, (2 * nw + 2) * 4));
    const SegOut so{rank, member, 0, tmp, tmp + n, tmp + 2 * n, cnt, cnt + nw + 1};
    CK(hipMemset(words, 0, 256));
    const uint64_t cmul = 1;   // bucket = D = key >> rb (17 bits), bsh = 0
    (void)cmul;
    hipLaunchKernelGGL(k_window_starts_tab, dim3((uint32_t)std::min<uint64_t>((nw + 256) / 256, 8192)), dim3(256), 0, 0,
                       (const uint32_t*)bstart, 1u << 17, n, nw, ws, wbk);
    hipLaunchKernelGGL(k_window_list, dim3((uint32_t)std::min<uint64_t>((nw + 255) / 256, 1024)), dim3(256), 0, 0,
                       (const uint32_t*)ws, nw, list, words);
    CK(hipDeviceSynchronize());
    uint32_t hw[16];
    CK(hipMemcpy(hw, words, 64, hipMemcpyDeviceToHost));
    std::printf("n=2^%d random key bits=%u windows=%u largest=%u\n", lg, rbits, hw[7], hw[5]);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        std::printf("%-40s %8.3f ms  %7.1f GB/s (24 B/suffix)\n", name, best, 24.0 * n / best / 1e6);
    };
    timeit("copy 12 B in + out (old item size)", [&] {
        hipLaunchKernelGGL(k_copy12, dim3(16384), dim3(256), 0, 0, keys, vals, n, okeys, ovals);
    });
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // the fixed-span 32-bit kernel over the one-bucket windows (k_window_split)
    auto fast = [&](const SegOut& o, bool probe) {
        CK(hipMemset(words + kRetryWord, 0, 12));
        hipLaunchKernelGGL(k_window_split, dim3(1024), dim3(256), 0, 0, (const uint32_t*)list, (const uint32_t*)ws, brf,
                           words, hdr, retry, 1u);
        if (probe)
            hipLaunchKernelGGL((k_bucket_sort<kBsBlock, kBsItems, ClockProbe>), dim3(kBsWpc * cus), dim3(kBsBlock), 0, 0,
                               (const uint64_t*)items, (const uint4*)hdr, rb, rb, ib, words, okeys, ovals, retry, o);
        else
            hipLaunchKernelGGL((k_bucket_sort<kBsBlock, kBsItems>), dim3(kBsWpc * cus), dim3(kBsBlock), 0, 0,
                               (const uint64_t*)items, (const uint4*)hdr, rb, rb, ib, words, okeys, ovals, retry, o);
    };
    timeit("bucket_sort (32-bit, prefetch)", [&] { fast(SegOut{}, false); });
    timeit("bucket_sort (32-bit, prefetch) + segments", [&] { fast(so, false); });
    for (uint32_t g : {512u, hw[7]}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "bucket_sort_wide grid %u", g);
        timeit(nm, [&] {
            hipLaunchKernelGGL((k_bucket_sort_wide<kBsBlock, kBsItems>), dim3(g), dim3(kBsBlock), 0, 0,
                               (const uint64_t*)items, br, (const uint32_t*)ws, (const uint32_t*)list,
                               words, ib, okeys, ovals, skew, SegOut{});
        });
        std::snprintf(nm, sizeof nm, "bucket_sort_wide + segments grid %u", g);
        timeit(nm, [&] {
            hipLaunchKernelGGL((k_bucket_sort_wide<kBsBlock, kBsItems>), dim3(g), dim3(kBsBlock), 0, 0,
                               (const uint64_t*)items, br, (const uint32_t*)ws, (const uint32_t*)list,
                               words, ib, okeys, ovals, skew, so);
        });
    }
    for (int fastk = 0; fastk < 2; ++fastk) {   // per-phase clock64 spans of thread 0, per window
        CK(hipMemset(words + 32, 0, 64));
        if (fastk)
            fast(so, true);
        else
            hipLaunchKernelGGL((k_bucket_sort_wide<kBsBlock, kBsItems, ClockProbe>), dim3(512), dim3(kBsBlock), 0, 0,
                               (const uint64_t*)items, br, (const uint32_t*)ws, (const uint32_t*)list, words, ib, okeys,
                               ovals, skew, so);
        CK(hipDeviceSynchronize());
        unsigned long long t[7];
        CK(hipMemcpy(t, words + 32, 56, hipMemcpyDeviceToHost));
        const char* nm[7] = {"load", "histogram", "scan", "scatter", "net-sort", "U+scan", "store+sync"};
        double tot = 0;
        for (int k = 0; k < 7; ++k) tot += (double)t[k];
        std::printf("%s phases:\n", fastk ? "bucket_sort (32-bit)" : "bucket_sort_wide");
        for (int k = 0; k < 7; ++k)
            std::printf("  phase %-12s %7.0f clk/window (%4.1f %%)\n", nm[k], (double)t[k] / hw[7], 100.0 * t[k] / tot);
    }
    CK(hipMemcpy(hw, words, 64, hipMemcpyDeviceToHost));
    std::printf("flags=%u skewed=%u heads=%u unsorted=%u groups=%u (accumulated over runs)\n", hw[6], hw[10], hw[0], hw[1], hw[2]);
    // check: output sorted within each window, keys monotone overall
    std::vector<uint64_t> h(std::min<uint64_t>(n, 1 << 24));
    fast(SegOut{}, false);
    CK(hipMemcpy(h.data(), okeys, h.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 1; i < h.size(); ++i) bad += h[i] < h[i - 1];
    std::printf("unsorted adjacent pairs in the first %zu: %zu\n", h.size(), bad);
    return 0;
}
