// microbench.hip -- times one LSD radix pass (64-bit key + 32-bit index, the
// pass the round-1 sort repeats) in isolation on n random keys, against the
// streaming copy of the same 24 bytes per suffix, and variants of the
// single-pass kernel with one phase removed (look-back / ranking / LDS
// staging) to see where its time goes.  Not part of libsa_hip.
//   build: make -C hpc_suffix_array_amd/csrc microbench
//   run:   hpc_suffix_array_amd/csrc/build/microbench [log2 n] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sa_onesweep.h"

using namespace sa;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ void k_rand_keys(uint64_t* keys, uint32_t* vals, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        keys[i] = z ^ (z >> 31);
        vals[i] = (uint32_t)i;
    }
}

// same striped tile layout as k_onesweep, identity destination
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_copy_striped(const uint64_t* __restrict__ ik, const uint32_t* __restrict__ iv,
                                                        uint64_t n, uint64_t* __restrict__ ok, uint32_t* __restrict__ ov) {
    constexpr int TILE = BLOCK * ITEMS;
    const uint64_t tb = (uint64_t)blockIdx.x * TILE;
    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t e = tb + (uint64_t)j * BLOCK + threadIdx.x;
        k[j] = e < n ? ik[e] : 0;
        v[j] = e < n ? iv[e] : 0;
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t e = tb + (uint64_t)j * BLOCK + threadIdx.x;
        if (e < n) {
            ok[e] = k[j];
            ov[e] = v[j];
        }
    }
}

__global__ void k_mismatch(const uint64_t* a, const uint32_t* av, const uint64_t* b, const uint32_t* bv, uint64_t n,
                           unsigned long long* out) {
    unsigned long long c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += (a[i] != b[i]) | (av[i] != bv[i]);
    if (c) atomicAdd(out, c);
}

// 16 bytes per lane per access
__global__ __launch_bounds__(256) void k_copy_vec(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t m) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) b[i] = a[i];
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
    }
    template <class F>
    double ms(F f, int reps) {
        f();   // warm
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            f();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float x;
            CK(hipEventElapsedTime(&x, a, b));
            t.push_back(x);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    }
};

int main(int argc, char** argv) {
    const int lg = argc > 1 ? std::atoi(argv[1]) : 30;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const uint64_t n = 1ull << lg;
    uint64_t *k0, *k1, *states;
    uint32_t *v0, *v1, *ws, *err;
    CK(hipMalloc(&k0, n * 8));
    CK(hipMalloc(&k1, n * 8));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&v1, n * 4));
    const uint64_t tiles_max = (n + 1023) / 1024 + 1;
    CK(hipMalloc(&states, tiles_max * kRadix * 8));
    CK(hipMemset(states, 0, tiles_max * kRadix * 8));
    CK(hipMalloc(&ws, 1 << 22));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    hipLaunchKernelGGL(k_rand_keys, dim3(4096), dim3(256), 0, 0, k0, v0, n, 12345ull);
    uint32_t* ghist = ws;
    uint32_t* base = ws + 4096;
    uint32_t* tick = ws + 8192;
    uint32_t* hist = ws + 16384;   // reduce-then-scan: 256 x up to 2048 chunks
    uint32_t* totals = ws + 16384 + 524288;
    CK(hipMemset(ghist, 0, 4096 * 4));
    SrcKeys src{k0, v0};
    hipLaunchKernelGGL(k_global_hist<SrcKeys>, dim3(2048), dim3(kBlock), 0, 0, src, n, 1u, ghist);
    hipLaunchKernelGGL(k_digit_base, dim3(1), dim3(kBlock), 0, 0, (const uint32_t*)ghist, base);
    CK(hipDeviceSynchronize());
    Timer T;
    const double bytes = 24.0 * n;
    auto report = [&](const char* name, double ms) {
        std::printf("{\"kernel\": \"%s\", \"n\": %llu, \"ms\": %.4f, \"GBps\": %.1f}\n", name, (unsigned long long)n, ms,
                    bytes / ms / 1e6);
        std::fflush(stdout);
    };
    report("copy_vec_24B", T.ms([&] {
        hipLaunchKernelGGL(k_copy_vec, dim3(8192), dim3(256), 0, 0, (const uint4*)k0, (uint4*)k1, n / 2);
        hipLaunchKernelGGL(k_copy_vec, dim3(8192), dim3(256), 0, 0, (const uint4*)v0, (uint4*)v1, n / 4);
    }, reps));
    report("copy_striped_256x16", T.ms([&] {
        hipLaunchKernelGGL((k_copy_striped<256, 16>), dim3((n + 4095) / 4096), dim3(256), 0, 0, k0, v0, n, k1, v1);
    }, reps));
    uint32_t epoch = 0;
    auto onesweep = [&](auto kern, int block, int tile) {
        return [&, kern, block, tile] {
            CK(hipMemsetAsync(tick, 0, 4));
            ++epoch;
            hipLaunchKernelGGL(kern, dim3((uint32_t)((n + tile - 1) / tile)), dim3(block), 0, 0, src, n, 0u, 8u,
                               (const uint32_t*)base, states, tick, epoch, k1, v1, err);
        };
    };
    report("onesweep_1024x4", T.ms(onesweep(k_onesweep<SrcKeys, 1024, 4>, 1024, 4096), reps));
    // the onesweep output is the reference the chunked variants are compared with
    uint64_t* kref;
    uint32_t* vref;
    unsigned long long* mism;
    CK(hipMalloc(&kref, n * 8));
    CK(hipMalloc(&vref, n * 4));
    CK(hipMalloc(&mism, 8));
    CK(hipMemcpy(kref, k1, n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(vref, v1, n * 4, hipMemcpyDeviceToDevice));
    auto verify = [&](const char* name) {
        CK(hipMemset(mism, 0, 8));
        hipLaunchKernelGGL(k_mismatch, dim3(4096), dim3(256), 0, 0, (const uint64_t*)k1, (const uint32_t*)v1,
                           (const uint64_t*)kref, (const uint32_t*)vref, n, mism);
        unsigned long long h = 0;
        CK(hipMemcpy(&h, mism, 8, hipMemcpyDeviceToHost));
        std::printf("{\"verify\": \"%s\", \"mismatches\": %llu}\n", name, h);
        std::fflush(stdout);
        CK(hipMemset(k1, 0, n * 8));
        CK(hipMemset(v1, 0, n * 4));
    };
    for (uint32_t want : {512u, 1024u, 2048u}) {
        Chunking ch;
        ch.n = n;
        const uint64_t tiles = (n + kTile - 1) / kTile;
        const uint64_t tpc = (tiles + want - 1) / want;
        ch.tiles_per_chunk = (uint32_t)tpc;
        ch.chunks = (uint32_t)((tiles + tpc - 1) / tpc);
        char name[64];
        std::snprintf(name, sizeof name, "reduce_scan_hist_c%u", ch.chunks);
        report(name, T.ms([&] {
            hipLaunchKernelGGL(k_hist<SrcKeys>, dim3(ch.chunks), dim3(kBlock), 0, 0, src, ch, 0u, 255u, hist);
        }, reps));
        hipLaunchKernelGGL(k_scan_rows, dim3(kRadix), dim3(kBlock), 0, 0, hist, ch.chunks, totals);
        CK(hipDeviceSynchronize());
        std::snprintf(name, sizeof name, "reduce_scan_scatter_c%u", ch.chunks);
        report(name, T.ms([&] {
            hipLaunchKernelGGL(k_scatter<SrcKeys>, dim3(ch.chunks), dim3(kBlock), 0, 0, src, ch, 0u, 8u,
                               (const uint32_t*)hist, (const uint32_t*)totals, k1, v1);
        }, reps));
        verify(name);
        std::snprintf(name, sizeof name, "scatter_pipe_1024x4_c%u", ch.chunks);
        report(name, T.ms([&] {
            hipLaunchKernelGGL((k_scatter_pipe<SrcKeys, 1024, 4>), dim3(ch.chunks), dim3(1024), 0, 0, src, ch, 0u, 8u,
                               (const uint32_t*)hist, (const uint32_t*)totals, k1, v1);
        }, reps));
        verify(name);
        std::snprintf(name, sizeof name, "scatter_pipe_512x8_c%u", ch.chunks);
        report(name, T.ms([&] {
            hipLaunchKernelGGL((k_scatter_pipe<SrcKeys, 512, 8>), dim3(ch.chunks), dim3(512), 0, 0, src, ch, 0u, 8u,
                               (const uint32_t*)hist, (const uint32_t*)totals, k1, v1);
        }, reps));
        verify(name);
    }
    uint32_t herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    std::printf("{\"lookback_errors\": %u}\n", herr);
    return 0;
}
