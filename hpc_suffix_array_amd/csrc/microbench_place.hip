// microbench_place.hip -- the re-rank's last step in isolation: 2^30 (idx,
// rank) pairs, grouped by idx >> B (bins of 2^B ranks, random order inside a
// bin), written to rank[idx].  Compares
//   xcd:  the workgroups of XCD x (w mod 8 = x) take bins x, x + 8, ... one
//         at a time, all of the XCD's workgroups on the same bin, so the
//         bin's 2^B x 4 bytes of rank[] sit in that XCD's L2 while its
//         random 4-byte writes arrive (merged there into whole lines);
//   any:  the same bins and slices with the bin of a workgroup not tied to
//         its XCD (bin = (w + t) mod bins);
//   copy: the pairs read and written back as a stream (the bytes' floor).
// Not part of libsa_hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                                    \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int kB = 256;

// pairs of bin b: [b << B, (b + 1) << B) of the pair array (a permutation of
// the bin's idx); a workgroup handles slice s of S of every bin it visits
template <bool XCD>
__global__ __launch_bounds__(kB) void k_place(const uint64_t* __restrict__ pairs, uint32_t B, uint32_t bins,
                                              uint32_t* __restrict__ rank) {
    const uint32_t w = blockIdx.x, G = gridDim.x;
    const uint32_t x = w % 8, per = G / 8, slice = w / 8;   // XCD x's per workgroups, this one's slice
    const uint64_t bsz = 1ull << B, ssz = bsz / per;
    for (uint32_t t = 0; t * 8 < bins; ++t) {
        const uint32_t b = XCD ? t * 8 + x : (t * 8 + x + slice * 8) % bins;
        if (b >= bins) break;
        const uint64_t p0 = ((uint64_t)b << B) + (uint64_t)slice * ssz;
        for (uint64_t i = threadIdx.x; i < ssz; i += kB * 4) {
            uint64_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = i + k * kB < ssz ? pairs[p0 + i + k * kB] : ~0ull;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (v[k] != ~0ull) rank[v[k] >> 32] = (uint32_t)v[k];
        }
    }
}

__global__ void k_copy(const uint64_t* __restrict__ in, uint64_t n, uint32_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)in[i];
}

int main() {
    const uint32_t LG = 30;
    const uint64_t n = 1ull << LG;
    std::vector<uint64_t> h(n);
    uint64_t st = 1;
    auto rnd = [&] {
        st += 0x9E3779B97F4A7C15ull;
        uint64_t z = st;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    uint64_t *d_pairs;
    uint32_t* d_rank;
    CK(hipMalloc(&d_pairs, n * 8));
    CK(hipMalloc(&d_rank, n * 4));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch) {
        std::vector<float> ts;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("%-44s median %.3f ms  min %.3f\n", name, ts[2], ts[0]);
    };
    timeit("copy 8 B in + 4 B out", [&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, d_pairs, n, d_rank); });
    for (uint32_t B : {18u, 19u, 20u, 22u}) {
        // bins of 2^B ranks, the idx of each bin in random order
        for (uint64_t i = 0; i < n; ++i) h[i] = (i << 32) | (uint32_t)i;
        const uint64_t bsz = 1ull << B;
        for (uint64_t b0 = 0; b0 < n; b0 += bsz)
            for (uint64_t i = bsz - 1; i > 0; --i) std::swap(h[b0 + i], h[b0 + rnd() % (i + 1)]);
        CK(hipMemcpy(d_pairs, h.data(), n * 8, hipMemcpyHostToDevice));
        const uint32_t bins = (uint32_t)(n >> B);
        for (int wpc : {2, 4, 8}) {
            const uint32_t G = (uint32_t)(cus * wpc);
            char nm[96];
            std::snprintf(nm, sizeof nm, "bins 2^%u (%u), %d WG/CU, per XCD", B, bins, wpc);
            timeit(nm, [&] { hipLaunchKernelGGL(k_place<true>, dim3(G), dim3(kB), 0, 0, d_pairs, B, bins, d_rank); });
            std::snprintf(nm, sizeof nm, "bins 2^%u (%u), %d WG/CU, any XCD", B, bins, wpc);
            timeit(nm, [&] { hipLaunchKernelGGL(k_place<false>, dim3(G), dim3(kB), 0, 0, d_pairs, B, bins, d_rank); });
        }
        // check
        std::vector<uint32_t> r(1 << 20);
        CK(hipMemcpy(r.data(), d_rank, r.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < r.size(); ++i) bad += r[i] != (uint32_t)i;
        std::printf("  check: %zu wrong of the first 2^20\n", bad);
    }
    return 0;
}
