// microbench_scatter.hip -- what a 4-byte rank scatter / gather over n text
// positions costs on one MI355X, the access the reference schedule's re-rank
// makes (rank[sa[p]] = R, manber_myers.c:116-124):
//   * fully random (every position of [0, n) once, in a random order);
//   * windowed: the same writes grouped by windows of 2^S positions (random
//     inside a window), read in window order, with the plain blockIdx order or
//     with each XCD walking its own run of windows;
//   * the multisplit that groups them: 8-byte (position, rank) items of one
//     tile split by position >> S into per-window cursors (LDS histogram, one
//     global atomic per window and tile).
// Not part of libsa_hip.
//   build: make -C hpc_suffix_array_amd/csrc microbench_scatter
//   run:   hpc_suffix_array_amd/csrc/build/microbench_scatter [log2 n] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

// bijection of [0, 2^lg): odd multiplies and xor-shifts
__device__ __forceinline__ uint32_t mix(uint32_t x, uint32_t lg) {
    const uint32_t mask = lg >= 32 ? 0xFFFFFFFFu : ((1u << lg) - 1u);
    x = (x * 0x9E3779B1u) & mask;
    x ^= x >> ((lg + 1) / 2);
    x = (x * 0x85EBCA6Bu) & mask;
    x ^= x >> (lg / 2 + 1);
    x = (x * 0xC2B2AE35u) & mask;
    x ^= x >> ((lg + 1) / 2);
    return x;
}

// perm[p] = window(p) | mix(low bits of p): random inside windows of 2^S
__global__ void k_perm(uint32_t* perm, uint64_t n, uint32_t S) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t lo = (uint32_t)p & ((S >= 32 ? 0u : (1u << S)) - 1u);
        perm[p] = (uint32_t)(p - lo) | mix(lo, S);
    }
}

constexpr int kB = 256;
constexpr int kI = 16;
constexpr int kT = kB * kI;

// out[perm[p]] = p over tiles of kT; xcd: tile order per XCD (8 runs)
template <bool XCD>
__global__ __launch_bounds__(kB) void k_scatter(const uint32_t* __restrict__ perm, uint64_t n,
                                                uint32_t* __restrict__ out) {
    uint64_t t = blockIdx.x;
    if (XCD) {
        const uint64_t per = gridDim.x / 8;
        t = (uint64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const uint64_t b = t * kT;
    uint32_t x[kI];
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        const uint64_t e = b + (uint64_t)j * kB + threadIdx.x;
        x[j] = e < n ? perm[e] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int j = 0; j < kI; ++j)
        if (x[j] != 0xFFFFFFFFu) out[x[j]] = (uint32_t)(b + j * kB + threadIdx.x);
}

template <bool XCD>
__global__ __launch_bounds__(kB) void k_gather(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ in,
                                               uint64_t n, uint32_t* __restrict__ out) {
    uint64_t t = blockIdx.x;
    if (XCD) {
        const uint64_t per = gridDim.x / 8;
        t = (uint64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const uint64_t b = t * kT;
    uint32_t x[kI];
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        const uint64_t e = b + (uint64_t)j * kB + threadIdx.x;
        x[j] = e < n ? perm[e] : 0xFFFFFFFFu;
    }
    uint32_t v[kI];
#pragma unroll
    for (int j = 0; j < kI; ++j) v[j] = x[j] != 0xFFFFFFFFu ? in[x[j]] : 0u;
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        const uint64_t e = b + (uint64_t)j * kB + threadIdx.x;
        if (e < n) out[e] = v[j];
    }
}

// scattered 8-byte (position, value) items -> windows of 2^S positions:
// LDS histogram, exclusive scan, one global atomic per (tile, window),
// items staged in LDS in window order and written out from there.
template <int BINS>
__global__ __launch_bounds__(kB) void k_split(const uint32_t* __restrict__ perm, uint64_t n, uint32_t S,
                                              uint32_t* __restrict__ cursor, uint64_t* __restrict__ out) {
    __shared__ uint32_t s_cnt[BINS];
    __shared__ uint32_t s_base[BINS];
    __shared__ uint64_t s_it[kT];
    __shared__ uint32_t s_tmp[kB / 64];
    for (int i = threadIdx.x; i < BINS; i += kB) s_cnt[i] = 0;
    __syncthreads();
    const uint64_t b = (uint64_t)blockIdx.x * kT;
    uint32_t x[kI], r[kI];
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        const uint64_t e = b + (uint64_t)j * kB + threadIdx.x;
        x[j] = e < n ? perm[e] : 0xFFFFFFFFu;
        r[j] = x[j] != 0xFFFFFFFFu ? atomicAdd(&s_cnt[x[j] >> S], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the bins (BINS / kB per thread)
    constexpr int PER = (BINS + kB - 1) / kB;
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x * PER + k;
        c[k] = i < BINS ? s_cnt[i] : 0u;
        sum += c[k];
    }
    uint32_t inc = sum;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) s_tmp[wv] = inc;
    __syncthreads();
    uint32_t off = inc - sum;
    for (int w = 0; w < wv; ++w) off += s_tmp[w];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x * PER + k;
        if (i < BINS) {
            s_base[i] = off;
            // global destination minus the local base: one atomic per bin
            const uint32_t g = c[k] ? atomicAdd(&cursor[i], c[k]) : 0u;
            s_cnt[i] = g - off;
        }
        off += c[k];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kI; ++j)
        if (x[j] != 0xFFFFFFFFu) s_it[s_base[x[j] >> S] + r[j]] = ((uint64_t)(b + j * kB + threadIdx.x) << 32) | x[j];
    __syncthreads();
    const uint32_t m = n - b < (uint64_t)kT ? (uint32_t)(n - b) : (uint32_t)kT;
    for (uint32_t i = threadIdx.x; i < m; i += kB) {
        const uint64_t it = s_it[i];
        const uint32_t bin = (uint32_t)it >> S;
        out[(uint32_t)(s_cnt[bin] + i)] = it;
    }
}

__global__ void k_cursor_init(uint32_t* cursor, uint32_t bins, uint32_t S) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < bins) cursor[i] = i << S;
}

// out[pos] = value for windowed 8-byte items (read in order)
template <bool XCD>
__global__ __launch_bounds__(kB) void k_place(const uint64_t* __restrict__ it, uint64_t n, uint32_t* __restrict__ out) {
    uint64_t t = blockIdx.x;
    if (XCD) {
        const uint64_t per = gridDim.x / 8;
        t = (uint64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const uint64_t b = t * kT;
    uint64_t v[kI];
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        const uint64_t e = b + (uint64_t)j * kB + threadIdx.x;
        v[j] = e < n ? it[e] : ~0ull;
    }
#pragma unroll
    for (int j = 0; j < kI; ++j)
        if (v[j] != ~0ull) out[(uint32_t)v[j]] = (uint32_t)(v[j] >> 32);
}

__global__ void k_check_inverse(const uint32_t* perm, const uint32_t* out, uint64_t n, unsigned long long* bad) {
    unsigned long long c = 0;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x)
        c += out[perm[p]] != (uint32_t)p;
    if (c) atomicAdd(bad, c);
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
    }
    template <class F>
    double ms(F f, int reps) {
        f();
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
    const uint32_t tiles = (uint32_t)(n / kT);
    uint32_t *perm, *out, *in, *cursor;
    uint64_t* items;
    unsigned long long* bad;
    CK(hipMalloc(&perm, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&items, n * 8));
    CK(hipMalloc(&cursor, 65536 * 4));
    CK(hipMalloc(&bad, 8));
    CK(hipMemset(in, 1, n * 4));
    Timer T;
    auto report = [&](const char* name, uint32_t S, double ms, double bytes) {
        std::printf("{\"kernel\": \"%s\", \"n\": %llu, \"window_log2\": %u, \"ms\": %.4f, \"GBps\": %.1f}\n", name,
                    (unsigned long long)n, S, ms, bytes / ms / 1e6);
        std::fflush(stdout);
    };
    auto check = [&](const char* name) {
        CK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(k_check_inverse, dim3(4096), dim3(256), 0, 0, perm, out, n, bad);
        unsigned long long h = 0;
        CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
        std::printf("{\"verify\": \"%s\", \"mismatches\": %llu}\n", name, h);
        std::fflush(stdout);
    };
    for (uint32_t S : {(uint32_t)lg, 24u, 22u, 20u, 19u, 18u, 16u}) {
        if (S > (uint32_t)lg) continue;
        hipLaunchKernelGGL(k_perm, dim3(4096), dim3(256), 0, 0, perm, n, S);
        CK(hipDeviceSynchronize());
        report("scatter", S, T.ms([&] { hipLaunchKernelGGL(k_scatter<false>, dim3(tiles), dim3(kB), 0, 0, perm, n, out); }, reps), 8.0 * n);
        check("scatter");
        report("scatter_xcd", S, T.ms([&] { hipLaunchKernelGGL(k_scatter<true>, dim3(tiles), dim3(kB), 0, 0, perm, n, out); }, reps), 8.0 * n);
        check("scatter_xcd");
        report("gather", S, T.ms([&] { hipLaunchKernelGGL(k_gather<false>, dim3(tiles), dim3(kB), 0, 0, perm, in, n, out); }, reps), 12.0 * n);
        report("gather_xcd", S, T.ms([&] { hipLaunchKernelGGL(k_gather<true>, dim3(tiles), dim3(kB), 0, 0, perm, in, n, out); }, reps), 12.0 * n);
    }
    // the split of fully random positions into windows, then the placement
    hipLaunchKernelGGL(k_perm, dim3(4096), dim3(256), 0, 0, perm, n, (uint32_t)lg);
    CK(hipDeviceSynchronize());
    auto split = [&](auto kern, uint32_t bins) {
        const uint32_t S = lg - __builtin_ctz(bins);
        report("split", S, T.ms([&] {
            hipLaunchKernelGGL(k_cursor_init, dim3((bins + 255) / 256), dim3(256), 0, 0, cursor, bins, S);
            hipLaunchKernelGGL(kern, dim3(tiles), dim3(kB), 0, 0, perm, n, S, cursor, items);
        }, reps), 12.0 * n);
        report("place", S, T.ms([&] { hipLaunchKernelGGL(k_place<false>, dim3(tiles), dim3(kB), 0, 0, items, n, out); }, reps), 12.0 * n);
        check("place");
        report("place_xcd", S, T.ms([&] { hipLaunchKernelGGL(k_place<true>, dim3(tiles), dim3(kB), 0, 0, items, n, out); }, reps), 12.0 * n);
        check("place_xcd");
    };
    split(k_split<256>, 256);
    split(k_split<1024>, 1024);
    split(k_split<2048>, 2048);
    split(k_split<4096>, 4096);
    return 0;
}
