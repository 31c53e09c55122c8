// microbench_radix.hip -- design space of one single-pass radix scatter
// (64-bit key + 32-bit value, the bucket passes of the bucketed first round)
// on n random keys: tile shape, ranking (stable ballots vs unstable LDS
// atomics), look-back width, against a streaming copy of the same bytes.
// Not part of libsa_hip.
//   build: make -C hpc_suffix_array_amd/csrc microbench_radix
//   run:   hpc_suffix_array_amd/csrc/build/microbench_radix [log2 n] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sa_split.h"

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

__global__ void k_copy12(const uint64_t* __restrict__ a, const uint32_t* __restrict__ av, uint64_t n,
                         uint64_t* __restrict__ b, uint32_t* __restrict__ bv) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        b[i] = a[i];
        bv[i] = av[i];
    }
}

// checks: output digit-sorted; multiset preserved via sum of keys^vals
__global__ void k_check(const uint64_t* k, const uint32_t* v, uint64_t n, uint32_t shift, uint32_t mask,
                        unsigned long long* out) {
    unsigned long long bad = 0, sum = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (i + 1 < n && ((k[i] >> shift) & mask) > ((k[i + 1] >> shift) & mask)) ++bad;
        sum += k[i] * 0x9E3779B97F4A7C15ull + v[i];
    }
    atomicAdd(out, bad);
    atomicAdd(out + 1, sum);
}

// RANK 0: stable (per-wave match-any from ballots, as k_onesweep)
// RANK 1: unstable (one LDS atomic per item returns its rank; the counts are
//         known right after it, so the tile's aggregate is published before
//         any staging work)
// LOOK:   predecessor states read per look-back step (0: offsets faked)
template <int BLOCK, int ITEMS, int RBITS, int RANK, int LOOK>
__global__ __launch_bounds__(BLOCK) void k_split(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                 uint64_t n, uint32_t shift, const uint32_t* __restrict__ digit_base,
                                                 uint64_t* __restrict__ states, uint32_t* __restrict__ ticket,
                                                 uint32_t epoch, uint64_t* __restrict__ out_keys,
                                                 uint32_t* __restrict__ out_vals, uint32_t* __restrict__ err) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int RADIX = 1 << RBITS;
    constexpr int RWAVES = RADIX / kWave;
    static_assert(BLOCK >= RADIX, "one thread per digit");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_vals[TILE];
    __shared__ uint16_t s_wcnt[RANK == 0 ? WAVES : 1][RADIX];
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile;

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t mask = RADIX - 1;
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    if constexpr (RANK == 0) {
        for (int i = threadIdx.x; i < WAVES * RADIX; i += BLOCK) (&s_wcnt[0][0])[i] = 0;
    } else {
        if (threadIdx.x < RADIX) s_cnt[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint64_t t = s_tile;
    const uint64_t tb = t * TILE;
    const uint32_t valid = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);
    uint64_t k[ITEMS];
    uint32_t v[ITEMS], d[ITEMS], r[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t le = wave * WTILE + j * kWave + lane;
        const bool ok = le < valid;
        k[j] = ok ? keys[tb + le] : 0ull;
        v[j] = ok ? vals[tb + le] : 0u;
        d[j] = ok ? (uint32_t)(k[j] >> shift) & mask : RADIX;
    }
    const uint32_t dg = threadIdx.x;
    uint32_t tile_cnt = 0;
    if constexpr (RANK == 0) {
        uint16_t* wc = s_wcnt[wave];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const bool ok = d[j] < (uint32_t)RADIX;
            uint64_t peers = __ballot(ok);
#pragma unroll
            for (int b = 0; b < RBITS; ++b) {
                const bool bit = (d[j] >> b) & 1u;
                const uint64_t bal = __ballot(bit);
                peers &= bit ? bal : ~bal;
            }
            uint32_t cnt = 0;
            if (ok) cnt = wc[d[j]];
            const uint32_t below = (uint32_t)__popcll(peers & lanemask_lt());
            r[j] = cnt + below;
            if (ok && below == 0) wc[d[j]] = (uint16_t)(cnt + (uint32_t)__popcll(peers));
        }
        __syncthreads();
        if (dg < (uint32_t)RADIX) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                const uint32_t x = s_wcnt[w][dg];
                s_wcnt[w][dg] = (uint16_t)tile_cnt;
                tile_cnt += x;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) r[j] = d[j] < (uint32_t)RADIX ? atomicAdd(&s_cnt[d[j]], 1u) : 0u;
        __syncthreads();
        if (dg < (uint32_t)RADIX) tile_cnt = s_cnt[dg];
    }
    const uint64_t tag = (uint64_t)(epoch & kEpochMask) << 48;
    if (dg < (uint32_t)RADIX && LOOK > 0) st_store(&states[t * RADIX + dg], (t == 0 ? kStPrefix : kStAgg) | tag | tile_cnt);
    {
        const uint32_t x = (dg < (uint32_t)RADIX) ? tile_cnt : 0u;
        const uint32_t inc = wave_inclusive_sum(x);
        if (lane == kWave - 1 && wave < (uint32_t)RWAVES) s_tmp[wave] = inc;
        __syncthreads();
        uint32_t off = 0;
#pragma unroll
        for (int w = 0; w < RWAVES; ++w) off += (w < (int)wave) ? s_tmp[w] : 0u;
        if (dg < (uint32_t)RADIX) s_start[dg] = (uint16_t)(off + inc - x);
    }
    if (dg < (uint32_t)RADIX) {
        uint64_t excl = 0;
        if constexpr (LOOK == 0) {
            excl = t * (uint64_t)(TILE / RADIX);
        } else if (t > 0) {
            int64_t tp = (int64_t)t - 1;
            uint32_t spins = 0;
            const uint32_t ep_now = epoch & kEpochMask;
            while (tp >= 0) {
                uint64_t sv[LOOK];
#pragma unroll
                for (int i = 0; i < LOOK; ++i)
                    sv[i] = (tp - i >= 0) ? st_load(&states[(uint64_t)(tp - i) * RADIX + dg]) : 0ull;
                int used = 0;
                bool done = false;
#pragma unroll
                for (int i = 0; i < LOOK; ++i) {
                    if (done || used != i) break;
                    if (tp - i < 0) {
                        done = true;
                        break;
                    }
                    const uint64_t status = sv[i] & (3ull << 62);
                    if (((uint32_t)(sv[i] >> 48) & kEpochMask) != ep_now || status == 0) break;
                    excl += sv[i] & kCountMask;
                    ++used;
                    if (status == kStPrefix) done = true;
                }
                if (done) break;
                tp -= used;
                if (used == 0) {
                    if (++spins > kSpinLimit) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            st_store(&states[t * RADIX + dg], kStPrefix | tag | ((excl + tile_cnt) & kCountMask));
        }
        s_gofs[dg] = digit_base[dg] + (uint32_t)excl;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (d[j] < (uint32_t)RADIX) {
            uint32_t pos = s_start[d[j]] + r[j];
            if constexpr (RANK == 0) pos += s_wcnt[wave][d[j]];
            s_keys[pos] = k[j];
            s_vals[pos] = v[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + threadIdx.x;
        if (q < valid) {
            const uint64_t key = s_keys[q];
            const uint32_t dd = (uint32_t)(key >> shift) & mask;
            const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
            if (g < n) {
                out_keys[g] = key;
                out_vals[g] = s_vals[q];
            }
        }
    }
}


// persistent variant of k_split<.., RANK 1, ..>: each workgroup takes tiles
// from the ticket in increasing order and issues the loads of its next tile
// right after ranking the current one, so they are in flight during the
// look-back, the LDS staging and the writes
template <int BLOCK, int ITEMS, int RBITS, int LOOK>
__global__ __launch_bounds__(BLOCK) void k_split_pf(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                    uint64_t n, uint32_t shift, const uint32_t* __restrict__ digit_base,
                                                    uint64_t* __restrict__ states, uint32_t* __restrict__ ticket,
                                                    uint32_t epoch, uint64_t* __restrict__ out_keys,
                                                    uint32_t* __restrict__ out_vals, uint32_t* __restrict__ err) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int RADIX = 1 << RBITS;
    constexpr int RWAVES = RADIX / kWave;
    static_assert(BLOCK >= RADIX, "one thread per digit");
    (void)WAVES;
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_vals[TILE];
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile[2];

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t mask = RADIX - 1;
    const uint64_t tiles = (n + TILE - 1) / TILE;
    const uint32_t dg = threadIdx.x;
    const uint64_t tag = (uint64_t)(epoch & kEpochMask) << 48;
    if (threadIdx.x == 0) s_tile[0] = atomicAdd(ticket, 1u);
    if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;
    __syncthreads();
    uint64_t t = s_tile[0];
    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    auto load = [&](uint64_t tt, uint64_t* kk, uint32_t* vv) {
        const uint64_t tb = tt * TILE;
        const uint32_t valid = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const uint64_t e = tb + (le < valid ? le : 0u);
            kk[j] = keys[e];
            vv[j] = vals[e];
        }
    };
    if (t < tiles) load(t, k, v);
    int par = 0;
    while (t < tiles) {
        const uint64_t tb = t * TILE;
        const uint32_t valid = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);
        if (threadIdx.x == 0) s_tile[par ^ 1] = atomicAdd(ticket, 1u);
        uint32_t d[ITEMS], r[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            d[j] = le < valid ? (uint32_t)(k[j] >> shift) & mask : RADIX;
            r[j] = d[j] < (uint32_t)RADIX ? atomicAdd(&s_cnt[d[j]], 1u) : 0u;
        }
        __syncthreads();
        const uint64_t tn = s_tile[par ^ 1];
        uint64_t kn[ITEMS];
        uint32_t vn[ITEMS];
        if (tn < tiles) load(tn, kn, vn);
        uint32_t tile_cnt = 0;
        if (dg < (uint32_t)RADIX) {
            tile_cnt = s_cnt[dg];
            s_cnt[dg] = 0;   // next tile (read by all before the next atomics: two barriers below)
            if (LOOK > 0) st_store(&states[t * RADIX + dg], (t == 0 ? kStPrefix : kStAgg) | tag | tile_cnt);
        }
        {
            const uint32_t x = (dg < (uint32_t)RADIX) ? tile_cnt : 0u;
            const uint32_t inc = wave_inclusive_sum(x);
            if (lane == kWave - 1 && wave < (uint32_t)RWAVES) s_tmp[wave] = inc;
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int w = 0; w < RWAVES; ++w) off += (w < (int)wave) ? s_tmp[w] : 0u;
            if (dg < (uint32_t)RADIX) s_start[dg] = (uint16_t)(off + inc - x);
        }
        if (dg < (uint32_t)RADIX) {
            uint64_t excl = 0;
            if constexpr (LOOK == 0) {
                excl = t * (uint64_t)(TILE / RADIX);
            } else if (t > 0) {
                int64_t tp = (int64_t)t - 1;
                uint32_t spins = 0;
                const uint32_t ep_now = epoch & kEpochMask;
                while (tp >= 0) {
                    uint64_t sv[LOOK];
#pragma unroll
                    for (int i = 0; i < LOOK; ++i)
                        sv[i] = (tp - i >= 0) ? st_load(&states[(uint64_t)(tp - i) * RADIX + dg]) : 0ull;
                    int used = 0;
                    bool done = false;
#pragma unroll
                    for (int i = 0; i < LOOK; ++i) {
                        if (done || used != i) break;
                        if (tp - i < 0) {
                            done = true;
                            break;
                        }
                        const uint64_t status = sv[i] & (3ull << 62);
                        if (((uint32_t)(sv[i] >> 48) & kEpochMask) != ep_now || status == 0) break;
                        excl += sv[i] & kCountMask;
                        ++used;
                        if (status == kStPrefix) done = true;
                    }
                    if (done) break;
                    tp -= used;
                    if (used == 0) {
                        if (++spins > kSpinLimit) {
                            atomicOr(err, 1u);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                st_store(&states[t * RADIX + dg], kStPrefix | tag | ((excl + tile_cnt) & kCountMask));
            }
            s_gofs[dg] = digit_base[dg] + (uint32_t)excl;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            if (d[j] < (uint32_t)RADIX) {
                const uint32_t pos = s_start[d[j]] + r[j];
                s_keys[pos] = k[j];
                s_vals[pos] = v[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t q = j * BLOCK + threadIdx.x;
            if (q < valid) {
                const uint64_t key = s_keys[q];
                const uint32_t dd = (uint32_t)(key >> shift) & mask;
                const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
                if (g < n) {
                    out_keys[g] = key;
                    out_vals[g] = s_vals[q];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            k[j] = kn[j];
            v[j] = vn[j];
        }
        t = tn;
        par ^= 1;
    }
}

__global__ void k_hist_bits(const uint64_t* k, uint64_t n, uint32_t shift, uint32_t mask, uint32_t* h) {
    __shared__ uint32_t s[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) s[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&s[(k[i] >> shift) & mask], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += blockDim.x)
        if (s[i]) atomicAdd(&h[i], s[i]);
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? std::atoi(argv[1]) : 30;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const uint64_t n = 1ull << lg;
    uint64_t *k0, *k1, *states;
    uint32_t *v0, *v1, *ws, *err;
    unsigned long long* chk;
    CK(hipMalloc(&k0, n * 8));
    CK(hipMalloc(&k1, n * 8));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&v1, n * 4));
    const uint64_t states_n = ((n + 1023) / 1024 + 1) * 1024;
    CK(hipMalloc(&states, states_n * 8));
    CK(hipMemset(states, 0, states_n * 8));
    CK(hipMalloc(&ws, 1 << 16));
    CK(hipMalloc(&err, 256));
    CK(hipMalloc(&chk, 16));
    CK(hipMemset(err, 0, 256));
    hipLaunchKernelGGL(k_rand_keys, dim3(4096), dim3(256), 0, 0, k0, v0, n, 12345ull);
    uint32_t* ghist = ws;        // [2][1024]
    uint32_t* base = ws + 2048;  // [2][1024]
    uint32_t* tick = ws + 4096;
    const uint32_t shift = 20;
    CK(hipMemset(ghist, 0, 8192));
    hipLaunchKernelGGL(k_hist_bits, dim3(1024), dim3(256), 0, 0, (const uint64_t*)k0, n, shift, 255u, ghist);
    hipLaunchKernelGGL(k_hist_bits, dim3(1024), dim3(256), 0, 0, (const uint64_t*)k0, n, shift, 511u, ghist + 1024);
    hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, 0, (const uint32_t*)ghist, 256u, base);
    hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, 0, (const uint32_t*)ghist + 1024, 512u, base + 1024);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto f) {
        f();
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float x;
            CK(hipEventElapsedTime(&x, e0, e1));
            t.push_back(x);
        }
        std::sort(t.begin(), t.end());
        return (double)t[t.size() / 2];
    };
    auto report = [&](const char* name, double ms, uint32_t bits) {
        unsigned long long h[2] = {0, 0};
        if (bits) {
            CK(hipMemset(chk, 0, 16));
            hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, 0, (const uint64_t*)k1, (const uint32_t*)v1, n, shift,
                               (1u << bits) - 1, chk);
            CK(hipMemcpy(h, chk, 16, hipMemcpyDeviceToHost));
        }
        std::printf("%-34s %8.3f ms %7.1f GB/s  unsorted=%llu sum=%016llx\n", name, ms, 24.0 * n / ms / 1e6, h[0], h[1]);
        std::fflush(stdout);
    };
    report("copy 12 B", timeit([&] {
        hipLaunchKernelGGL(k_copy12, dim3(16384), dim3(256), 0, 0, (const uint64_t*)k0, (const uint32_t*)v0, n, k1, v1);
    }), 0);
    uint32_t epoch = 0;
#define RUN(B, I, RB, RK, LK)                                                                                  \
    do {                                                                                                       \
        auto f = [&] {                                                                                         \
            CK(hipMemsetAsync(tick, 0, 4));                                                                    \
            ++epoch;                                                                                           \
            hipLaunchKernelGGL((k_split<B, I, RB, RK, LK>), dim3((uint32_t)((n + B * I - 1) / (B * I))), dim3(B), 0, 0, \
                               (const uint64_t*)k0, (const uint32_t*)v0, n, shift,                             \
                               (const uint32_t*)(base + (RB == 9 ? 1024 : 0)), states, tick, epoch, k1, v1, err); \
        };                                                                                                     \
        const double ms = timeit(f);                                                                           \
        report("split " #B "x" #I " bits" #RB " rank" #RK " look" #LK, ms, LK ? RB : 0);                      \
    } while (0)
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    RUN(1024, 4, 8, 0, 4);
    RUN(1024, 4, 9, 0, 4);
    // product passes (sa_split.h): A = 8 bits at 20 unstable into k1/v1,
    // B = 9 bits at 28 stable w.r.t. A's digit into k2/v2 (sorted by 17 bits)
    uint64_t* k2;
    uint32_t* v2;
    CK(hipMalloc(&k2, n * 8));
    CK(hipMalloc(&v2, n * 4));
    CK(hipMemset(ghist, 0, 8192));
    hipLaunchKernelGGL(k_hist_bits, dim3(1024), dim3(256), 0, 0, (const uint64_t*)k0, n, 28u, 511u, ghist + 1024);
    hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, 0, (const uint32_t*)ghist + 1024, 512u, base + 1024);
    auto passA = [&] {
        CK(hipMemsetAsync(tick, 0, 4));
        ++epoch;
        hipLaunchKernelGGL((k_split<SrcKeys, 8, false>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0, SrcKeys{k0, v0}, n,
                           shift, 0u, 0u, (const uint32_t*)base, states, tick, epoch, k1, v1, err);
    };
    auto passB = [&] {
        CK(hipMemsetAsync(tick, 0, 4));
        ++epoch;
        hipLaunchKernelGGL((k_split<SrcKeys, 9, true>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0, SrcKeys{k1, v1}, n,
                           28u, shift, 255u, (const uint32_t*)(base + 1024), states, tick, epoch, k2, v2, err);
    };
    report("k_split A 8 bits unstable", timeit(passA), 8);
    auto passB0 = [&] {
        CK(hipMemsetAsync(tick, 0, 4));
        ++epoch;
        hipLaunchKernelGGL((k_split<SrcKeys, 9, false>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0, SrcKeys{k1, v1}, n,
                           28u, shift, 255u, (const uint32_t*)(base + 1024), states, tick, epoch, k2, v2, err);
    };
    report("k_split B 9 bits unstable", timeit(passB0), 0);
    const double msb = timeit(passB);
    {
        unsigned long long h[2] = {0, 0};
        CK(hipMemset(chk, 0, 16));
        hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, 0, (const uint64_t*)k2, (const uint32_t*)v2, n, shift,
                           (1u << 17) - 1, chk);
        CK(hipMemcpy(h, chk, 16, hipMemcpyDeviceToHost));
        std::printf("%-34s %8.3f ms %7.1f GB/s  unsorted(17 bits)=%llu sum=%016llx\n", "k_split B 9 bits stable", msb,
                    24.0 * n / msb / 1e6, h[0], h[1]);
    }
#define RUNI(RB, ST, IT)                                                                                      \
    do {                                                                                                      \
        auto f = [&] {                                                                                        \
            CK(hipMemsetAsync(tick, 0, 4));                                                                   \
            ++epoch;                                                                                          \
            if (RB == 8)                                                                                      \
                hipLaunchKernelGGL((k_split<SrcKeys, 8, ST, false, IT>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0, \
                                   SrcKeys{k0, v0}, n, shift, 0u, 0u, (const uint32_t*)base, states, tick, epoch, k1, v1, err); \
            else                                                                                              \
                hipLaunchKernelGGL((k_split<SrcKeys, 9, ST, false, IT>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0, \
                                   SrcKeys{k1, v1}, n, 28u, shift, 255u, (const uint32_t*)(base + 1024), states, tick, \
                                   epoch, k2, v2, err);                                                       \
        };                                                                                                    \
        report("k_split bits" #RB " stable" #ST " items " #IT, timeit(f), 0);                                   \
    } while (0)
    RUNI(8, false, 8);
    RUNI(8, false, 10);
    RUNI(8, false, 12);
    RUNI(9, true, 8);
    RUNI(9, true, 10);
    RUNI(9, true, 12);
    auto phases = [&](const char* name, auto launch) {
        CK(hipMemset(err, 0, 256));
        launch();
        CK(hipDeviceSynchronize());
        unsigned long long tp[5];
        CK(hipMemcpy(tp, err + 2, 40, hipMemcpyDeviceToHost));
        double tot = 0;
        for (int q = 0; q < 5; ++q) tot += (double)tp[q];
        const char* nm[5] = {"load+rank", "publish+scan", "lookback", "stage", "write"};
        std::printf("%s phases:", name);
        for (int q = 0; q < 5; ++q) std::printf("  %s %.1f%%", nm[q], 100.0 * tp[q] / tot);
        unsigned long long ls[2];
        CK(hipMemcpy(ls, err + 12, 16, hipMemcpyDeviceToHost));
        const double tiles = (double)((n + kSpTile - 1) / kSpTile);
        std::printf("  (%.0f clk per tile; look-back steps per tile-digit %.2f, empty %.2f)\n", tot / tiles,
                    ls[0] / tiles / 256.0, ls[1] / tiles / 256.0);
    };
    phases("A", [&] {
        CK(hipMemsetAsync(tick, 0, 4));
        ++epoch;
        hipLaunchKernelGGL((k_split<SrcKeys, 8, false, true>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0,
                           SrcKeys{k0, v0}, n, shift, 0u, 0u, (const uint32_t*)base, states, tick, epoch, k1, v1, err);
    });
    phases("B", [&] {
        CK(hipMemsetAsync(tick, 0, 4));
        ++epoch;
        hipLaunchKernelGGL((k_split<SrcKeys, 9, true, true>), dim3((uint32_t)cus), dim3(kSpBlock), 0, 0,
                           SrcKeys{k1, v1}, n, 28u, shift, 255u, (const uint32_t*)(base + 1024), states, tick, epoch, k2,
                           v2, err);
    });
    CK(hipMemset(err, 0, 8));
    uint32_t herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    std::printf("lookback_errors %u\n", herr);
    return 0;
}
