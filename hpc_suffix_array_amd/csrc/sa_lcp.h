// sa_lcp.h -- LCP array and longest repeated substring on the GPU
// (replaces build_lcp_array, manber_myers.c:135-157, and the scan of
// find_longest_repeated_substring, :159-182).
//
// Kasai's loop (:146-155) is sequential through h.  The same values come from
// the permuted LCP array PLCP[i] = lcp(i, PHI[i]), PHI[SA[r]] = SA[r-1]
// (placed by the checker's coalesced permutation, sa_check.h PhiSrc, not a
// random scatter):
//   * i is *reducible* when text[i-1] == text[PHI[i]-1]; then
//     PHI[i-1] = PHI[i]-1 and PLCP[i] = PLCP[i-1] - 1 (Kasai's own invariant);
//   * the other (irreducible) positions are compared directly; their lcp values
//     sum to at most 2 n log2 n (Kaerkkaeinen, Manzini & Puglisi, CPM 2009);
//   * PLCP[i] + i never decreases along i (Kasai: PLCP[i] >= PLCP[i-1] - 1), so
//     the reducible values are an inclusive max-scan of v[i] = PLCP[i] + i over
//     the irreducible positions (v = 0 elsewhere), minus i;
//   * LCP[r] = PLCP[SA[r]], LCP[0] = 0 (:147).
// Direct comparisons run 8 bytes at a time.  A pair still equal after
// kDirect bytes is handed to the cooperative rounds: round k compares the
// window [lo_k, 4 lo_k) of every surviving pair, kSeg bytes per workgroup item,
// with an atomicMin of the first mismatch -- a long repeat (a 1 GiB run of one
// byte) is spread over the whole GPU instead of one thread.  The launch
// sequence is fixed (no host sync): each round reads its pair count from HBM.
#pragma once

#include "sa_kernels.h"

namespace sa {

constexpr uint32_t kPhiNone = 0xFFFFFFFFu;
constexpr uint32_t kDirect = 128;     // bytes a thread compares before handing a pair off
constexpr uint32_t kSeg = 2048;       // bytes per workgroup item in the cooperative rounds (256 x 8)
constexpr int kLongRounds = 14;       // kDirect * 4^13 >= 2^32: every pair resolves

// little-endian 8 bytes at p (any alignment); bytes at or past n read as 0.
// Inside the text two aligned words are read and funnel-shifted: each holds at
// least one byte below n, so neither can cross into an unmapped page.
__device__ __forceinline__ uint64_t load8(const uint8_t* __restrict__ text, uint64_t p, uint64_t n) {
    if (p + 8 <= n) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(text + p);
        const uint64_t* w = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
        const uint32_t sh = (uint32_t)(a & 7) * 8;
        const uint64_t lo = w[0];
        if (sh == 0) return lo;
        return (lo >> sh) | (w[1] << (64 - sh));
    }
    uint64_t x = 0;
    for (uint64_t b = p; b < n && b < p + 8; ++b) x |= (uint64_t)text[b] << (8 * (b - p));
    return x;
}

// first offset in [off, off + 8) where the suffixes at a and b differ, capped
// at lim (the shorter suffix's length); ~0 when the 8 bytes agree below lim.
__device__ __forceinline__ uint64_t mismatch8(const uint8_t* __restrict__ text, uint64_t n, uint64_t a, uint64_t b,
                                              uint64_t off, uint64_t lim) {
    if (off >= lim) return lim;
    const uint64_t d = load8(text, a + off, n) ^ load8(text, b + off, n);
    uint64_t m = d ? off + (uint64_t)(__builtin_ctzll(d) >> 3) : ~0ull;
    if (off + 8 > lim && m > lim) m = lim;
    return m;
}

// v[i] = PLCP[i] + i for irreducible i, 0 for reducible i; pairs still equal
// after kDirect bytes go to the first cooperative list with mm = ~0.
// phi1 = PHI + 1 (the permutation's placement, sa_check.h PhiSrc): 0 = none,
// so phi1 - 1 wraps to kPhiNone
__global__ __launch_bounds__(kBlock) void k_plcp_irreducible(const uint8_t* __restrict__ text, uint64_t n,
                                                             const uint32_t* __restrict__ phi1,
                                                             uint32_t* __restrict__ v,
                                                             uint64_t* __restrict__ list, uint32_t* __restrict__ mm,
                                                             uint32_t* __restrict__ cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint32_t j = phi1[i] - 1u;
        if (j == kPhiNone) {   // the smallest suffix: LCP[0] = 0 is fixed, PLCP unused
            v[i] = 0;
            continue;
        }
        if (i > 0 && j > 0 && phi1[i - 1] != 0u && text[i - 1] == text[j - 1]) {
            v[i] = 0;   // reducible: PLCP[i] = PLCP[i-1] - 1
            continue;
        }
        const uint64_t lim = n - (i > j ? i : j);
        uint64_t m = ~0ull;
        for (uint64_t off = 0; off < kDirect && m == ~0ull; off += 8) m = mismatch8(text, n, i, j, off, lim);
        if (m != ~0ull) {
            v[i] = (uint32_t)(m + i);
        } else {
            const uint32_t q = atomicAdd(cnt, 1u);
            list[q] = (i << 32) | j;
            mm[q] = 0xFFFFFFFFu;
            v[i] = 0;   // written by the round that resolves it
        }
    }
}

// round k of the cooperative comparison: window [lo, hi) of every listed pair
__global__ __launch_bounds__(kBlock) void k_plcp_long(const uint8_t* __restrict__ text, uint64_t n,
                                                      const uint64_t* __restrict__ list,
                                                      const uint32_t* __restrict__ cnt, uint64_t lo, uint64_t hi,
                                                      uint32_t* __restrict__ mm) {
    const uint64_t pairs = *cnt;
    if (pairs == 0) return;
    const uint64_t segs = (hi - lo + kSeg - 1) / kSeg;
    const uint64_t items = pairs * segs;
    for (uint64_t w = blockIdx.x; w < items; w += gridDim.x) {
        const uint64_t p = w / segs, sg = w - p * segs;
        const uint64_t e = list[p];
        const uint64_t a = e >> 32, b = e & 0xFFFFFFFFull;
        const uint64_t lim = n - (a > b ? a : b);
        const uint64_t off = lo + sg * kSeg + (uint64_t)threadIdx.x * 8;
        if (off >= hi || off > lim) continue;
        const uint64_t m = mismatch8(text, n, a, b, off, lim);
        if (m != ~0ull) atomicMin(&mm[p], (uint32_t)m);
    }
}

// resolve the pairs whose window held a mismatch; move the rest to the next list
__global__ __launch_bounds__(kBlock) void k_plcp_settle(const uint64_t* __restrict__ list,
                                                        const uint32_t* __restrict__ cnt, uint32_t* __restrict__ mm,
                                                        uint32_t* __restrict__ v, uint64_t* __restrict__ next,
                                                        uint32_t* __restrict__ next_cnt) {
    const uint32_t pairs = *cnt;
    for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < pairs; p += gridDim.x * kBlock) {
        const uint64_t e = list[p];
        const uint32_t m = mm[p];
        mm[p] = 0xFFFFFFFFu;   // the next list reuses slots below its (smaller) count
        if (m != 0xFFFFFFFFu) {
            v[e >> 32] = (uint32_t)(m + (e >> 32));
        } else {
            next[atomicAdd(next_cnt, 1u)] = e;
        }
    }
}

// inclusive max-scan of v in place, chunked like the radix kernels:
// per-chunk maxima, their exclusive scan, then a carried scan per chunk that
// writes PLCP[i] = max-scan(v)[i] - i.
__device__ __forceinline__ uint32_t wave_inclusive_max(uint32_t x) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, kWave);
        if ((int)lane_id() >= o) x = x > y ? x : y;
    }
    return x;
}

__global__ __launch_bounds__(kBlock) void k_chunk_max(const uint32_t* __restrict__ v, Chunking ch,
                                                      uint32_t* __restrict__ cmax) {
    __shared__ uint32_t s[kWaves];
    const uint64_t e0 = ch.begin(blockIdx.x), e1 = ch.end(blockIdx.x);
    uint32_t m = 0;
    for (uint64_t i = e0 + threadIdx.x; i < e1; i += kBlock) m = m > v[i] ? m : v[i];
    m = wave_inclusive_max(m);
    if (lane_id() == kWave - 1) s[wave_id()] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kWaves; ++w) t = t > s[w] ? t : s[w];
        cmax[blockIdx.x] = t;
    }
}

// exclusive max-scan of the chunk maxima (one workgroup; blocks of kBlock * 16
// chunks with a carry, so any chunk count is scanned -- SA_MAX_CHUNKS is a
// build-time override)
__global__ __launch_bounds__(kBlock) void k_scan_chunk_max(uint32_t* __restrict__ cmax, uint32_t chunks) {
    __shared__ uint32_t s[kWaves];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < chunks; base += kBlock * 16) {
        uint32_t x[16], m = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = base + threadIdx.x * 16 + j;
            x[j] = i < chunks ? cmax[i] : 0u;
            m = m > x[j] ? m : x[j];
        }
        const uint32_t inc = wave_inclusive_max(m);
        if (lane_id() == kWave - 1) s[wave_id()] = inc;
        __syncthreads();
        uint32_t run = carry, blk = carry;
        for (int w = 0; w < kWaves; ++w) {
            if (w < (int)wave_id()) run = run > s[w] ? run : s[w];
            blk = blk > s[w] ? blk : s[w];
        }
        uint32_t ex = __shfl_up(inc, 1, kWave);
        if (lane_id() == 0) ex = 0;
        run = run > ex ? run : ex;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = base + threadIdx.x * 16 + j;
            if (i < chunks) cmax[i] = run;
            run = run > x[j] ? run : x[j];
        }
        carry = blk;
        __syncthreads();   // s[] is rewritten by the next block
    }
}

__global__ __launch_bounds__(kBlock) void k_plcp_apply(uint32_t* __restrict__ v, Chunking ch,
                                                       const uint32_t* __restrict__ cmax) {
    __shared__ uint32_t s[kWaves];
    const uint64_t e0 = ch.begin(blockIdx.x), e1 = ch.end(blockIdx.x);
    uint32_t carry = cmax[blockIdx.x];
    for (uint64_t tb = e0; tb < e1; tb += kBlock) {
        const uint64_t i = tb + threadIdx.x;
        const uint32_t x = i < e1 ? v[i] : 0u;
        const uint32_t inc = wave_inclusive_max(x);
        if (lane_id() == kWave - 1) s[wave_id()] = inc;
        __syncthreads();
        uint32_t run = carry;
        uint32_t all = carry;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            if (w < (int)wave_id()) run = run > s[w] ? run : s[w];
            all = all > s[w] ? all : s[w];
        }
        run = run > inc ? run : inc;
        if (i < e1) v[i] = run - (uint32_t)i;   // PLCP[i] (garbage only at SA[0], never read)
        carry = all;
        __syncthreads();
    }
}

// LCP[r] = PLCP[SA[r]], LCP[0] = 0; best = max over r >= 1 of (LCP[r] << 32 | ~r)
// (first r with the strictly largest value, as :165-171)
__global__ __launch_bounds__(kBlock) void k_lcp_gather(const uint32_t* __restrict__ sa, uint64_t n,
                                                       const uint32_t* __restrict__ plcp,
                                                       uint32_t* __restrict__ lcp,
                                                       unsigned long long* __restrict__ best) {
    unsigned long long b = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r < n; r += (uint64_t)gridDim.x * kBlock) {
        const uint32_t q = sa[r];
        const uint32_t x = (r && q < n) ? plcp[q] : 0u;
        lcp[r] = x;
        const unsigned long long k = ((unsigned long long)x << 32) | (0xFFFFFFFFull - r);
        b = b > k ? b : k;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(b, o, kWave);
        b = b > y ? b : y;
    }
    if (lane_id() == 0 && (b >> 32)) atomicMax(best, b);
}

// the LRS over the finished LCP array: max over r >= 1 of (LCP[r] << 32 | ~r)
// (first r with the strictly largest value, as :165-171)
__global__ __launch_bounds__(kBlock) void k_lcp_best(const uint32_t* __restrict__ lcp, uint64_t n,
                                                     unsigned long long* __restrict__ best) {
    unsigned long long b = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x + 1; r < n; r += (uint64_t)gridDim.x * kBlock) {
        const unsigned long long k = ((unsigned long long)lcp[r] << 32) | (0xFFFFFFFFull - r);
        b = b > k ? b : k;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(b, o, kWave);
        b = b > y ? b : y;
    }
    if (lane_id() == 0 && (b >> 32)) atomicMax(best, b);
}

}  // namespace sa
