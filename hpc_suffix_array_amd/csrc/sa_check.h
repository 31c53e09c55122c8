// sa_check.h -- the O(n) suffix-array checker (replaces is_valid_suffix_array,
// manber_myers.c:184-202, which every caller runs after a build,
// main_sequential.c:120) as two coalesced permutations.
//
// The reference compares each adjacent pair of sorted suffixes.  The same
// verdict, in O(n):  SA is a permutation of 0..n-1, and for every r >= 1 with
// a = SA[r-1], b = SA[r]:  (text[a], ISA[a+1]) < (text[b], ISA[b+1])
// (ISA[n] = -1: the empty suffix is the smallest; equal first bytes are
// ordered by the rest of the suffix, whose position ISA gives).
//
// As two random scatters / gathers over n-entry arrays (ISA[SA[r]] = r, then
// ISA[SA[r] + 1] twice per r) that cost 111 ms at 1 GiB (r05: 38.7 and 358 GB
// of traffic for ~24 GB of algorithmic bytes).  Here each random access is an
// MSD permutation by destination, as the reference schedule's re-rank
// (sa_permute.h): a level-1 pass bins (destination, value) pairs into <= 256
// bins of 2^s1 destinations (the slots of bin b are known from b: the
// destinations of a permutation are exactly [b 2^s1, (b+1) 2^s1)), a split
// pass bins each bin again into sub-bins of 2^s2, and one workgroup per
// sub-bin places its pairs in LDS and writes or checks them whole.
//
//   pass A  pairs (SA[r], r + 1), read sequentially from SA -> ISA'[x] = r + 1
//           (k_perm_place, the re-rank's own placement: 0 = a hole).  SA is a
//           permutation iff no SA[r] >= n, every bin and sub-bin cursor ends
//           at its exact size, and no placed slot is a hole or out of place.
//   pass B  pairs (ISA'[i] - 1, text[i], ISA'[i+1]) read sequentially (ISA'[n]
//           = 0) -> at sorted position r = ISA[i] the key (text[SA[r]],
//           ISA'[SA[r]+1]), placed in LDS per 2^13-entry sub-bin, where
//           adjacent keys are compared in place; each sub-bin's first and
//           last key go to a small table that k_chk_tiles compares across
//           sub-bins.  Nothing else is written.
//
// Bytes per suffix: A 4 + 8, 8 + 8, 8 + 4; B 5 + 8, 8 + 8, 8 = 77 B, all
// streamed (or runs of ~32 pairs), against ~24 B read at random before.
// Error bits (err word): 1 SA entry >= n, 2 / 4 pass A pair out of place /
// hole, 8 pass B pair out of place, 16 a cursor off its bin's size, 32 / 64
// adjacent keys out of order inside / across sub-bins; 128 a level-1 stripe
// overflowed (not a verdict: the check runs again with one stripe).
#pragma once
#include <type_traits>

#include "sa_kernels.h"
#include "sa_permute.h"

namespace sa {

constexpr uint32_t kChkSubA = kPermSub;   // pass A sub-bins: 2^14 u32 slots in LDS
constexpr uint32_t kChkSubB = 13;         // pass B sub-bins: 2^13 u32 values + 2^13 text bytes
constexpr int kChkBlock = 1024;
constexpr int kChkItems = 8;

// pass A source: element r -> destination SA[r], pair (SA[r] << 32 | r + 1)
struct ChkSrcA {
    const uint32_t* __restrict__ sa;
    static constexpr int DSH = 32;
    static constexpr int kNb = 0;   // pair_w needs no neighbour word (see ChkSrcB)
    __device__ __forceinline__ uint32_t word(uint64_t r) const { return sa[r]; }
    __device__ __forceinline__ uint64_t dest_w(uint32_t x, uint64_t n, uint32_t& bad) const {
        if (x >= n) {
            bad |= 1u;
            return ~0ull;
        }
        return x;
    }
    __device__ __forceinline__ uint64_t pair_w(uint64_t r, uint64_t d, uint64_t, uint32_t, uint32_t) const {
        return (d << 32) | (uint32_t)(r + 1);
    }
};

// pass B source: element i -> destination ISA'[i] - 1, pair (destination's
// low s1 bits << 40 | text[i] << 32 | ISA'[i + 1]) (s1 <= 24)
struct ChkSrcB {
    const uint32_t* __restrict__ isa;
    const uint8_t* __restrict__ text;
    static constexpr int DSH = 40;
    // kNb = +1: pair_w(i) needs word(i + 1), the next lane's word (k_chk_bin
    // passes it by a lane shuffle; only a wave's last lane loads it)
    static constexpr int kNb = 1;
    __device__ __forceinline__ uint32_t word(uint64_t i) const { return isa[i]; }
    __device__ __forceinline__ uint64_t dest_w(uint32_t x, uint64_t n, uint32_t& bad) const {
        if (x == 0u || x > n) {
            bad |= 8u;
            return ~0ull;
        }
        return x - 1u;
    }
    __device__ __forceinline__ uint64_t pair_w(uint64_t i, uint64_t d, uint64_t n, uint32_t s1, uint32_t nx) const {
        return ((d & ((1ull << s1) - 1ull)) << 40) | ((uint64_t)text[i] << 32) | (i + 1 < n ? nx : 0u);
    }
};

// LCP's ISA + 1 (sa_lcp.h: LCP[r] = PLCP[SA[r]] by two permutations instead
// of a random gather): pass A's source under its own name, so profiles keep
// the two apart
struct IsaSrc : ChkSrcA {};

// LCP[r] = PLCP[i] placed at r = ISA[i] (isa1 = ISA + 1, from IsaSrc); LCP[0]
// = 0 (PLCP at SA[0] is unused, :147)
struct PlcpSrc {
    const uint32_t* __restrict__ isa1;
    const uint32_t* __restrict__ plcp;
    static constexpr int DSH = 32;
    static constexpr int kNb = 0;
    __device__ __forceinline__ uint32_t word(uint64_t i) const { return isa1[i]; }
    __device__ __forceinline__ uint64_t dest_w(uint32_t x, uint64_t n, uint32_t& bad) const {
        if (x == 0u || x > n) {   // (an invalid SA only)
            bad |= 8u;
            return ~0ull;
        }
        return x - 1u;
    }
    __device__ __forceinline__ uint64_t pair_w(uint64_t i, uint64_t d, uint64_t, uint32_t, uint32_t) const {
        return (d << 32) | (d ? plcp[i] : 0u);
    }
};

// LCP's PHI (sa_lcp.h) by the same permutation: element r -> destination
// SA[r], value PHI'[SA[r]] = SA[r - 1] + 1 (0 for r = 0: no predecessor;
// a hole of an invalid SA reads as 0 too, so PHI' - 1 never indexes past n)
struct PhiSrc {
    const uint32_t* __restrict__ sa;
    static constexpr int DSH = 32;
    // kNb = -1: pair_w(r) needs word(r - 1), the previous lane's word
    static constexpr int kNb = -1;
    __device__ __forceinline__ uint32_t word(uint64_t r) const { return sa[r]; }
    __device__ __forceinline__ uint64_t dest_w(uint32_t x, uint64_t n, uint32_t&) const {
        return x < n ? (uint64_t)x : ~0ull;
    }
    __device__ __forceinline__ uint64_t pair_w(uint64_t r, uint64_t d, uint64_t n, uint32_t, uint32_t p) const {
        return (d << 32) | (r && p < n ? p + 1u : 0u);
    }
};

// Level 1's output: bin b's pairs, or with stripes (st > 1) the pairs of bin
// b claimed by the workgroups of XCD-aligned stripe q = w mod st, at
// [(b st + q) scap, + scap).  One cursor per bin took a device-scope claim
// from every tile on each of 256 addresses (131 K claims per address at 1 GiB,
// serialised at ~19 ns: the checker's level-1 passes ran at 3 TB/s against
// the split pass's 5.2); eight stripes cut that eightfold.  A stripe that
// fills up (an adversarial input: a valid permutation splits every bin
// evenly over the stripes, +-0.1 %) drops its pair and raises bit 128; the
// host then runs the permutation again with one stripe.
struct BinStripes {
    uint32_t st = 1;      // stripes per bin
    uint64_t scap = 0;    // pairs per (bin, stripe) region (st > 1)
};

// Level 1: tile of BLOCK x ITEMS elements -> pairs staged in LDS by bin
// (d >> s1), each bin's slots claimed from its (stripe's) cursor, one
// device-scope atomic per tile and bin, and written as runs.  A slot at or
// past its bin's size (a non-permutation) is dropped; the cursor test flags it.
// NB: level-1 bins (256; 512 / 1024 cut the same-address collisions of the
// LDS rank atomics, 64 lanes over 256 counters, at shorter runs)
template <int BLOCK, int ITEMS, class Src, int NB = 256>
__global__ __launch_bounds__(BLOCK) void k_chk_bin(Src src, uint64_t n, uint32_t s1, uint32_t* __restrict__ cur,
                                                    uint64_t* __restrict__ out, uint32_t* __restrict__ err,
                                                    BinStripes bs = BinStripes{}) {
    constexpr int T = BLOCK * ITEMS;
    static_assert(BLOCK >= NB, "one thread per bin");
    using BinT = typename std::conditional<(NB > 256), uint16_t, uint8_t>::type;
    __shared__ uint64_t s_pair[T];
    __shared__ BinT s_bin[T];
    __shared__ uint32_t s_cnt[NB];
    __shared__ uint32_t s_start[NB + 1];
    __shared__ uint32_t s_gofs[NB];
    __shared__ uint32_t s_tmp[NB / kWave];
    const uint32_t tid = threadIdx.x;
    const uint64_t tb = (uint64_t)blockIdx.x * T;
    const uint32_t q = blockIdx.x % bs.st;
    if (tid < (uint32_t)NB) s_cnt[tid] = 0;
    __syncthreads();
    uint32_t bad = 0;
    uint64_t d[ITEMS];
    uint64_t p[ITEMS];
    uint32_t slot[ITEMS];
    {   // (a source: word(e), dest_w(word), pair_w(e, dest, n, s1, neighbour word))
        // every element's word loaded first, all loads in flight before the
        // first use (separate dest / pair loops ran pass A's level 1 at 4.26
        // ms, this 3.4); an element's neighbour word (e + kNb) is the
        // adjacent lane's: a lane shuffle, and one load by the wave's edge
        // lane (ChkSrcB 5.41 -> 4.69 ms, PhiSrc 4.60 -> 3.37)
        const uint32_t lane = lane_id();
        uint32_t x[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t e = tb + (uint64_t)j * BLOCK + tid;
            x[j] = e < n ? src.word(e) : 0u;
        }
        uint32_t nb[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t e = tb + (uint64_t)j * BLOCK + tid;
            if constexpr (Src::kNb == 0) {
                nb[j] = 0u;
            } else if constexpr (Src::kNb > 0) {
                nb[j] = (uint32_t)__shfl_down((int)x[j], 1, kWave);
                if (lane == kWave - 1) nb[j] = e + 1 < n ? src.word(e + 1) : 0u;
            } else {
                nb[j] = (uint32_t)__shfl_up((int)x[j], 1, kWave);
                if (lane == 0) nb[j] = e > 0 && e - 1 < n ? src.word(e - 1) : 0u;
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t e = tb + (uint64_t)j * BLOCK + tid;
            d[j] = e < n ? src.dest_w(x[j], n, bad) : ~0ull;
            p[j] = d[j] != ~0ull ? src.pair_w(e, d[j], n, s1, nb[j]) : 0ull;
            slot[j] = d[j] != ~0ull ? atomicAdd(&s_cnt[(uint32_t)(d[j] >> s1)], 1u) : 0u;
        }
    }
    __syncthreads();
    const uint32_t cnt = tid < (uint32_t)NB ? s_cnt[tid] : 0u;
    const uint32_t st = perm_scan<NB>(cnt, s_tmp);
    if (tid < (uint32_t)NB) {
        s_start[tid] = st;
        if (tid == NB - 1) s_start[NB] = st + cnt;
        s_gofs[tid] = cnt ? atomicAdd(&cur[q * NB + tid], cnt) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        if (d[j] != ~0ull) {
            const uint32_t b = (uint32_t)(d[j] >> s1);
            const uint32_t x = s_start[b] + slot[j];
            s_pair[x] = p[j];
            s_bin[x] = (BinT)b;
        }
    __syncthreads();
    const uint32_t tot = s_start[NB];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t x = j * BLOCK + tid;
        if (x < tot) {
            const uint32_t b = s_bin[x];
            const uint64_t g = (uint64_t)s_gofs[b] + (x - s_start[b]);
            if (bs.st > 1) {
                if (g < bs.scap) out[((uint64_t)b * bs.st + q) * bs.scap + g] = s_pair[x];
                else bad |= 128u;
            } else {
                const uint64_t b0 = (uint64_t)b << s1;
                const uint64_t bsz = (n - b0) < (1ull << s1) ? n - b0 : (1ull << s1);
                if (g < bsz) out[b0 + g] = s_pair[x];
            }
        }
    }
    if (bad) atomicOr(err, bad);
}

// Level 2 over striped level-1 output: workgroup w takes tile t of region
// (bin b, stripe q), b's regions all on XCD b mod 8 (w mod 8, so that one
// L2 merges the partial lines where consecutive tiles' runs of a sub-bin
// meet, as k_perm_split); the region's fill is its level-1 cursor.  Pairs
// into 2^s2-entry sub-bins of the final layout by their cursors (as
// k_perm_split; CLAMP: a slot past its sub-bin is dropped).
// grid = 8 ceil(nb1 / 8) st tps, tps = ceil(scap / T).
template <int BLOCK, int ITEMS, int DSH, int TAG = 0>
__global__ __launch_bounds__(BLOCK) void k_chk_split(const uint64_t* __restrict__ in, uint64_t n, uint32_t s1,
                                                      uint32_t s2, BinStripes bs, uint32_t tps,
                                                      const uint32_t* __restrict__ fill, uint32_t fstride,
                                                      uint32_t* __restrict__ cur, uint64_t* __restrict__ out) {
    constexpr int T = BLOCK * ITEMS;
    constexpr int NB = kPermMaxSub;
    static_assert(BLOCK >= NB, "one thread per sub-bin");
    __shared__ uint64_t s_pair[T];
    __shared__ uint32_t s_cnt[NB];
    __shared__ uint32_t s_start[NB];
    __shared__ uint32_t s_gofs[NB];
    __shared__ uint32_t s_tmp[NB / kWave];
    const uint32_t tid = threadIdx.x;
    uint32_t R = blockIdx.x >> 3;
    const uint32_t t = R % tps;
    R /= tps;
    const uint32_t q = R % bs.st;
    const uint32_t b = (R / bs.st) * 8u + (blockIdx.x & 7u);
    const uint64_t bin0 = (uint64_t)b << s1;
    if (bin0 >= n) return;   // uniform over the workgroup
    const uint64_t f = fill[q * fstride + b] < bs.scap ? fill[q * fstride + b] : bs.scap;
    const uint64_t t0 = (uint64_t)t * T;
    if (t0 >= f) return;
    const uint32_t valid = (uint32_t)((f - t0) < (uint64_t)T ? (f - t0) : (uint64_t)T);
    const uint64_t src0 = ((uint64_t)b * bs.st + q) * bs.scap + t0;
    const uint32_t nsub = 1u << (s1 - s2);
    if (tid < (uint32_t)NB) s_cnt[tid] = 0;
    __syncthreads();
    uint64_t p[ITEMS];
    uint32_t sub[ITEMS], slot[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t x = j * BLOCK + tid;
        p[j] = in[src0 + (x < valid ? x : valid - 1)];   // every load before the first use
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t x = j * BLOCK + tid;
        sub[j] = x < valid ? ((uint32_t)(p[j] >> DSH) >> s2) & (nsub - 1u) : NB;
        slot[j] = sub[j] < (uint32_t)NB ? atomicAdd(&s_cnt[sub[j]], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t cnt = tid < (uint32_t)NB ? s_cnt[tid] : 0u;
    const uint32_t st = perm_scan<NB>(cnt, s_tmp);
    if (tid < (uint32_t)NB) {
        s_start[tid] = st;
        s_gofs[tid] = cnt ? (uint32_t)bin0 + (tid << s2) + atomicAdd(&cur[(uint64_t)b * nsub + tid], cnt) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        if (sub[j] < (uint32_t)NB) s_pair[s_start[sub[j]] + slot[j]] = p[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t x = j * BLOCK + tid;
        if (x < valid) {
            const uint64_t v = s_pair[x];
            const uint32_t sb = ((uint32_t)(v >> DSH) >> s2) & (nsub - 1u);
            const uint64_t g = (uint64_t)s_gofs[sb] + (x - s_start[sb]);
            const uint64_t s0 = bin0 + ((uint64_t)sb << s2);
            if (g < n && g < s0 + (1ull << s2)) out[g] = v;
        }
    }
}

// every cursor at its bin's / sub-bin's exact size (else bit 16); a bin's
// level-1 count is the sum over its stripes
__global__ __launch_bounds__(kBlock) void k_chk_cursors(const uint32_t* __restrict__ cur1,
                                                        const uint32_t* __restrict__ cur2, uint64_t n, uint32_t s1,
                                                        uint32_t s2, uint32_t nb1, uint32_t* __restrict__ err,
                                                        uint32_t st = 1, uint32_t fstride = 256) {
    const uint32_t nsub = 1u << (s1 - s2);
    const uint64_t total = (uint64_t)nb1 * (s1 > s2 ? nsub + 1 : 1);
    bool bad = false;
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < total; k += (uint64_t)gridDim.x * kBlock) {
        uint64_t lo, width;
        uint64_t got = 0;
        if (k < nb1) {
            lo = k << s1;
            width = 1ull << s1;
            for (uint32_t q = 0; q < st; ++q) got += cur1[q * fstride + k];
        } else {
            const uint64_t t = k - nb1;
            lo = (t / nsub << s1) + ((t % nsub) << s2);
            width = 1ull << s2;
            got = cur2[t];
        }
        const uint64_t want = lo >= n ? 0 : (n - lo < width ? n - lo : width);
        bad |= got != want;
    }
    if (bad) atomicOr(err, 16u);
}

// pass B level 3: one workgroup per 2^kChkSubB sorted positions.  The keys
// (text[SA[r]] << 32 | ISA'[SA[r] + 1]) land in LDS by r; adjacent ones must
// rise strictly (bit 32); the sub-bin's first and last key go to ends[2 sb],
// ends[2 sb + 1] for k_chk_tiles.  A pair whose destination is not in this
// sub-bin raises bit 8 (only after a failed pass A).
// SUB: the sub-bin bits (kChkSubB; 14 above 2^31 suffixes, where 2^13-entry
// sub-bins would need more than the split pass's 1024 per bin)
template <int BLOCK, int SUB = kChkSubB>
__global__ __launch_bounds__(BLOCK) void k_chk_place(const uint64_t* __restrict__ in, uint64_t n, uint32_t s1,
                                                      uint64_t* __restrict__ ends, uint32_t* __restrict__ err) {
    constexpr uint32_t S = 1u << SUB;
    constexpr int ITEMS = S / BLOCK;
    static_assert(ITEMS * BLOCK == (int)S, "whole sub-bins per workgroup");
    __shared__ uint32_t s_v[S];
    __shared__ uint8_t s_t[S];
    const uint32_t sb = blockIdx.x;
    const uint64_t base = (uint64_t)sb << SUB;
    const uint32_t valid = (uint32_t)((n - base) < (uint64_t)S ? (n - base) : (uint64_t)S);
    const uint32_t rel = (uint32_t)(base & ((1ull << s1) - 1ull));   // the sub-bin's offset in its bin
    uint64_t p[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + threadIdx.x;
        p[j] = in[base + (q < valid ? q : valid - 1)];
    }
    uint32_t bad = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + threadIdx.x;
        if (q < valid) {
            const uint32_t dl = (uint32_t)(p[j] >> 40);
            const uint32_t x = dl - rel;
            if (x >= valid) {
                bad |= 8u;
                continue;
            }
            s_v[x] = (uint32_t)p[j];
            s_t[x] = (uint8_t)(p[j] >> 32);
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + threadIdx.x;
        if (q + 1 < valid) {
            const uint64_t a = ((uint64_t)s_t[q] << 32) | s_v[q];
            const uint64_t b = ((uint64_t)s_t[q + 1] << 32) | s_v[q + 1];
            if (!(a < b)) bad |= 32u;
        }
    }
    if (threadIdx.x == 0) {
        ends[2 * (uint64_t)sb] = ((uint64_t)s_t[0] << 32) | s_v[0];
        ends[2 * (uint64_t)sb + 1] = ((uint64_t)s_t[valid - 1] << 32) | s_v[valid - 1];
    }
    if (bad) atomicOr(err, bad);
}

// the last key of each sub-bin below the first key of the next (else bit 64)
__global__ __launch_bounds__(kBlock) void k_chk_tiles(const uint64_t* __restrict__ ends, uint64_t nsb,
                                                      uint32_t* __restrict__ err) {
    bool bad = false;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t + 1 < nsb; t += (uint64_t)gridDim.x * kBlock)
        bad |= !(ends[2 * t + 1] < ends[2 * t + 2]);
    if (bad) atomicOr(err, 64u);
}

}  // namespace sa
