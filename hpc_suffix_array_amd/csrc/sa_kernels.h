// sa_kernels.h -- CDNA4 (gfx950, wave64) kernels of one Manber-Myers
// rank-doubling round.  Replaces the loop body of build_suffix_array,
// src/sequential/manber_myers.c:97-125 of the reference:
//
//   reference loop nest (file:line)          kernel here
//   init            :88-92                   k_init_rank
//   counting sort   :15-34 (x2, :42,:45)     k_hist -> k_scan_rows -> k_scatter
//                                            (8-bit LSD digits over the packed
//                                            key (r[i] << w) | r[i+h])
//   re-rank         :101-110                 k_heads -> k_scan_heads -> k_rerank
//   update          :116-124                 fused into the next round's first
//                                            k_hist / k_scatter (key built from
//                                            rank[i], rank[i+h] in text order)
//
// Layout in HBM (n symbols, all arrays 256-byte aligned):
//   rank  u32[n]   dense rank of the h-prefix of suffix i, 1..D; 0 = past end
//   keys  u64[n]x2 ping-pong (r0 << w) | r1, r0, r1 < 2^w, 2w <= 64
//   vals  u32[n]x2 suffix index carried with its key (one of them is the
//                  caller's SA buffer, so the last pass lands in place)
//   hist  u32[256 * C]   per (digit, chunk) counts, digit-major, scanned in place
//
// A chunk is a contiguous run of tiles handled by one workgroup in every
// kernel, so the chunk-local histograms of k_hist are exactly the offsets
// k_scatter needs (reduce-then-scan radix sort; no inter-workgroup waits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sa_search.h"

namespace sa {

constexpr int kWave = 64;
constexpr int kBlock = 256;                 // 4 waves
constexpr int kWaves = kBlock / kWave;
constexpr int kItems = 16;                  // keys per lane per tile
constexpr int kTile = kBlock * kItems;      // 4096 suffixes per tile
constexpr int kWaveTile = kWave * kItems;   // 1024 per wave
constexpr int kRadix = 256;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ uint32_t wave_id() { return threadIdx.x / kWave; }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// ---------------------------------------------------------------------------
// key sources: where a radix pass reads its (key, idx) pairs
// ---------------------------------------------------------------------------
// First pass of a round: build the pair key from ranks in TEXT order
// (coalesced: rank[i] and rank[i+h] are two sequential streams), index = i.
// This is the update step of manber_myers.c:116-124 fused into the sort.
struct SrcRank {
    const uint32_t* __restrict__ rank;
    uint64_t n;
    uint64_t h;
    uint32_t w;
    __device__ __forceinline__ uint64_t key(uint64_t e) const {
        const uint64_t r0 = rank[e];
        const uint64_t r1 = (e + h < n) ? rank[e + h] : 0u;
        return (r0 << w) | r1;
    }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return (uint32_t)e; }
    // two-step form (loads, then the key) for the prefetch of sa_lsd.h k_lsd
    static constexpr bool kRaw = true;
    __device__ __forceinline__ uint64_t raw(uint64_t e) const {
        return (uint64_t)rank[e] | ((uint64_t)((e + h < n) ? rank[e + h] : 0u) << 32);
    }
    __device__ __forceinline__ uint64_t finish(uint64_t r, uint64_t) const {
        return ((r & 0xFFFFFFFFull) << w) | (r >> 32);
    }
};

// Packed schedule, first round: key = the first K symbols of suffix i packed
// base B = sigma + 1 (dense codes 1..sigma, 0 = past the end), so key order
// is the lexicographic order of K-prefixes with the end smallest.  Replaces
// rounds h = 1 .. K/2 of the reference loop (manber_myers.c:88-125) by one
// sort.  B^K <= 2^64 is guaranteed by the host.
struct SrcText {
    const uint8_t* __restrict__ text;
    const uint16_t* __restrict__ code;  // 256-entry byte -> dense code 1..sigma
    uint64_t n;
    uint64_t base;
    uint32_t K;
    __device__ __forceinline__ uint64_t key(uint64_t e) const {
        uint64_t x = 0;
        if (e + K <= n) {
            for (uint32_t t = 0; t < K; ++t) x = x * base + code[text[e + t]];
        } else {
            for (uint32_t t = 0; t < K; ++t) x = x * base + ((e + t < n) ? code[text[e + t]] : 0u);
        }
        return x;
    }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return (uint32_t)e; }
};

// Key layout of the bucketed first round (sa_bucket.h): key1 = D << rb | low
// with D the dense s-symbol prefix and, for a suffix of length L >= s, low =
// s + the dense next R symbols (0 past the end) times (R + 1) plus the number
// of them before the end (L - 1 for a suffix of length L < s).
// Compact variant (cmp = 1): low = 2 r + [L >= K] for every suffix (D and r
// with digit 0 past the end) -- one bit instead of log2(R + 1) for the end
// and no offset for the suffixes shorter than s, so low fills its rb bits
// (the local sort's sub-buckets stay uniform).  Exact when no two of the
// text's last K - 1 suffixes share (D, r), which the host checks on the
// text's tail before choosing it (short_suffix_ties, sa_round1.h): a short
// suffix then differs from every other short one in (D, r), and from the
// longer suffixes continuing it with the smallest symbol -- equal (D, r), it
// is their prefix -- in the bit.
// E-only variant (cmp = 2): low = r, no end bit -- one bit less, which lets
// a non-power-of-two alphabet's first pass write packed 8-byte items (1 GiB
// alnum / ascii127: 65 -> 64 bits).  A short suffix S then shares its key
// with the suffixes continuing it with the smallest symbol; round 2 orders
// them (S + K is past the end: rank 0).  Exact when the text's last K
// suffixes have distinct (D, r) (short_suffix_ties over K, host-checked;
// tests/test_key1_layout.py runs the packed doubling on it).
struct BucketSpec {
    uint64_t pow_s1;   // sigma^(s-1)
    uint64_t powR1;    // sigma^(R-1)
    uint64_t cmul;     // floor(2^48 / sigma^s): bucket = (D * cmul) >> bsh
    uint32_t sigma, s, R, rb;
    uint32_t bb, bsh;  // bucket bits (16..18), bsh = 48 - bb
    uint32_t cmp;      // 1: compact low, 2: E-only low
};

// low of a suffix of length L with next-R-symbols value r (see BucketSpec)
__host__ __device__ __forceinline__ uint64_t bucket_low(const BucketSpec& b, uint64_t r, uint64_t L) {
    if (b.cmp == 2) return r;
    if (b.cmp) return 2 * r + (L >= b.s + b.R ? 1u : 0u);
    if (L < b.s) return L - 1;
    const uint64_t tl = L - b.s < b.R ? L - b.s : b.R;
    return b.s + r * (b.R + 1) + tl;
}

// byte -> dense digit (code - 1, absent bytes 0) from the global code table
struct CodeMap {
    const uint16_t* __restrict__ code;
    __device__ __forceinline__ uint32_t operator[](uint32_t b) const {
        const uint32_t c = code[b];
        return c ? c - 1u : 0u;
    }
};

// key1 of suffix j (sa_bucket.h layout) from the text in HBM: the bytes of
// [j, j + K) arrive as independent aligned words (one memory latency instead
// of K dependent byte + table loads), digits through the LDS byte map (code -
// 1; 0 past the end).  FULL = false: only D (the bucket's input).
constexpr int kKeyWords = 8;   // K <= 29 symbols; longer keys take the byte loop

// Map: byte -> digit by operator[] (the LDS byte map of load_map, or
// CodeMap over the global code table).
template <bool FULL, class Map>
__device__ __forceinline__ uint64_t key1_words(const uint8_t* __restrict__ text, uint64_t n, const Map& s_map,
                                               const BucketSpec& b, uint64_t j, uint32_t* D_out) {
    const uint32_t K = FULL ? b.s + b.R : b.s;
    uint64_t D = 0, r = 0;
    if (K + 3 <= 4 * kKeyWords) {
        const uint64_t base = j & ~3ull;
        const uint32_t sh = (uint32_t)(j & 3);
        uint32_t w[kKeyWords + 1];
#pragma unroll
        for (int q = 0; q <= kKeyWords; ++q) {
            const uint64_t a = base + 4ull * q;
            if (a + 4 <= n) {
                w[q] = *reinterpret_cast<const uint32_t*>(text + a);
            } else {
                uint32_t v = 0;
                for (int i = 0; i < 4; ++i)
                    if (a + i < n) v |= (uint32_t)text[a + i] << (8 * i);
                w[q] = v;
            }
        }
#pragma unroll
        for (int q = 0; q < kKeyWords; ++q) {
            const uint32_t x = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t t = 4 * q + i;
                if (t < K) {
                    const uint32_t c = (j + t < n) ? (uint32_t)s_map[(x >> (8 * i)) & 0xFFu] : 0u;
                    if (t < b.s) D = D * b.sigma + c;
                    else r = r * b.sigma + c;
                }
            }
        }
    } else {
        for (uint32_t t = 0; t < K; ++t) {
            const uint32_t c = (j + t < n) ? (uint32_t)s_map[text[j + t]] : 0u;
            if (t < b.s) D = D * b.sigma + c;
            else r = r * b.sigma + c;
        }
    }
    *D_out = (uint32_t)D;
    if (!FULL) return 0;
    return (D << b.rb) | bucket_low(b, r, n - j);
}

// Packed schedule, later rounds: only the suffixes whose group is not yet a
// singleton (compacted in SA order: idx, dense group id g).  key =
// (g << wr) | rank[idx + h]; rank is the group-head position + 1 (0 = past
// the end), so sorting by key refines every group by its next h symbols.
//
// kSparse: after a first round that left few suffixes unsorted, rank[] is
// only maintained for those (flagged in `member`); the rank of any other
// position j is its round-1 group head, found by a binary search of its
// packed K-symbol key in the round-1 sorted keys (a singleton's head is its
// own SA position).  This avoids a random scatter of all n ranks.
struct RankLookup {
    const uint32_t* __restrict__ rank;
    const uint32_t* __restrict__ member;   // bitmap of round-1 unsorted positions
    const uint64_t* __restrict__ keys1;    // round-1 sorted packed keys (n)
    const uint8_t* __restrict__ text;
    const uint16_t* __restrict__ code;
    uint64_t n;
    uint64_t base;
    uint32_t K;
    uint32_t bucketed;                     // 1: keys1 holds key1 (BucketSpec layout)
    BucketSpec bs;
    const uint32_t* __restrict__ bstart;   // bucketed: bucket start positions (2^bb + 1), or null
    const uint32_t* __restrict__ sa;       // bucketed: the SA (key1 of the sampled-out slots)
    uint32_t ksh;                          // bucketed: keys1 holds every 2^ksh-th key1
    __device__ __forceinline__ uint32_t sparse(uint64_t j) const {
        if ((member[j >> 5] >> (j & 31)) & 1u) return rank[j];
        uint64_t x = 0;
        uint64_t lo = 0, len = n;      // lower_bound(keys1, x), inside x's bucket when known
        if (bucketed) {
            const CodeMap map{code};
            uint32_t D;
            x = key1_words<true>(text, n, map, bs, j, &D);
            if (bstart) {
                const uint32_t b = (uint32_t)(((uint64_t)D * bs.cmul) >> bs.bsh);
                lo = bstart[b];
                len = bstart[b + 1] - lo;
            }
            auto key_at = [&](uint64_t p) {
                uint32_t d;
                return key1_words<true>(text, n, map, bs, p, &d);
            };
            return (uint32_t)lower_bound_sampled(keys1, ksh, sa, lo, lo + len, x, key_at) + 1u;
        } else {
            for (uint32_t t = 0; t < K; ++t) x = x * base + ((j + t < n) ? code[text[j + t]] : 0u);
        }
        while (len > 0) {
            const uint64_t half = len >> 1;
            if (keys1[lo + half] < x) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        return (uint32_t)lo + 1u;
    }
};

template <bool kSparse>
struct SrcU {
    const uint32_t* __restrict__ u_idx;
    const uint32_t* __restrict__ u_g;
    RankLookup rl;
    uint64_t h;
    uint32_t wr;
    __device__ __forceinline__ uint64_t key(uint64_t e) const {
        const uint64_t i = u_idx[e];
        uint64_t r1 = 0;
        if (i + h < rl.n) r1 = kSparse ? rl.sparse(i + h) : rl.rank[i + h];
        return ((uint64_t)u_g[e] << wr) | r1;
    }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return u_idx[e]; }
};

// The first unsorted-set round after a bucketed round 1 (h = K, sparse
// ranks): rank[x + K] is the round-1 rank of suffix x + K, and round 1 sorted
// every suffix by its K-symbol key1 -- equal key1 <=> one round-1 group <=>
// equal rank, and key1 order = rank order.  So key1(x + K) + 1 (0 past the
// end), rebuilt from the text (a few independent word loads), orders and
// ties the members exactly as rank[x + K] does, without the sample search of
// the SA that RankLookup::sparse needs for a suffix outside the unsorted set.
// kb: bits of key1 + 1 (the host checks kb + bits of the group ids <= 64).
struct SrcUKey1 {
    const uint32_t* __restrict__ u_idx;
    const uint32_t* __restrict__ u_g;
    RankLookup rl;
    uint64_t h;
    uint32_t kb;
    __device__ __forceinline__ uint64_t key(uint64_t e) const {
        const uint64_t i = u_idx[e];
        uint64_t r1 = 0;
        if (i + h < rl.n) {
            uint32_t D;
            r1 = key1_words<true>(rl.text, rl.n, CodeMap{rl.code}, rl.bs, i + h, &D) + 1u;
        }
        return ((uint64_t)u_g[e] << kb) | r1;
    }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return u_idx[e]; }
};

// The key1 samples of the sorted round-1 suffixes (every 2^ksh-th SA
// position; RankLookup::sparse searches them), rebuilt from the SA and the
// text when k_bucket_sort did not write them (SegOut::samples = 0).  Round 2
// reorders only inside round-1 groups, whose members share key1, so the
// samples are the same after it.
__global__ __launch_bounds__(kBlock) void k_key1_samples(const uint8_t* __restrict__ text, uint64_t n,
                                                         const uint16_t* __restrict__ code, BucketSpec bs,
                                                         const uint32_t* __restrict__ sa, uint32_t ksh,
                                                         uint64_t* __restrict__ keys1) {
    const uint64_t ns = (n + (1ull << ksh) - 1) >> ksh;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < ns; t += (uint64_t)gridDim.x * kBlock) {
        uint32_t D;
        keys1[t] = key1_words<true>(text, n, CodeMap{code}, bs, sa[t << ksh], &D);
    }
}

// An unsorted-set round whose groups are all small (most are pairs on
// random text): each group -- a run of equal u_g, contiguous in SA order --
// is sorted by its keys (g, rank[i + h]) in registers by the lane at its
// first member, instead of a full LSD radix sort of the set.  Groups larger
// than kUsLimit set *flag and are left unwritten (the caller then runs the
// radix sort).  Equal keys may come out in any order: the round only needs
// the classes of equal keys and their order, later rounds re-sort ties.
constexpr int kUsLimit = 8;

__device__ __forceinline__ void us_cx(uint64_t& ka, uint32_t& va, uint64_t& kb, uint32_t& vb) {
    if (kb < ka) {
        const uint64_t tk = ka;
        ka = kb;
        kb = tk;
        const uint32_t tv = va;
        va = vb;
        vb = tv;
    }
}

template <class Src>
__global__ __launch_bounds__(kBlock) void k_usort_small(Src src, const uint32_t* __restrict__ u_g, uint64_t m,
                                                        uint64_t* __restrict__ out_keys,
                                                        uint32_t* __restrict__ out_vals, uint32_t* __restrict__ flag) {
    for (uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x; s < m; s += (uint64_t)gridDim.x * kBlock) {
        const uint32_t g = u_g[s];
        if (s > 0 && u_g[s - 1] == g) continue;
        uint32_t len = 1;
        while (len <= kUsLimit && s + len < m && u_g[s + len] == g) ++len;
        if (len > kUsLimit) {
            atomicOr(flag, 1u);
            continue;
        }
        uint64_t k[kUsLimit];
        uint32_t v[kUsLimit];
#pragma unroll
        for (int j = 0; j < kUsLimit; ++j) {
            k[j] = ~0ull;
            v[j] = 0;
            if ((uint32_t)j < len) {
                k[j] = src.key(s + j);
                v[j] = src.val(s + j);
            }
        }
        // Batcher odd-even merge sort of 8 (19 compare-exchanges)
        us_cx(k[0], v[0], k[1], v[1]); us_cx(k[2], v[2], k[3], v[3]);
        us_cx(k[4], v[4], k[5], v[5]); us_cx(k[6], v[6], k[7], v[7]);
        us_cx(k[0], v[0], k[2], v[2]); us_cx(k[1], v[1], k[3], v[3]);
        us_cx(k[4], v[4], k[6], v[6]); us_cx(k[5], v[5], k[7], v[7]);
        us_cx(k[1], v[1], k[2], v[2]); us_cx(k[5], v[5], k[6], v[6]);
        us_cx(k[0], v[0], k[4], v[4]); us_cx(k[1], v[1], k[5], v[5]);
        us_cx(k[2], v[2], k[6], v[6]); us_cx(k[3], v[3], k[7], v[7]);
        us_cx(k[2], v[2], k[4], v[4]); us_cx(k[3], v[3], k[5], v[5]);
        us_cx(k[1], v[1], k[2], v[2]); us_cx(k[3], v[3], k[4], v[4]);
        us_cx(k[5], v[5], k[6], v[6]);
#pragma unroll
        for (int j = 0; j < kUsLimit; ++j) {
            if ((uint32_t)j < len) {
                out_keys[s + j] = k[j];
                out_vals[s + j] = v[j];
            }
        }
    }
}

// The keys of an unsorted-set round, one lane per suffix (each a sparse rank
// look-up: a chain of dependent loads), for k_usort_small to read: the
// group's first lane no longer walks its members' look-ups one after another.
template <class Src>
__global__ __launch_bounds__(kBlock) void k_usort_keys(Src src, uint64_t m, uint64_t* __restrict__ out_keys) {
    for (uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x; s < m; s += (uint64_t)gridDim.x * kBlock)
        out_keys[s] = src.key(s);
}

// Later passes: the previous pass's output.
struct SrcKeys {
    const uint64_t* __restrict__ keys;
    const uint32_t* __restrict__ vals;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return keys[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return vals[e]; }
};

// Keys already materialised in text order (k_pack_text), index = position.
struct SrcKeysIota {
    const uint64_t* __restrict__ keys;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return keys[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return (uint32_t)e; }
};

// Radix digit of a key, bits [shift, shift + nbits): a source may define
// digit() (the bucketed first round sorts by a function of the key, see
// sa_bucket.h); otherwise the digit is the key's own bits.
template <class S>
__device__ __forceinline__ auto src_digit(const S& s, uint64_t k, uint32_t shift, uint32_t mask, int)
    -> decltype(s.digit(k, shift, mask)) {
    return s.digit(k, shift, mask);
}
template <class S>
__device__ __forceinline__ uint32_t src_digit(const S&, uint64_t k, uint32_t shift, uint32_t mask, long) {
    return (uint32_t)(k >> shift) & mask;
}

struct Chunking {
    uint64_t n;
    uint32_t tiles_per_chunk;
    uint32_t chunks;
    __device__ __forceinline__ uint64_t begin(uint32_t c) const {
        const uint64_t b = (uint64_t)c * tiles_per_chunk * kTile;
        return b < n ? b : n;
    }
    __device__ __forceinline__ uint64_t end(uint32_t c) const {
        const uint64_t e = ((uint64_t)c + 1) * tiles_per_chunk * kTile;
        return e < n ? e : n;
    }
};

// ---------------------------------------------------------------------------
// scans
// ---------------------------------------------------------------------------
// Inclusive sum over the wave by DPP: row_shr 1 / 2 / 4 / 8 inside each
// 16-lane row, then row_bcast 15 / 31 across rows (lanes without a source
// add 0).  The __shfl_up form took six ds_bpermute lane addresses and six
// lane masks that the compiler hoisted out of the kernels' loops: in the
// first bucket pass and the LSD passes they spilled to scratch, and each
// reload waited for every store in flight.
#ifndef SA_DPP_SCAN
#define SA_DPP_SCAN 1
#endif
// row_bcast:15 / :31 exist on the wave64 GFX9 family only (gfx950 is one);
// the library is built for gfx950 alone, so another target is an error here
// rather than a silently wrong scan.
#if SA_DPP_SCAN && defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "wave_inclusive_sum: DPP row_bcast needs a GFX9-family target (build with -DSA_DPP_SCAN=0 otherwise)"
#endif
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t x) {
#if SA_DPP_SCAN
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
#else
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, kWave);
        if ((int)lane_id() >= o) x += y;
    }
    return x;
#endif
}

// exclusive sum over the 256 threads of the block; s_tmp holds kWaves words.
__device__ __forceinline__ uint32_t block_exclusive_sum(uint32_t x, uint32_t* s_tmp, uint32_t* total) {
    const uint32_t inc = wave_inclusive_sum(x);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t v = s_tmp[w];
        off += (w < (int)wave_id()) ? v : 0u;
        tot += v;
    }
    __syncthreads();
    if (total) *total = tot;
    return off + inc - x;
}

// ---------------------------------------------------------------------------
// init: rank_1[i] = text[i] + 1 (manber_myers.c:88-92; unsigned bytes, the
// +1 keeps 0 free for the end-of-string sentinel, as get_rank_val :10-12)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_init_rank(const uint8_t* __restrict__ text, uint64_t n,
                                                      uint32_t* __restrict__ rank) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 4 <= n && (((uintptr_t)(text + i)) & 3) == 0) {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(text + i);
            uint4 r;
            r.x = (v & 0xFFu) + 1u;
            r.y = ((v >> 8) & 0xFFu) + 1u;
            r.z = ((v >> 16) & 0xFFu) + 1u;
            r.w = (v >> 24) + 1u;
            *reinterpret_cast<uint4*>(rank + i) = r;
        } else {
            for (uint64_t j = i; j < n && j < i + 4; ++j) rank[j] = (uint32_t)text[j] + 1u;
        }
    }
}

// The reference schedule's first ranks as DENSE codes (code[byte] = 1..sigma
// in byte order, 0 = past the end): the same order as text[i] + 1, so every
// round's D_j and the round count are the reference's, but the first
// round's key spans 2 bit_width(sigma) bits instead of 18 (DNA: one radix
// pass of 6 bits instead of three of 8).
__global__ __launch_bounds__(kBlock) void k_init_rank_dense(const uint8_t* __restrict__ text, uint64_t n,
                                                            const uint16_t* __restrict__ code,
                                                            uint32_t* __restrict__ rank) {
    __shared__ uint16_t s_code[256];
    s_code[threadIdx.x] = code[threadIdx.x];
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 4 <= n && (((uintptr_t)(text + i)) & 3) == 0) {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(text + i);
            uint4 r;
            r.x = s_code[v & 0xFFu];
            r.y = s_code[(v >> 8) & 0xFFu];
            r.z = s_code[(v >> 16) & 0xFFu];
            r.w = s_code[v >> 24];
            *reinterpret_cast<uint4*>(rank + i) = r;
        } else {
            for (uint64_t j = i; j < n && j < i + 4; ++j) rank[j] = s_code[text[j]];
        }
    }
}

// ---------------------------------------------------------------------------
// radix upsweep: per-(digit, chunk) counts.  Per-wave LDS histograms keep the
// LDS atomics of different waves apart (counting_sort_radix_seq :19-21).
// ---------------------------------------------------------------------------
template <class Src>
__global__ __launch_bounds__(kBlock) void k_hist(Src src, Chunking ch, uint32_t shift, uint32_t mask,
                                                 uint32_t* __restrict__ hist) {
    __shared__ uint32_t s_hist[kWaves][kRadix];
    for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    uint32_t* my = s_hist[wave_id()];
    for (uint64_t base = e0; base < e1; base += kTile) {
        uint32_t d[kItems];
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t e = base + (uint64_t)j * kBlock + threadIdx.x;
            d[j] = (e < e1) ? (uint32_t)(src.key(e) >> shift) & mask : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int j = 0; j < kItems; ++j)
            if (d[j] != 0xFFFFFFFFu) atomicAdd(&my[d[j]], 1u);
    }
    __syncthreads();
    const int dgt = threadIdx.x;   // kBlock == kRadix
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += s_hist[w][dgt];
    hist[(uint64_t)dgt * ch.chunks + c] = s;
}

// ---------------------------------------------------------------------------
// scan of one digit row of hist (C chunk counts) in place; totals[d] = sum.
// One workgroup per digit (counting_sort_radix_seq prefix step :23-25).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_scan_rows(uint32_t* __restrict__ hist, uint32_t chunks,
                                                      uint32_t* __restrict__ totals) {
    __shared__ uint32_t s_tmp[kWaves];
    uint32_t* row = hist + (uint64_t)blockIdx.x * chunks;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < chunks; base += kBlock * 4) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = base + threadIdx.x * 4 + j;
            v[j] = (i < chunks) ? row[i] : 0u;
            sum += v[j];
        }
        uint32_t tot;
        uint32_t off = block_exclusive_sum(sum, s_tmp, &tot) + carry;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = base + threadIdx.x * 4 + j;
            if (i < chunks) row[i] = off;
            off += v[j];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// ---------------------------------------------------------------------------
// radix downsweep: stable scatter of one 8-bit digit.
//  1. each wave ranks its 1024 keys in order (j-major, lane-minor) with a
//     match-any built from `nbits` ballots; a per-wave LDS counter per digit
//  2. per-digit wave prefixes + block exclusive scan give the tile layout
//  3. keys/vals are placed digit-sorted in LDS, then written so that
//     consecutive lanes write consecutive addresses of one digit run
// (counting_sort_radix_seq scatter :27-31, which is stable by scanning
// backwards; here stability comes from ranking in input order.)
// ---------------------------------------------------------------------------
template <class Src>
__global__ __launch_bounds__(kBlock) void k_scatter(Src src, Chunking ch, uint32_t shift, uint32_t nbits,
                                                    const uint32_t* __restrict__ hist,
                                                    const uint32_t* __restrict__ totals,
                                                    uint64_t* __restrict__ out_keys,
                                                    uint32_t* __restrict__ out_vals) {
    __shared__ uint64_t s_keys[kTile];
    __shared__ uint32_t s_vals[kTile];
    __shared__ uint32_t s_wcnt[kWaves][kRadix];
    __shared__ uint32_t s_start[kRadix];
    __shared__ uint32_t s_run[kRadix];
    __shared__ uint32_t s_tmp[kWaves];

    const uint32_t mask = (1u << nbits) - 1u;
    const uint32_t c = blockIdx.x;
    const uint32_t dgt = threadIdx.x;     // this thread's digit in per-digit phases
    const uint32_t wave = wave_id(), lane = lane_id();
    {
        const uint32_t base = block_exclusive_sum(totals[dgt], s_tmp, nullptr);
        s_run[dgt] = base + hist[(uint64_t)dgt * ch.chunks + c];
    }
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint32_t valid = (uint32_t)((e1 - tb) < (uint64_t)kTile ? (e1 - tb) : (uint64_t)kTile);
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s_wcnt[w][dgt] = 0;
        __syncthreads();

        uint64_t k[kItems];
        uint32_t v[kItems];
        uint32_t d[kItems];
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint32_t le = wave * kWaveTile + j * kWave + lane;
            const bool ok = le < valid;
            k[j] = ok ? src.key(tb + le) : 0ull;
            v[j] = ok ? src.val(tb + le) : 0u;
            d[j] = ok ? (uint32_t)(k[j] >> shift) & mask : kRadix;
        }
        uint32_t r[kItems];
        uint32_t* wc = s_wcnt[wave];
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const bool ok = d[j] < (uint32_t)kRadix;
            uint64_t peers = __ballot(ok);
            for (uint32_t b = 0; b < nbits; ++b) {
                const bool bit = (d[j] >> b) & 1u;
                const uint64_t bal = __ballot(bit);
                peers &= bit ? bal : ~bal;
            }
            uint32_t cnt = 0;
            if (ok) cnt = wc[d[j]];
            const uint32_t below = (uint32_t)__popcll(peers & lanemask_lt());
            r[j] = cnt + below;
            if (ok && below == 0) wc[d[j]] = cnt + (uint32_t)__popcll(peers);
        }
        __syncthreads();
        // per digit: prefix over waves, then block scan over digits
        uint32_t tile_cnt = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t x = s_wcnt[w][dgt];
            s_wcnt[w][dgt] = tile_cnt;
            tile_cnt += x;
        }
        const uint32_t start = block_exclusive_sum(tile_cnt, s_tmp, nullptr);
        s_start[dgt] = start;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            if (d[j] < (uint32_t)kRadix) {
                const uint32_t pos = s_start[d[j]] + s_wcnt[wave][d[j]] + r[j];
                s_keys[pos] = k[j];
                s_vals[pos] = v[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint32_t q = j * kBlock + threadIdx.x;
            if (q < valid) {
                const uint64_t key = s_keys[q];
                const uint32_t dd = (uint32_t)(key >> shift) & mask;
                const uint64_t g = (uint64_t)s_run[dd] + (q - s_start[dd]);
                if (g < ch.n) {   // always true for consistent offsets; never fault
                    out_keys[g] = key;
                    out_vals[g] = s_vals[q];
                }
            }
        }
        __syncthreads();
        s_run[dgt] += tile_cnt;
        // the next tile's first __syncthreads orders this update before use
    }
}

// ---------------------------------------------------------------------------
// re-rank (manber_myers.c:101-110): head flag = key differs from its
// predecessor in sorted order; dense rank = inclusive count of heads.
// Each wave owns a contiguous 1024-key slice of the tile: rows of 64 keys,
// ballot + popcount give the in-row prefix.
// ---------------------------------------------------------------------------
// kshift: the key is the word's bits above kshift (packed (key, idx) items of
// the reference schedule, sa_onesweep.h k_lsd; 0 otherwise); key_out is the
// whole word, prev_last the previous row's last KEY.
__device__ __forceinline__ uint64_t wave_heads(const uint64_t* __restrict__ keys, uint64_t row0,
                                               uint64_t lim, uint64_t& prev_last, uint64_t& key_out,
                                               bool& ok_out, uint32_t kshift = 0) {
    const uint64_t e = row0 + lane_id();
    const bool ok = e < lim;
    const uint64_t word = ok ? keys[e] : 0ull;
    const uint64_t key = word >> kshift;
    uint64_t prev = __shfl_up(key, 1, kWave);
    if (lane_id() == 0) prev = prev_last;
    prev_last = __shfl(key, kWave - 1, kWave);
    const bool head = ok && (e == 0 || key != prev);
    key_out = word;
    ok_out = ok;
    return __ballot(head);
}

__global__ __launch_bounds__(kBlock) void k_heads(const uint64_t* __restrict__ keys, Chunking ch,
                                                  uint32_t* __restrict__ counts, uint32_t kshift = 0) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    uint32_t cnt = 0;
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint64_t w0 = tb + (uint64_t)wave_id() * kWaveTile;
        uint64_t prev_last = (w0 > 0 && w0 < e1) ? keys[w0 - 1] >> kshift : 0ull;
#pragma unroll 4
        for (int j = 0; j < kItems; ++j) {
            uint64_t key;
            bool ok;
            const uint64_t m = wave_heads(keys, w0 + (uint64_t)j * kWave, e1, prev_last, key, ok, kshift);
            cnt += (uint32_t)__popcll(m);
        }
    }
    // every lane holds the wave count; combine waves
    uint32_t tot;
    block_exclusive_sum(lane_id() == 0 ? cnt : 0u, s_tmp, &tot);
    if (threadIdx.x == 0) counts[c] = tot;
}

// exclusive scan of the C chunk head counts (one workgroup); *d_total = D.
__global__ __launch_bounds__(kBlock) void k_scan_heads(uint32_t* __restrict__ counts, uint32_t chunks,
                                                       uint32_t* __restrict__ d_total) {
    __shared__ uint32_t s_tmp[kWaves];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < chunks; base += kBlock * 4) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = base + threadIdx.x * 4 + j;
            v[j] = (i < chunks) ? counts[i] : 0u;
            sum += v[j];
        }
        uint32_t tot;
        uint32_t off = block_exclusive_sum(sum, s_tmp, &tot) + carry;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = base + threadIdx.x * 4 + j;
            if (i < chunks) counts[i] = off;
            off += v[j];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *d_total = carry;
}

// rank[idx[p]] = heads(0..p) for every sorted position p.
__global__ __launch_bounds__(kBlock) void k_rerank(const uint64_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ idx, Chunking ch,
                                                   const uint32_t* __restrict__ chunk_off,
                                                   uint32_t* __restrict__ rank) {
    __shared__ uint32_t s_wtot[kWaves];
    __shared__ uint32_t s_tmp[kWaves];
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    uint32_t run = chunk_off[c];
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint64_t w0 = tb + (uint64_t)wave_id() * kWaveTile;
        uint64_t prev_last = (w0 > 0 && w0 < e1) ? keys[w0 - 1] : 0ull;
        uint64_t m[kItems];
        uint32_t wsum = 0;
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            uint64_t key;
            bool ok;
            m[j] = wave_heads(keys, w0 + (uint64_t)j * kWave, e1, prev_last, key, ok);
            wsum += (uint32_t)__popcll(m[j]);
        }
        if (lane_id() == 0) s_wtot[wave_id()] = wsum;
        __syncthreads();
        uint32_t woff = run, ttot = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t x = s_wtot[w];
            woff += (w < (int)wave_id()) ? x : 0u;
            ttot += x;
        }
        __syncthreads();
        const uint64_t le_mask = lanemask_lt() | (1ull << lane_id());
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t e = w0 + (uint64_t)j * kWave + lane_id();
            if (e < e1) {
                const uint32_t x = idx[e];
                if (x < ch.n) rank[x] = woff + (uint32_t)__popcll(m[j] & le_mask);
            }
            woff += (uint32_t)__popcll(m[j]);
        }
        run += ttot;
    }
    (void)s_tmp;
}


// ---------------------------------------------------------------------------
// alphabet presence: bit b of present[b >> 5] is set when byte b occurs.
// Presence is all the dense codes need; it is kept in 8 registers per lane
// (no LDS atomics, so a 4-symbol text costs no bank conflicts), OR-reduced
// over the wave, one atomicOr per word per wave.
// (one LDS atomic per 16-byte chunk inside one 32-symbol block instead of 16
// measured equal at 1 GiB DNA in r02, profiles/r02_bd_ab_alpha_fast.txt; in
// r05 0.255-0.263 -> 0.235-0.243 ms, profiles/r05_am_ab_alpha_chunk_*.txt;
// two chunks per lane in flight instead of one made no further difference)
__global__ __launch_bounds__(kBlock) void k_alphabet(const uint8_t* __restrict__ text, uint64_t n,
                                                     uint32_t* __restrict__ present) {
    // a private 256-bit mask per lane in LDS, set by one atomic OR per byte
    // (no return value; a stride of 9 words keeps 32 lanes on 32 banks) --
    // selecting the mask word in registers cost 8 compares per byte
    __shared__ uint32_t s_m[kBlock * 9];
    uint32_t* m = s_m + threadIdx.x * 9;
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = 0;
    auto add = [&](uint32_t b) { atomicOr(&m[b >> 5], 1u << (b & 31u)); };
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * 16;
    // 16-byte chunks, the next one in flight while this one is added (the
    // loop waited on each load: 1 GiB in 0.29 ms, 3.7 TB/s); chunks that
    // are not whole and aligned go byte by byte
    auto whole = [&](uint64_t i) { return i + 16 <= n && (((uintptr_t)(text + i)) & 15) == 0; };
    uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 16;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (i < n && whole(i)) v = *reinterpret_cast<const uint4*>(text + i);
    // a wave whose lanes together have seen all 256 byte values stops
    // reading (presence cannot grow further): checked after steps 1, 2, 4,
    // 8, ... so a text with fewer values (DNA) pays a few checks per wave;
    // byte256 text reads ~1 KiB per wave instead of its whole share
    uint32_t step = 0;
    for (; i < n; i += stride) {
        if (step && (step & (step - 1)) == 0) {   // uniform
            uint32_t all = ~0u;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                uint32_t x = m[q];
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) x |= __shfl_xor(x, o, kWave);
                all &= x;
            }
            if (all == ~0u) break;
        }
        ++step;
        const uint64_t in = i + stride;
        uint4 vn = make_uint4(0u, 0u, 0u, 0u);
        if (in < n && whole(in)) vn = *reinterpret_cast<const uint4*>(text + in);
        if (whole(i)) {
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
            // the 16 bytes in one 32-value word of the mask (DNA, one case of
            // letters: every chunk): their bits OR-ed in registers, one LDS
            // atomic per chunk instead of one per byte
            uint32_t o = v.x | v.y | v.z | v.w, a = v.x & v.y & v.z & v.w;
            o |= o >> 16;
            o |= o >> 8;
            a &= a >> 16;
            a &= a >> 8;
            if (((o ^ a) & 0xE0u) == 0u) {
                uint32_t bits = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int b = 0; b < 4; ++b) bits |= 1u << ((w4[q] >> (8 * b)) & 31u);
                atomicOr(&m[(o & 0xFFu) >> 5], bits);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int b = 0; b < 4; ++b) add((w4[q] >> (8 * b)) & 0xFFu);
            }
        } else {
            for (uint64_t j = i; j < n && j < i + 16; ++j) add(text[j]);
        }
        v = vn;
    }
    // one global atomic per word and workgroup, and none for bits already
    // set there (8 same-address atomics per wave serialised in the L2: 0.4 ms
    // of byte256's alphabet pass once its waves stopped early)
    __shared__ uint32_t s_or[8];
    if (threadIdx.x < 8) s_or[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t x = m[i];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x |= __shfl_xor(x, o, kWave);
        if (lane_id() == 0 && x) atomicOr(&s_or[i], x);
    }
    __syncthreads();
    if (threadIdx.x < 8) {
        const uint32_t x = s_or[threadIdx.x];
        if (x & ~__hip_atomic_load(&present[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicOr(&present[threadIdx.x], x);
    }
}

// ---------------------------------------------------------------------------
// packed schedule, round 1 key build: key(i) = sum_t code(i+t) B^(K-1-t),
// t < K.  One tile of codes (+ K-1 halo) is staged in LDS; each lane builds
// 16 consecutive keys, the first by Horner, the rest by the rolling update
// key' = (key - c_out B^(K-1)) B + c_in.  Histograms are taken here too:
// with passes == 0 the digit-0 histogram per chunk (reduce-then-scan sort,
// same chunking as k_hist); with passes > 0 the global histograms of all
// passes' digits (single-pass sort, ghist[passes][256]).
// ---------------------------------------------------------------------------
// Adds one wave's keys to LDS digit histograms, one atomic per run of equal
// digits across neighbouring lanes (as hist_add_runs, sa_onesweep.h), for a
// wave whose lanes may hold no key (valid false); called by every lane of
// the wave: invalid lanes form runs of their own that add nothing.  Passes
// [p_lo, p_hi) are counted, pass p into histogram row row0 + p.
__device__ __forceinline__ void hist_add_runs_valid(uint32_t (*s_h)[kRadix], uint64_t k, bool valid, uint32_t p_lo,
                                                    uint32_t p_hi, uint32_t row0) {
    const uint32_t lane = lane_id();
    const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    for (uint32_t p = p_lo; p < p_hi; ++p) {
        const uint32_t d = valid ? ((uint32_t)(k >> (8 * p)) & 0xFFu) : 0x100u;
        const uint32_t dl = __shfl_up(d, 1, 64);
        const bool head = lane == 0 || dl != d;
        const uint64_t hm = __ballot(head) & above;
        const uint32_t next = hm ? (uint32_t)__ffsll((long long)hm) - 1u : 64u;
        if (head && valid) atomicAdd(&s_h[row0 + p][d], next - lane);
    }
}

constexpr int kPackRun = kTile / kBlock;   // 16 consecutive keys per lane
constexpr int kMaxK = 64;
constexpr int kPackMaxPasses = 8;

// text points at the first position keyed (lo); `avail` bytes are readable
// from there (n - lo); ch.n keys are produced.
__global__ __launch_bounds__(kBlock) void k_pack_text(const uint8_t* __restrict__ text, uint64_t avail,
                                                      const uint16_t* __restrict__ code, Chunking ch,
                                                      uint64_t base, uint64_t top, uint32_t K,
                                                      uint64_t* __restrict__ keys, uint32_t* __restrict__ hist,
                                                      uint32_t passes, uint32_t* __restrict__ ghist) {
    __shared__ uint16_t s_code[256];
    __shared__ uint16_t s_c[kTile + kMaxK];
    __shared__ uint32_t s_hist[kPackMaxPasses][kRadix];
    // keys staged for a coalesced store; one u64 of padding per 16 keys keeps
    // the lane-strided writes (16 keys apart) off a single LDS bank
    __shared__ uint64_t s_k[kTile + kTile / kPackRun];
    s_code[threadIdx.x] = code[threadIdx.x];
    for (int i = threadIdx.x; i < kPackMaxPasses * kRadix; i += kBlock) (&s_hist[0][0])[i] = 0;
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    const uint64_t n = avail;
    // one LDS atomic per run of equal digits across neighbouring lanes (every
    // lane calls it): a degenerate text's keys are all equal, and one atomic
    // per lane and pass put 64 lanes on one bin (29.7 of round 1's 103 ms at
    // 1 GiB a x 2^30)
    auto count = [&](uint64_t key, bool valid) {
        if (passes == 0) hist_add_runs_valid(s_hist, key, valid, 0, 1, wave_id());
        else hist_add_runs_valid(s_hist, key, valid, 0, passes, 0);
    };
    __syncthreads();
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        {   // 16 text bytes per lane (one dwordx4), then the K-1 halo
            const uint64_t i = tb + (uint64_t)threadIdx.x * 16;
            uint16_t* dst = s_c + threadIdx.x * 16;
            if (i + 16 <= n && (((uintptr_t)(text + i)) & 15) == 0) {
                const uint4 v = *reinterpret_cast<const uint4*>(text + i);
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int b = 0; b < 4; ++b) dst[4 * q + b] = s_code[(w4[q] >> (8 * b)) & 0xFFu];
            } else {
                for (int q = 0; q < 16; ++q) dst[q] = (i + q < n) ? s_code[text[i + q]] : (uint16_t)0;
            }
            if (threadIdx.x < K) {
                const uint64_t h = tb + kTile + threadIdx.x;
                s_c[kTile + threadIdx.x] = (h < n) ? s_code[text[h]] : (uint16_t)0;
            }
        }
        __syncthreads();
        const uint32_t l0 = threadIdx.x * kPackRun;
        uint64_t x = 0;
        for (uint32_t t = 0; t < K; ++t) x = x * base + s_c[l0 + t];
        uint64_t* kd = s_k + threadIdx.x * (kPackRun + 1);
        kd[0] = x;
        count(x, tb + l0 < e1);
#pragma unroll
        for (int j = 1; j < kPackRun; ++j) {
            x = (x - (uint64_t)s_c[l0 + j - 1] * top) * base + s_c[l0 + j - 1 + K];
            kd[j] = x;
            count(x, tb + l0 + j < e1);
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kPackRun; ++j) {
            const uint32_t q = j * kBlock + threadIdx.x;
            const uint64_t g = tb + q;
            if (g < e1) keys[g] = s_k[q + q / kPackRun];
        }
        __syncthreads();
    }
    if (passes == 0) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += s_hist[w][threadIdx.x];
        if (hist) hist[(uint64_t)threadIdx.x * ch.chunks + c] = s;
    } else {
        for (uint32_t p = 0; p < passes; ++p) {
            const uint32_t v = s_hist[p][threadIdx.x];
            if (v) atomicAdd(&ghist[p * kRadix + threadIdx.x], v);
        }
    }
}

// ---------------------------------------------------------------------------
// Segments of a sorted key sequence s = 0..m-1 (packed schedule).
//   head(s)   key[s] != key[s-1]               (manber_myers.c:104-105)
//   single(s) head(s) and head(s+1)            (group of size 1: final)
//   inU(s)    !single(s)                       (still unsorted)
//   uhead(s)  head(s) and inU(s)               (first member of an unsorted group)
// pos(s) maps a sorted index to its SA position: identity in the first round,
// the compacted position array in later rounds.
// ---------------------------------------------------------------------------
struct PosIdentity {
    __device__ __forceinline__ uint32_t operator()(uint64_t s) const { return (uint32_t)s; }
};
struct PosArray {
    const uint32_t* __restrict__ p;
    __device__ __forceinline__ uint32_t operator()(uint64_t s) const { return p[s]; }
};
// the pivot round 1's sorted rest (sa_pivot.h): t0 keys below the pivot at
// 0..t0-1, then a gap of t1 tied suffixes, then the keys above it
struct PosGap {
    uint64_t t0, t1;
    __device__ __forceinline__ uint32_t operator()(uint64_t s) const { return (uint32_t)(s < t0 ? s : s + t1); }
};

// Keys of one wave's 16 rows of 64 (s = w0 + 64 j + lane), all loads issued
// before any is used; lane 0 / 63 also fetch the key before / after its row.
struct SegRows {
    uint64_t k[kItems], lo[kItems];
    __device__ __forceinline__ void load(const uint64_t* __restrict__ keys, uint64_t w0, uint64_t m) {
        const uint32_t lane = lane_id();
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t s = w0 + (uint64_t)j * kWave + lane;
            k[j] = s < m ? keys[s] : ~0ull;
            const uint64_t nb = lane == 0 ? s - 1 : s + 1;   // lanes 1..62 load nothing extra
            const bool edge = (lane == 0 && s > 0 && s - 1 < m) || (lane == kWave - 1 && s + 1 < m);
            lo[j] = edge ? keys[nb] : 0ull;
        }
    }
};

__device__ __forceinline__ void seg_masks_reg(uint64_t k, uint64_t edge, uint64_t s, uint64_t m, uint64_t& mf,
                                              uint64_t& mu, uint64_t& muh) {
    const uint32_t lane = lane_id();
    uint64_t prev = __shfl_up(k, 1, kWave);
    uint64_t next = __shfl_down(k, 1, kWave);
    if (lane == 0) prev = edge;
    if (lane == kWave - 1) next = edge;
    bool f = false, u = false;
    if (s < m) {
        f = (s == 0) || prev != k;
        const bool nf = (s + 1 >= m) || next != k;
        u = !(f && nf);
    }
    mf = __ballot(f);
    mu = __ballot(u);
    muh = __ballot(f && u);
}

// one row of 64 consecutive sorted keys starting at rb (s = rb + lane); the
// neighbours come from the adjacent lanes, only lanes 0 / 63 load one more key
__device__ __forceinline__ void seg_masks(const uint64_t* __restrict__ keys, uint64_t s, uint64_t m,
                                          uint64_t& mf, uint64_t& mu, uint64_t& muh) {
    const uint32_t lane = lane_id();
    const uint64_t k = s < m ? keys[s] : ~0ull;
    uint64_t prev = __shfl_up(k, 1, kWave);
    uint64_t next = __shfl_down(k, 1, kWave);
    if (lane == 0) prev = (s > 0 && s - 1 < m) ? keys[s - 1] : ~k;
    if (lane == kWave - 1) next = (s + 1 < m) ? keys[s + 1] : ~k;
    bool f = false, u = false;
    if (s < m) {
        f = (s == 0) || prev != k;
        const bool nf = (s + 1 >= m) || next != k;
        u = !(f && nf);
    }
    mf = __ballot(f);
    mu = __ballot(u);
    muh = __ballot(f && u);
}

// per chunk: number of heads, unsorted members, unsorted groups, and
// (last head index + 1) or 0.
__global__ __launch_bounds__(kBlock) void k_seg_count(const uint64_t* __restrict__ keys, Chunking ch,
                                                      uint32_t* __restrict__ c_heads, uint32_t* __restrict__ c_u,
                                                      uint32_t* __restrict__ c_uh, uint32_t* __restrict__ c_last) {
    __shared__ uint32_t s_v[4][kWaves];
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    uint32_t nh = 0, nu = 0, nuh = 0, last = 0;
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint64_t w0 = tb + (uint64_t)wave_id() * kWaveTile;
        SegRows rows;
        rows.load(keys, w0, ch.n);
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t rb = w0 + (uint64_t)j * kWave;
            uint64_t mf, mu, muh;
            // neighbours are compared across chunk borders (global m = ch.n);
            // lanes past the chunk end are counted by the next chunk
            seg_masks_reg(rows.k[j], rows.lo[j], rb + lane_id(), ch.n, mf, mu, muh);
            if (rb >= e1) continue;
            const uint64_t lim = e1 - rb >= 64 ? ~0ull : ((1ull << (e1 - rb)) - 1ull);
            mf &= lim;
            mu &= lim;
            muh &= lim;
            nh += __popcll(mf);
            nu += __popcll(mu);
            nuh += __popcll(muh);
            if (mf) last = (uint32_t)(rb + 63 - __clzll(mf)) + 1u;
        }
    }
    if (lane_id() == 0) {
        s_v[0][wave_id()] = nh;
        s_v[1][wave_id()] = nu;
        s_v[2][wave_id()] = nuh;
        s_v[3][wave_id()] = last;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0, d = 0, l = 0;
        for (int w = 0; w < kWaves; ++w) {
            a += s_v[0][w];
            b += s_v[1][w];
            d += s_v[2][w];
            l = s_v[3][w] > l ? s_v[3][w] : l;
        }
        c_heads[c] = a;
        c_u[c] = b;
        c_uh[c] = d;
        c_last[c] = l;
    }
}

// exclusive sums of c_heads/c_u/c_uh and exclusive max of c_last over the
// chunks (one workgroup; chunks <= a few thousand); totals -> words[0..2].
__global__ __launch_bounds__(kBlock) void k_seg_scan(uint32_t* __restrict__ c_heads, uint32_t* __restrict__ c_u,
                                                     uint32_t* __restrict__ c_uh, uint32_t* __restrict__ c_last,
                                                     uint32_t chunks, uint32_t* __restrict__ words) {
    __shared__ uint32_t s_tmp[kWaves];
    __shared__ uint32_t s_max[kBlock];
    uint32_t* arr[3] = {c_heads, c_u, c_uh};
    for (int a = 0; a < 3; ++a) {
        uint32_t carry = 0;
        for (uint32_t base = 0; base < chunks; base += kBlock * 4) {
            uint32_t v[4], sum = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t i = base + threadIdx.x * 4 + j;
                v[j] = (i < chunks) ? arr[a][i] : 0u;
                sum += v[j];
            }
            uint32_t tot;
            uint32_t off = block_exclusive_sum(sum, s_tmp, &tot) + carry;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t i = base + threadIdx.x * 4 + j;
                if (i < chunks) arr[a][i] = off;
                off += v[j];
            }
            carry += tot;
        }
        if (threadIdx.x == 0) words[a] = carry;
        __syncthreads();
    }
    // exclusive running max of c_last (Hillis-Steele in LDS, kBlock per step)
    uint32_t carry = 0;
    for (uint32_t base = 0; base < chunks; base += kBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = (i < chunks) ? c_last[i] : 0u;
        s_max[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < kBlock; o <<= 1) {
            const uint32_t y = (threadIdx.x >= (uint32_t)o) ? s_max[threadIdx.x - o] : 0u;
            __syncthreads();
            if (y > s_max[threadIdx.x]) s_max[threadIdx.x] = y;
            __syncthreads();
        }
        const uint32_t incl = s_max[threadIdx.x] > carry ? s_max[threadIdx.x] : carry;
        const uint32_t prev = threadIdx.x ? s_max[threadIdx.x - 1] : 0u;
        const uint32_t excl = prev > carry ? prev : carry;
        if (i < chunks) c_last[i] = excl;
        __syncthreads();
        const uint32_t blk = s_max[kBlock - 1];
        carry = blk > carry ? blk : carry;
        (void)incl;
        __syncthreads();
    }
}

// Where rank[x] lives: rank[x] itself (prefix == nullptr: the n-entry rank
// array of one GPU), or the range-partitioned build's compact map -- only
// the members of this rank's round-1 unsorted set have ranks, in text order:
// rank[prefix[x >> 8] + the members of x's 256-bit block below x], prefix
// the exclusive popcount scan of the member bitmap per 8-word block
// (sa_dist.h; one word per 256 positions: the scan writes n / 64 bytes, not
// n / 8).  The block's 32 bytes share one cache line.  n / 8 + n / 64 +
// 4 |U| bytes per rank instead of 4 n.
struct RankMap {
    const uint32_t* __restrict__ member = nullptr;   // 32-byte aligned, whole blocks
    const uint32_t* __restrict__ prefix = nullptr;
    __device__ __forceinline__ uint64_t slot(uint32_t x) const {
        if (!prefix) return x;
        const uint32_t g = x >> 8, k = (x >> 5) & 7u;
        const uint4* p = reinterpret_cast<const uint4*>(member) + 2 * (uint64_t)g;
        const uint4 a = p[0], c = p[1];
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
        uint32_t cnt = prefix[g];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q)
            cnt += (uint32_t)__popc(q < k ? w[q] : q == k ? (w[q] & ((1u << (x & 31u)) - 1u)) : 0u);
        return cnt;
    }
};

// Per sorted index s (idx = sorted suffix index):
//   rank[idx]   = pos(head of s's group) + 1  (at rm.slot(idx))
//   sa[pos(s)]  = idx                               (when sa != nullptr)
//   unsorted members are compacted, in order, to (u_pos, u_idx, u_g) with
//   u_g the dense id of their group among unsorted groups (+ g_off: the
//   tied-block round puts its tied groups first, sa_pivot.h); gsn (when
//   given) the first slot of each of those groups.
template <class Pos>
__global__ __launch_bounds__(kBlock) void k_seg_write(const uint64_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ idx, Chunking ch, Pos pos,
                                                      const uint32_t* __restrict__ o_u,
                                                      const uint32_t* __restrict__ o_uh,
                                                      const uint32_t* __restrict__ o_last,
                                                      uint32_t* __restrict__ rank, uint32_t* __restrict__ sa,
                                                      uint32_t* __restrict__ u_pos, uint32_t* __restrict__ u_idx,
                                                      uint32_t* __restrict__ u_g, uint32_t* __restrict__ member,
                                                      int dense_rank, uint32_t rank_off, RankMap rm = RankMap{},
                                                      uint32_t g_off = 0, uint32_t* __restrict__ gsn = nullptr,
                                                      uint32_t q_off = 0) {
    __shared__ uint64_t s_m[kWaves][kItems][3];
    __shared__ uint32_t s_w[3][kWaves];
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    const uint32_t wave = wave_id(), lane = lane_id();
    const uint64_t lt = lanemask_lt(), le = lt | (1ull << lane);
    uint32_t run_u = o_u[c], run_uh = o_uh[c], run_last = o_last[c];
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint64_t w0 = tb + (uint64_t)wave * kWaveTile;
        uint32_t cu = 0, cuh = 0, lf = 0;
        SegRows rows;
        rows.load(keys, w0, ch.n);
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t rb = w0 + (uint64_t)j * kWave;
            uint64_t mf = 0, mu = 0, muh = 0;
            seg_masks_reg(rows.k[j], rows.lo[j], rb + lane, ch.n, mf, mu, muh);
            if (rb >= e1) {
                mf = mu = muh = 0;
            } else {
                const uint64_t lim = e1 - rb >= 64 ? ~0ull : ((1ull << (e1 - rb)) - 1ull);
                mf &= lim;
                mu &= lim;
                muh &= lim;
            }
            if (lane == 0) {
                s_m[wave][j][0] = mf;
                s_m[wave][j][1] = mu;
                s_m[wave][j][2] = muh;
            }
            cu += __popcll(mu);
            cuh += __popcll(muh);
            if (mf) lf = (uint32_t)(rb + 63 - __clzll(mf)) + 1u;
        }
        if (lane == 0) {
            s_w[0][wave] = cu;
            s_w[1][wave] = cuh;
            s_w[2][wave] = lf;
        }
        __syncthreads();
        uint32_t off_u = run_u, off_uh = run_uh, carried = run_last;
        uint32_t tu = 0, tuh = 0, tl = run_last;
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t a = s_w[0][w], b = s_w[1][w], l = s_w[2][w];
            if (w < (int)wave) {
                off_u += a;
                off_uh += b;
                carried = l > carried ? l : carried;
            }
            tu += a;
            tuh += b;
            tl = l > tl ? l : tl;
        }
        // every row's index and position loaded before any is used; the
        // position of a member's group head comes from its row by a shuffle,
        // or is carried from the last head of an earlier row (one load per
        // wave and tile instead of a dependent load per member)
        uint32_t xs[kItems], ps[kItems];
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t s = w0 + (uint64_t)j * kWave + lane;
            xs[j] = s < e1 ? idx[s] : 0u;
            ps[j] = s < e1 ? pos(s) : 0u;
        }
        uint32_t carried_pos = carried > 0 ? pos((uint64_t)carried - 1u) : 0u;
#pragma unroll
        for (int j = 0; j < kItems; ++j) {
            const uint64_t rb = w0 + (uint64_t)j * kWave;
            const uint64_t mf = s_m[wave][j][0], mu = s_m[wave][j][1], muh = s_m[wave][j][2];
            const uint64_t s = rb + lane;
            const uint64_t mh = mf & le;
            const uint32_t hl = mh ? 63u - (uint32_t)__clzll(mh) : 0u;
            const uint32_t hrow = (uint32_t)__shfl((int)ps[j], (int)hl, kWave);
            const uint32_t hp = mh ? hrow : carried_pos;
            // sparse first round: rows without unsorted members write nothing
            if ((dense_rank || sa || mu) && s < e1) {
                const uint32_t x = xs[j];
                const uint32_t p = ps[j];
                const bool in_u = (mu >> lane) & 1ull;
                if (dense_rank || in_u) rank[rm.slot(x)] = rank_off + hp + 1u;
                if (sa) sa[p] = x;
                if (member && in_u) atomicOr(&member[x >> 5], 1u << (x & 31));
                if (in_u) {
                    const uint32_t q = off_u + (uint32_t)__popcll(mu & lt);
                    u_pos[q] = p;
                    u_idx[q] = x;
                    const uint32_t gl = off_uh + (uint32_t)__popcll(muh & le) - 1u;
                    u_g[q] = g_off + gl;
                    // the group's first slot, for the next round's pivot split
                    // (gsn is offset by g_off, q by q_off: the set's slot)
                    if (gsn && ((muh >> lane) & 1ull)) gsn[gl] = q_off + q;
                }
            }
            off_u += __popcll(mu);
            off_uh += __popcll(muh);
            if (mf) {
                const uint32_t ll = 63u - (uint32_t)__clzll(mf);
                carried = (uint32_t)(rb + ll) + 1u;
                carried_pos = (uint32_t)__shfl((int)ps[j], (int)ll, kWave);
            }
        }
        run_u += tu;
        run_uh += tuh;
        run_last = tl;
        __syncthreads();
    }
}

}  // namespace sa
