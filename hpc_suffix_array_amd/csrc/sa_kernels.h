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
};

// Later passes: the previous pass's output.
struct SrcKeys {
    const uint64_t* __restrict__ keys;
    const uint32_t* __restrict__ vals;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return keys[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return vals[e]; }
};

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
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t x) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, kWave);
        if ((int)lane_id() >= o) x += y;
    }
    return x;
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
__device__ __forceinline__ uint64_t wave_heads(const uint64_t* __restrict__ keys, uint64_t row0,
                                               uint64_t lim, uint64_t& prev_last, uint64_t& key_out,
                                               bool& ok_out) {
    const uint64_t e = row0 + lane_id();
    const bool ok = e < lim;
    const uint64_t key = ok ? keys[e] : 0ull;
    uint64_t prev = __shfl_up(key, 1, kWave);
    if (lane_id() == 0) prev = prev_last;
    prev_last = __shfl(key, kWave - 1, kWave);
    const bool head = ok && (e == 0 || key != prev);
    key_out = key;
    ok_out = ok;
    return __ballot(head);
}

__global__ __launch_bounds__(kBlock) void k_heads(const uint64_t* __restrict__ keys, Chunking ch,
                                                  uint32_t* __restrict__ counts) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    uint32_t cnt = 0;
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint64_t w0 = tb + (uint64_t)wave_id() * kWaveTile;
        uint64_t prev_last = (w0 > 0 && w0 < e1) ? keys[w0 - 1] : 0ull;
#pragma unroll 4
        for (int j = 0; j < kItems; ++j) {
            uint64_t key;
            bool ok;
            const uint64_t m = wave_heads(keys, w0 + (uint64_t)j * kWave, e1, prev_last, key, ok);
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

}  // namespace sa
