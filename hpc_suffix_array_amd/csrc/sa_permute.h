// sa_permute.h -- the re-rank scatter of the reference schedule as a
// coalesced permutation by suffix index.
//
// manber_myers.c:101-110 writes rank_array[suffixes[i].index] = current_rank
// for every sorted position i: one random 4-byte write per suffix.  As one
// kernel (k_rerank) that is 39.5 ms per round at n = 2^30 (r02_a: every
// write its own HBM line).  Here the same values reach rank[] in three
// coalesced steps, an MSD partition of the (idx, rank) pairs by idx:
//
//   k_perm_rank   sorted keys + idx -> dense rank of each sorted position
//                 (head flags, as k_rerank) -> pair (idx << 32 | rank),
//                 partitioned by idx >> s1 into <= 256 bins.  idx is a
//                 permutation of 0..n-1, so bin b holds exactly the idx of
//                 [b << s1, (b + 1) << s1): its place is known without a
//                 histogram, and tiles take their slots in it from a
//                 per-bin atomic cursor (the order inside a bin is free).
//   k_perm_split  each bin partitioned again by (idx >> s2) & (nsub - 1)
//                 into 2^s2-entry sub-bins (skipped when s1 == s2).
//   k_perm_place  one workgroup per sub-bin: the pairs land in an LDS copy
//                 of rank[sub-bin] by idx, which is then written out whole.
//
// Bytes per suffix: 12 read + 8 written, 8 + 8, 8 + 4 (48 B, all streamed
// or in runs of ~32 pairs) instead of 12 read + one random 4-byte write.
#pragma once
#include "sa_kernels.h"
#include "sa_lsd.h"

namespace sa {

constexpr uint32_t kPermSub = 14;   // sub-bin = 2^14 ranks = 64 KiB of LDS
constexpr int kPermBlock = 1024;
constexpr int kPermItems = 8;       // 8192 pairs per tile (64 KiB staged)
constexpr uint32_t kPermMaxSub = 1024;

// bin shifts for n suffixes: <= 256 first-level bins, sub-bins of 2^kPermSub
struct PermPlan {
    uint32_t s1, s2, nb1, nsub, tpb;   // tpb: k_perm_split tiles per bin
};

// exclusive scan of x over the first NB threads of a BLOCK-thread workgroup
// (every thread calls it; s_tmp holds NB / kWave words)
template <int NB>
__device__ __forceinline__ uint32_t perm_scan(uint32_t x, uint32_t* s_tmp) {
    const uint32_t inc = wave_inclusive_sum(x);
    if (lane_id() == kWave - 1 && wave_id() < (uint32_t)(NB / kWave)) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int w = 0; w < NB / kWave; ++w) off += (w < (int)wave_id()) ? s_tmp[w] : 0u;
    return off + inc - x;
}

// Loads the words of wave slice [w0, w0 + 64 ITEMS) (rows of 64) and the
// key before it, all issued before any use (wave_heads row by row waited
// for each row's load in turn), and returns the rows' head masks: key =
// word >> kshift, head = first position or key != its predecessor's.
template <int ITEMS>
__device__ __forceinline__ void slice_heads(const uint64_t* __restrict__ keys, uint64_t w0, uint64_t e1,
                                            uint32_t kshift, uint64_t* wd, uint64_t* m) {
    const uint32_t lane = lane_id();
    uint64_t prev_last = (w0 > 0 && w0 < e1) ? keys[w0 - 1] : 0ull;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t e = w0 + (uint64_t)j * kWave + lane;
        wd[j] = e < e1 ? keys[e] : 0ull;
    }
    prev_last >>= kshift;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t e = w0 + (uint64_t)j * kWave + lane;
        const uint64_t key = wd[j] >> kshift;
        uint64_t prev = __shfl_up(key, 1, kWave);
        if (lane == 0) prev = prev_last;
        prev_last = __shfl(key, kWave - 1, kWave);
        m[j] = __ballot(e < e1 && (e == 0 || key != prev));
    }
}

// Head counts per first-level tile (sorted positions [t T, (t + 1) T));
// k_scan_heads turns them into offsets and D.
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_tile_heads(const uint64_t* __restrict__ keys, uint64_t n,
                                                       uint32_t kshift, uint32_t* __restrict__ counts) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int WT = kWave * ITEMS;
    __shared__ uint32_t s_w[WAVES];
    const uint64_t tb = (uint64_t)blockIdx.x * BLOCK * ITEMS;
    const uint64_t e1 = (tb + BLOCK * ITEMS) < n ? tb + BLOCK * ITEMS : n;
    uint64_t wd[ITEMS], m[ITEMS];
    slice_heads<ITEMS>(keys, tb + (uint64_t)wave_id() * WT, e1, kshift, wd, m);
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) cnt += (uint32_t)__popcll(m[j]);
    if (lane_id() == 0) s_w[wave_id()] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) t += s_w[w];
        counts[blockIdx.x] = t;
    }
}

// Level 1: one workgroup per tile of BLOCK x ITEMS sorted positions (tile_off
// = heads before the tile, k_tile_heads + k_scan_heads); wave w owns a
// contiguous slice of 64 x ITEMS of it.  Slots in a bin come from the bin's
// cursor, one device-scope atomic per tile and bin (exact per-tile offsets
// from a counting pass measured slower: 223.5 vs 216 ms for the 1 GiB DNA
// reference schedule, the counts' scattered writes and scan cost more).
// PACKED: keys are (key << kshift | idx) items (sa_lsd.h k_lsd), idx unused.
// (Per-XCD sub-ranges of the bins -- tile t claiming from cursor (t mod 8,
// bin) inside its queue's share of the bin, the shares counted by the
// round's last LSD pass -- saved ~0.5 ms of the three levels' 44 ms per
// 1 GiB build and cost the LSD passes ~7 ms of LDS atomics: removed,
// profiles/r05_k_ab_refsched_perm_xq.txt.)
template <int BLOCK, int ITEMS, bool PACKED>
__global__ __launch_bounds__(BLOCK) void k_perm_rank(const uint64_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ idx, uint64_t n,
                                                      const uint32_t* __restrict__ tile_off, uint32_t s1,
                                                      uint32_t kshift, uint32_t* __restrict__ cur,
                                                      uint64_t* __restrict__ out) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int WT = kWave * ITEMS;
    constexpr int T = BLOCK * ITEMS;
    constexpr int NB = 256;
    static_assert(BLOCK >= NB, "one thread per bin");
    __shared__ uint64_t s_pair[T];
    __shared__ uint32_t s_cnt[NB];
    __shared__ uint32_t s_start[NB];
    __shared__ uint32_t s_gofs[NB];
    __shared__ uint32_t s_wtot[WAVES];
    __shared__ uint32_t s_tmp[NB / kWave];
    const uint32_t tid = threadIdx.x, wave = wave_id(), lane = lane_id();
    const uint64_t tb = (uint64_t)blockIdx.x * T;
    const uint64_t e1 = (tb + T) < n ? tb + T : n;
    const uint32_t valid = (uint32_t)(e1 - tb);
    if (tid < (uint32_t)NB) s_cnt[tid] = 0;
    const uint64_t le_mask = lanemask_lt() | (1ull << lane);
    const uint64_t w0 = tb + (uint64_t)wave * WT;
    uint32_t x[ITEMS];
    if constexpr (!PACKED) {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t e = w0 + (uint64_t)j * kWave + lane;
            x[j] = e < e1 ? idx[e] : ~0u;
        }
    }
    uint64_t wd[ITEMS], m[ITEMS];
    slice_heads<ITEMS>(keys, w0, e1, kshift, wd, m);
    uint32_t wsum = 0;
    const uint64_t imask = (1ull << kshift) - 1ull;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        wsum += (uint32_t)__popcll(m[j]);
        if constexpr (PACKED) x[j] = (w0 + (uint64_t)j * kWave + lane) < e1 ? (uint32_t)(wd[j] & imask) : ~0u;
    }
    if (lane == 0) s_wtot[wave] = wsum;
    __syncthreads();
    uint32_t woff = tile_off[blockIdx.x];
#pragma unroll
    for (int w = 0; w < WAVES; ++w) woff += (w < (int)wave) ? s_wtot[w] : 0u;
    uint32_t slot[ITEMS];
    uint64_t pr[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t r = woff + (uint32_t)__popcll(m[j] & le_mask);
        woff += (uint32_t)__popcll(m[j]);
        pr[j] = ((uint64_t)x[j] << 32) | r;
        slot[j] = x[j] != ~0u ? atomicAdd(&s_cnt[x[j] >> s1], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t cnt = tid < (uint32_t)NB ? s_cnt[tid] : 0u;
    const uint32_t st = perm_scan<NB>(cnt, s_tmp);
    if (tid < (uint32_t)NB) {
        s_start[tid] = st;
        s_gofs[tid] = cnt ? (tid << s1) + atomicAdd(&cur[tid], cnt) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        if (x[j] != ~0u) s_pair[s_start[x[j] >> s1] + slot[j]] = pr[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + tid;
        if (q < valid) {
            const uint64_t p = s_pair[q];
            const uint32_t b = (uint32_t)(p >> 32) >> s1;
            const uint64_t g = (uint64_t)s_gofs[b] + (q - s_start[b]);
            if (g < n) out[g] = p;
        }
    }
}

// Level 2: tile t of bin b.  Workgroup w runs on XCD w mod 8 (round robin),
// so bin b's tiles go to the workgroups w = 8 (t + tpb (b / 8)) + b mod 8:
// every tile of a bin on one XCD, whose L2 then merges the partial lines
// where consecutive tiles' runs of a sub-bin meet (~8 pairs per sub-bin and
// tile) -- one bin per XCD at a time instead of each bin's tiles dealt over
// all eight.  grid = 8 ceil(nb1 / 8) tpb.
// DSH: the pair's destination (absolute, or relative to its bin: only its
// low s1 bits are read) sits at bit DSH (the checker's pass B packs a text
// byte between it and the value, sa_check.h).  CLAMP: a slot past its
// sub-bin (a non-permutation; the checker's cursor test flags it) is dropped
// instead of written into the next sub-bin.
template <int BLOCK, int ITEMS, int DSH = 32, bool CLAMP = false, int TAG = 0>
__global__ __launch_bounds__(BLOCK) void k_perm_split(const uint64_t* __restrict__ in, uint64_t n, uint32_t s1,
                                                       uint32_t s2, uint32_t tpb, uint32_t* __restrict__ cur,
                                                       uint64_t* __restrict__ out) {
    constexpr int T = BLOCK * ITEMS;
    constexpr int NB = kPermMaxSub;
    static_assert(BLOCK >= NB, "one thread per sub-bin");
    __shared__ uint64_t s_pair[T];
    __shared__ uint32_t s_cnt[NB];
    __shared__ uint32_t s_start[NB];
    __shared__ uint32_t s_gofs[NB];
    __shared__ uint32_t s_tmp[NB / kWave];
    const uint32_t tid = threadIdx.x;
    const uint32_t r = blockIdx.x / 8u;
    const uint32_t b = (r / tpb) * 8u + (blockIdx.x & 7u), t = r % tpb;
    const uint32_t nsub = 1u << (s1 - s2);
    const uint64_t bin0 = (uint64_t)b << s1;
    const uint64_t bin1 = (bin0 + (1ull << s1)) < n ? bin0 + (1ull << s1) : n;
    const uint64_t tb = bin0 + (uint64_t)t * T;
    if (tb >= bin1) return;   // uniform over the workgroup
    const uint32_t valid = (uint32_t)((bin1 - tb) < (uint64_t)T ? (bin1 - tb) : (uint64_t)T);
    if (tid < (uint32_t)NB) s_cnt[tid] = 0;
    __syncthreads();
    uint64_t p[ITEMS];
    uint32_t sub[ITEMS], slot[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + tid;
        p[j] = in[tb + (q < valid ? q : valid - 1)];   // every load before the first use
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t q = j * BLOCK + tid;
        sub[j] = q < valid ? ((uint32_t)(p[j] >> DSH) >> s2) & (nsub - 1u) : NB;
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
        const uint32_t q = j * BLOCK + tid;
        if (q < valid) {
            const uint64_t v = s_pair[q];
            const uint32_t sb = ((uint32_t)(v >> DSH) >> s2) & (nsub - 1u);
            const uint64_t g = (uint64_t)s_gofs[sb] + (q - s_start[sb]);
            if (CLAMP) {
                const uint64_t s0 = bin0 + ((uint64_t)sb << s2);
                if (g < n && g < s0 + (1ull << s2)) out[g] = v;
            } else if (g < n) {
                out[g] = v;
            }
        }
    }
}

// Level 2 as persistent workgroups (k_perm_split's work, one tile of
// BLOCK x ITEMS pairs at a time): the one-tile-per-workgroup kernels run their
// load -> rank -> claim -> stage -> write chain with nothing in flight but the
// other workgroup of the CU (a permutation level ran at ~3-5 TB/s); here the
// next tile's pairs are loaded while the current one is staged and written.
// XCD q (workgroup w mod 8) takes the tiles of the bins b = q mod 8 from its
// own ticket tickets[q] (all tiles of a bin on one XCD, whose L2 merges the
// partial lines where consecutive tiles' runs of a sub-bin meet).  A bin's
// pairs: [b 2^s1, + its size) (st == 1), or its st stripe regions of level 1
// (sa_check.h BinStripes: region (b, q') at (b st + q') scap, filled to
// fill[q' fstride + b]), tpr tiles per region.  CLAMP: a slot past its
// sub-bin is dropped.  grid: a multiple of 8.
template <int BLOCK, int ITEMS, int DSH = 32, bool CLAMP = false, int TAG = 0>
__global__ __launch_bounds__(BLOCK) void k_split_p(const uint64_t* __restrict__ in, uint64_t n, uint32_t s1,
                                                    uint32_t s2, uint32_t nb1, uint32_t st, uint64_t scap,
                                                    uint32_t tpr, const uint32_t* __restrict__ fill, uint32_t fstride,
                                                    uint32_t* __restrict__ cur, uint64_t* __restrict__ out,
                                                    uint32_t* __restrict__ tickets) {
    constexpr int T = BLOCK * ITEMS;
    constexpr int NB = kPermMaxSub;
    static_assert(BLOCK >= NB, "one thread per sub-bin");
    __shared__ uint64_t s_pair[T];
    __shared__ uint32_t s_cnt[NB];
    __shared__ uint32_t s_start[NB];
    __shared__ uint32_t s_gofs[NB];
    __shared__ uint32_t s_tmp[NB / kWave];
    __shared__ uint32_t s_q[2];
    const uint32_t tid = threadIdx.x;
    const uint32_t q = blockIdx.x & 7u;
    const uint32_t nbq = nb1 > q ? (nb1 - q + 7u) / 8u : 0u;
    const uint32_t ntiles = nbq * st * tpr;
    const uint32_t nsub = 1u << (s1 - s2);
    // ticket x of queue q -> its bin and the tile's pairs [src0, src0 + valid)
    auto decode = [&](uint32_t x, uint32_t& b, uint64_t& src0, uint32_t& valid) {
        const uint32_t tt = x % tpr, r = x / tpr, sq = r % st;
        b = q + 8u * (r / st);
        const uint64_t b0 = (uint64_t)b << s1;
        uint64_t f, base;
        if (st == 1) {
            f = (n - b0) < (1ull << s1) ? n - b0 : (1ull << s1);
            base = b0;
        } else {
            f = fill[sq * fstride + b];
            f = f < scap ? f : scap;
            base = ((uint64_t)b * st + sq) * scap;
        }
        const uint64_t t0 = (uint64_t)tt * T;
        valid = t0 < f ? (uint32_t)((f - t0) < (uint64_t)T ? (f - t0) : (uint64_t)T) : 0u;
        src0 = base + t0;
    };
    uint64_t p[ITEMS];
    auto load = [&](uint64_t src0, uint32_t valid) {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t x = j * BLOCK + tid;
            p[j] = valid ? in[src0 + (x < valid ? x : valid - 1)] : 0ull;
        }
    };
    if (tid < (uint32_t)NB) s_cnt[tid] = 0;
    if (tid == 0) s_q[0] = atomicAdd(&tickets[q], 1u);
    __syncthreads();
    uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[0]);
    uint32_t b = 0, valid = 0;
    uint64_t src0 = 0;
    if (x < ntiles) {
        decode(x, b, src0, valid);
        load(src0, valid);
    }
    uint32_t par = 0;
    while (x < ntiles) {
        if (tid == 0) s_q[par ^ 1u] = atomicAdd(&tickets[q], 1u);   // the next tile's ticket
        const uint64_t bin0 = (uint64_t)b << s1;
        uint32_t sub[ITEMS], slot[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t xx = j * BLOCK + tid;
            sub[j] = xx < valid ? ((uint32_t)(p[j] >> DSH) >> s2) & (nsub - 1u) : NB;
            slot[j] = sub[j] < (uint32_t)NB ? atomicAdd(&s_cnt[sub[j]], 1u) : 0u;
        }
        __syncthreads();
        const uint32_t cnt = tid < (uint32_t)NB ? s_cnt[tid] : 0u;
        const uint32_t stt = perm_scan<NB>(cnt, s_tmp);
        if (tid < (uint32_t)NB) {
            s_start[tid] = stt;
            s_gofs[tid] = cnt ? (uint32_t)bin0 + (tid << s2) + atomicAdd(&cur[(uint64_t)b * nsub + tid], cnt) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            if (sub[j] < (uint32_t)NB) s_pair[s_start[sub[j]] + slot[j]] = p[j];
        // the tile is in LDS: the next tile's pairs go out now
        const uint32_t xn = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[par ^ 1u]);
        const uint32_t vcur = valid, bcur = b;
        if (xn < ntiles) {
            decode(xn, b, src0, valid);
            __builtin_amdgcn_sched_barrier(0);
            load(src0, valid);
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t xx = j * BLOCK + tid;
            if (xx < vcur) {
                const uint64_t v = s_pair[xx];
                const uint32_t sb = ((uint32_t)(v >> DSH) >> s2) & (nsub - 1u);
                const uint64_t g = (uint64_t)s_gofs[sb] + (xx - s_start[sb]);
                if (CLAMP) {
                    const uint64_t s0 = ((uint64_t)bcur << s1) + ((uint64_t)sb << s2);
                    if (g < n && g < s0 + (1ull << s2)) out[g] = v;
                } else if (g < n) {
                    out[g] = v;
                }
            }
        }
        if (tid < (uint32_t)NB) s_cnt[tid] = 0;
        __syncthreads();   // s_pair / s_start / s_gofs reused by the next tile
        x = xn;
        par ^= 1u;
    }
}

// The next reference round's first-digit counts, taken while the ranks are
// written (the LSD sort's histogram kernel then skips its 8-byte-per-suffix
// read): its key of position i is (rank[i] << w | rank[i + h]) with the
// first digit in the low `bits` bits of rank[i + h] (bits <= w), so rank[j]
// counts for i = j - h, in that position's queue of the next round's LSD
// passes (sa_lsd.h XQ: out[q][digit]); positions i >= n - h (rank[i + h] =
// 0: digit 0) are added by workgroup 0.
struct NextHist {
    uint32_t* out = nullptr;   // [8][kLsdMaxRadix]; nullptr: none
    uint32_t mask = 0;
    uint64_t h = 0;
    QDiv qd;
    uint64_t qspan = 0;        // positions per queue (qd divides by it)
};

// Level 3: sub-bins of 2^kPermSub ranks, one at a time; a pair whose idx lies
// outside the sub-bin (a broken partition) raises err bit 1 and is dropped.
// Dense ranks are >= 1, so the sub-bin's LDS copy starts at 0 and a slot
// still 0 at the write (a missing or duplicated idx) raises err bit 2.
// HIST: the NextHist counts; each workgroup takes a contiguous run of
// sub-bins (spb of them), whose positions lie in at most two queues of the
// next round, counted in LDS (2 x 1024 words: two workgroups per CU still)
// and added to the global counts once.
// TAG: 1 for the checker's pass A (sa_check.h), 2 for LCP's PHI (sa_lcp.h),
// so profiles tell them apart
template <int BLOCK, bool HIST = false, int TAG = 0>
__global__ __launch_bounds__(BLOCK) void k_perm_place(const uint64_t* __restrict__ in, uint64_t n,
                                                       uint32_t* __restrict__ rank, uint32_t* __restrict__ err,
                                                       NextHist nh = NextHist{}, uint32_t spb = 1) {
    constexpr uint32_t S = 1u << kPermSub;
    __shared__ uint32_t s_r[S];
    __shared__ uint32_t s_h[HIST ? 2 * kLsdMaxRadix : 1];
    const uint32_t nsub = (uint32_t)((n + S - 1) >> kPermSub);
    const uint32_t sb0 = HIST ? blockIdx.x * spb : blockIdx.x;
    const uint32_t sb1 = HIST ? std::min(nsub, sb0 + spb) : std::min(nsub, sb0 + 1);
    // the queue of this workgroup's first counted position
    const uint64_t j0 = std::max<uint64_t>((uint64_t)sb0 << kPermSub, nh.h);
    const uint32_t q0 = HIST ? nh.qd.q(j0 - nh.h) : 0u;
    if constexpr (HIST) {
        for (uint32_t i = threadIdx.x; i < 2 * kLsdMaxRadix; i += BLOCK) s_h[i] = 0u;
    }
    auto count = [&](uint64_t j, uint32_t r) {
        if (HIST && j >= nh.h) {
            const uint32_t dq = nh.qd.q(j - nh.h) - q0;   // 0 or 1
            const uint32_t d = r & nh.mask;
            if (dq < 2u) atomicAdd(&s_h[dq * kLsdMaxRadix + d], 1u);
            else atomicAdd(&nh.out[(q0 + dq) * kLsdMaxRadix + d], 1u);   // (not reached: spb sub-bins < a queue)
        }
    };
    bool bad = false, hole = false;
    for (uint32_t sb = sb0; sb < sb1; ++sb) {
        const uint64_t base = (uint64_t)sb << kPermSub;
        const uint32_t valid = (uint32_t)((n - base) < (uint64_t)S ? (n - base) : (uint64_t)S);
        __syncthreads();   // s_r of the previous sub-bin read out
        for (uint32_t q = threadIdx.x; q < valid; q += BLOCK) s_r[q] = 0u;
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < valid; q += BLOCK) {
            const uint64_t p = in[base + q];
            const uint32_t x = (uint32_t)(p >> 32);
            if ((x >> kPermSub) != sb || (x & (S - 1u)) >= valid) {
                bad = true;
                continue;
            }
            s_r[x & (S - 1u)] = (uint32_t)p;
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x * 4; q < valid; q += BLOCK * 4) {
            if (q + 4 <= valid) {
                uint4 v;
                v.x = s_r[q];
                v.y = s_r[q + 1];
                v.z = s_r[q + 2];
                v.w = s_r[q + 3];
                hole |= (v.x == 0u) | (v.y == 0u) | (v.z == 0u) | (v.w == 0u);
                *reinterpret_cast<uint4*>(rank + base + q) = v;
                count(base + q, v.x);
                count(base + q + 1, v.y);
                count(base + q + 2, v.z);
                count(base + q + 3, v.w);
            } else {
                for (uint32_t i = q; i < valid; ++i) {
                    hole |= s_r[i] == 0u;
                    rank[base + i] = s_r[i];
                    count(base + i, s_r[i]);
                }
            }
        }
    }
    if (bad) atomicOr(err, 2u);
    if (hole) atomicOr(err, 4u);
    if constexpr (HIST) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 2 * kLsdMaxRadix; i += BLOCK)
            if (s_h[i] && q0 + i / kLsdMaxRadix < 8u) atomicAdd(&nh.out[q0 * kLsdMaxRadix + i], s_h[i]);
        if (blockIdx.x == 0 && threadIdx.x < 8) {   // positions [n - h, n) of queue t: digit 0
            const uint64_t lo = nh.h < n ? n - nh.h : 0;
            const uint64_t a = std::max<uint64_t>(lo, threadIdx.x * nh.qspan);
            const uint64_t b = std::min<uint64_t>(n, (threadIdx.x + 1) * nh.qspan);
            if (b > a) atomicAdd(&nh.out[threadIdx.x * kLsdMaxRadix], (uint32_t)(b - a));
        }
    }
}

}  // namespace sa
