// sa_lsd.h -- the reference schedule's per-round LSD radix sort
// (radix_sort_suffixes_seq, manber_myers.c:37-48: a stable counting pass on
// rank[1], then on rank[0]) as single-pass digit scatters over the packed
// key (rank[i] << w) | rank[i + h].
//
// Against k_onesweep (sa_onesweep.h, one 4096-pair tile per workgroup):
//   * persistent workgroups taking 8192-pair tiles from a ticket in order,
//     the next tile's loads in flight during the look-back, the LDS staging
//     and the writes (the structure of sa_split.h's k_split; same deadlock
//     argument: a tile waits only on tiles of running workgroups);
//   * stable ranks from per-wave match-any ballots (the counting sort's
//     stability, :27-31, is what LSD needs; LDS atomics would not keep it);
//   * digits of 8 to 10 bits, the widths chosen per round by lsd_plan
//     (sa_build.hip), so an 18-bit key takes two passes instead of three;
//   * PACKED: while key bits + index bits <= 64 the pass moves one 64-bit
//     item (key << ib | index) -- 16 bytes per pair and pass instead of 24;
//   * each pass counts the next pass's digits of the keys it ranks (one LDS
//     atomic per key, flushed per workgroup), so the histogram kernel reads
//     the ranks for the first digit only (k_lsd_hist over every digit of a
//     60-bit key: 6.6 ms at 2^30);
//   * the first pass prefetches the raw rank words and builds the keys when
//     its tile is ranked (building them at the load made the staging wait).
#pragma once
#include "sa_split.h"

namespace sa {

#ifndef SA_LSD_LOOK
#define SA_LSD_LOOK 4   // predecessor states read per look-back step (8: 1.02x, 16: 1.3x the pass time)
#endif
#ifndef SA_HIST_PREFETCH
#define SA_HIST_PREFETCH 1   // k_lsd_hist issues the next step's loads before counting this one's
#endif
#ifndef SA_LSD_PROF
#define SA_LSD_PROF 0       // per-phase clock64 spans of k_lsd printed per pass (diagnostic builds)
#endif
// workgroup shapes (A/B overridable): PACKED passes of <= 9-bit digits and
// unpacked ones; 10-bit digits always take 1024 x 8 (one thread per digit).
// 1 GiB DNA reference schedule (interleaved A/B, one box): packed 1024 x 8
// 194.6 / 195.0 ms, 512 x 12 (two workgroups per CU) 191.4 / 191.7, 512 x 8
// 202.3; unpacked 512 x 8 206 (kept 1024 x 8); 512 x 16 spills 45-78 VGPRs.
#ifndef SA_LSD_PK_BLOCK
#define SA_LSD_PK_BLOCK 512
#endif
#ifndef SA_LSD_PK_ITEMS
#define SA_LSD_PK_ITEMS 12
#endif
#ifndef SA_LSD_UP_BLOCK
#define SA_LSD_UP_BLOCK 1024
#endif
#ifndef SA_LSD_UP_ITEMS
#define SA_LSD_UP_ITEMS 8
#endif
// XQ passes (below): 1024 x 8 for every digit width (their per-queue
// next-pass counters take 32 KiB of LDS)
template <bool PACKED, int RBITS, bool XQ = false>
constexpr int lsd_block() { return XQ || RBITS > 9 ? 1024 : PACKED ? SA_LSD_PK_BLOCK : SA_LSD_UP_BLOCK; }
template <bool PACKED, int RBITS, bool XQ = false>
constexpr int lsd_items() { return XQ || RBITS > 9 ? 8 : PACKED ? SA_LSD_PK_ITEMS : SA_LSD_UP_ITEMS; }
constexpr int kLsdMaxRadix = 1024;
constexpr int kLsdXqTile = 1024 * 8;
// per-queue counts of every pass, the bases of one, the tickets of every pass
constexpr int kLsdXqWords = kMaxPasses * 8 * kLsdMaxRadix + 8 * kLsdMaxRadix + kMaxPasses * 8 * 32;
#ifndef SA_LSD_XQ
#define SA_LSD_XQ 1
#endif

// ---------------------------------------------------------------------------
// XQ passes (round 5; the second bucket pass's per-XCD queues, sa_split.h
// SegXq, made stable): queue q = workgroup mod 8 (= its XCD) takes the tiles
// of the q-th eighth of the input, [q tpq, (q + 1) tpq), from its own ticket,
// and its items of digit d go to [base(d) + sum_{q' < q} count(q', d), ...):
// the output stays in (digit, tile) order -- stable, as the LSD sort needs --
// while each (queue, digit) run is written by one XCD, whose L2 merges the
// partial lines at the run ends.  The decoupled look-back runs over the
// queue's own tiles.  count(q, d) of a pass is counted by the pass before it
// (the item's queue in the next pass is its output position over the queue
// span) or, for the first pass of a round, by k_lsd_hist.
// ---------------------------------------------------------------------------
// floor(g / qspan) as the high half of g * ceil(2^64 / qspan): exact for g <
// 2^33 and qspan < 2^31 (the error g / 2^64 stays below 1 / qspan)
struct QDiv {
    uint64_t magic = 0;   // 0: one queue
    __device__ __forceinline__ uint32_t q(uint64_t g) const { return magic ? (uint32_t)__umul64hi(g, magic) : 0u; }
};

// the passes of one sort: digit p is bits [shift[p], shift[p] + bits[p])
struct LsdPlan {
    uint32_t P;
    uint32_t shift[kMaxPasses];
    uint32_t bits[kMaxPasses];
};

// First pass of a PACKED round: item = ((rank[i] << w | rank[i+h]) << ib) | i.
struct SrcRankPk {
    const uint32_t* __restrict__ rank;
    uint64_t n;
    uint64_t h;
    uint32_t w, ib;
    __device__ __forceinline__ uint64_t key(uint64_t e) const {
        const uint64_t r0 = rank[e];
        const uint64_t r1 = (e + h < n) ? rank[e + h] : 0u;
        return (((r0 << w) | r1) << ib) | e;
    }
    __device__ __forceinline__ uint32_t val(uint64_t) const { return 0u; }
    // two-step form for a prefetch: the loads, then the key (k_lsd issues
    // the next tile's loads before the staging and builds keys only when the
    // tile is ranked, so nothing waits for them in between)
    static constexpr bool kRaw = true;
    __device__ __forceinline__ uint64_t raw(uint64_t e) const {
        return (uint64_t)rank[e] | ((uint64_t)((e + h < n) ? rank[e + h] : 0u) << 32);
    }
    __device__ __forceinline__ uint64_t finish(uint64_t r, uint64_t e) const {
        return ((((r & 0xFFFFFFFFull) << w) | (r >> 32)) << ib) | e;
    }
};

// the two-step (raw, finish) form of a source, when it has one
template <class S, class = void>
struct has_raw { static constexpr bool value = false; };
template <class S>
struct has_raw<S, decltype((void)S::kRaw)> { static constexpr bool value = S::kRaw; };

// Later passes of a PACKED round: the items themselves.
struct SrcItems {
    const uint64_t* __restrict__ keys;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return keys[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t) const { return 0u; }
};

// Digit totals of every pass of the plan in one read of the first source
// (the multiset of keys is the same in every pass); one atomic per run of
// equal digits across neighbouring lanes (hist_add_runs: a degenerate
// text's equal keys would otherwise put 64 lanes on one bin).
// qd.magic != 0 (XQ, plan.P = 1): the first digit counted per queue of the
// input position, ghist[q][d].
template <class Src>
__global__ __launch_bounds__(kBlock) void k_lsd_hist(Src src, uint64_t n, LsdPlan plan,
                                                     uint32_t* __restrict__ ghist, QDiv qd = QDiv{}) {
    static_assert(kMaxPasses >= 8, "the per-queue counts use the per-pass rows");
    __shared__ uint32_t s_h[kMaxPasses * kLsdMaxRadix];
    const uint32_t rows = qd.magic ? 8u : plan.P;
    for (uint32_t i = threadIdx.x; i < rows * kLsdMaxRadix; i += kBlock) s_h[i] = 0;
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    // 8 keys per lane per step, all loads issued before the counting, and
    // the next step's issued before this one's are counted
    constexpr int U = 8;
    const uint64_t step = (uint64_t)gridDim.x * kBlock * U;
    uint64_t kn[U];
    auto load = [&](uint64_t b2, uint64_t (&kk)[U]) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t e = b2 + (uint64_t)j * kBlock + threadIdx.x;
            kk[j] = src.key(e < n ? e : n - 1);
        }
    };
    if (SA_HIST_PREFETCH && (uint64_t)blockIdx.x * kBlock * U < n) load((uint64_t)blockIdx.x * kBlock * U, kn);
    for (uint64_t b = (uint64_t)blockIdx.x * kBlock * U; b < n; b += step) {
        uint64_t k[U];
        if constexpr (SA_HIST_PREFETCH) {
#pragma unroll
            for (int j = 0; j < U; ++j) k[j] = kn[j];
            load(b + step < n ? b + step : b, kn);
        } else {
            load(b, k);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t e = b + (uint64_t)j * kBlock + threadIdx.x;
            if (e >= n) break;   // the active lanes stay a prefix of the wave
            const uint32_t nact = (uint32_t)__popcll(__ballot(1));
            const uint32_t qrow = qd.q(e);   // XQ: the input position's queue
            for (uint32_t p = 0; p < plan.P; ++p) {
                const uint32_t d = (uint32_t)(k[j] >> plan.shift[p]) & ((1u << plan.bits[p]) - 1u);
                const uint32_t slot = (qd.magic ? qrow : p) * kLsdMaxRadix + d;
                const uint32_t dl = __shfl_up(slot, 1, 64);
                const bool head = lane == 0 || dl != slot;
                const uint64_t hm = __ballot(head) & above;
                const uint32_t next = hm ? (uint32_t)__ffsll((long long)hm) - 1u : nact;
                if (head) atomicAdd(&s_h[slot], next - lane);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < rows * kLsdMaxRadix; i += kBlock)
        if (s_h[i]) atomicAdd(&ghist[i], s_h[i]);
}

// XQ bases of one pass from its per-queue counts qh[q][d] (one 1024-thread
// workgroup): qbase[q][d] = (digits below d, all queues) + (digit d in queues
// below q)
__global__ __launch_bounds__(1024) void k_lsd_qbase(const uint32_t* __restrict__ qh, uint32_t bins,
                                                    uint32_t* __restrict__ qbase) {
    __shared__ uint32_t s_tmp[16];
    const uint32_t i = threadIdx.x;
    uint32_t c[8], tot = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        c[q] = i < bins ? qh[q * kLsdMaxRadix + i] : 0u;
        tot += c[q];
    }
    const uint32_t inc = wave_inclusive_sum(tot);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t w = 0; w < wave_id(); ++w) off += s_tmp[w];
    uint32_t b = off + inc - tot;
    if (i < bins)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            qbase[q * kLsdMaxRadix + i] = b;
            b += c[q];
        }
}

// base[p][d] = exclusive scan of ghist[p][..] (one 1024-thread workgroup per pass)
__global__ __launch_bounds__(1024) void k_lsd_base(const uint32_t* __restrict__ ghist, LsdPlan plan,
                                                   uint32_t* __restrict__ base) {
    __shared__ uint32_t s_tmp[16];
    const uint32_t p = blockIdx.x, i = threadIdx.x;
    const uint32_t bins = 1u << plan.bits[p];
    const uint32_t x = i < bins ? ghist[p * kLsdMaxRadix + i] : 0u;
    const uint32_t inc = wave_inclusive_sum(x);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t w = 0; w < wave_id(); ++w) off += s_tmp[w];
    if (i < bins) base[p * kLsdMaxRadix + i] = off + inc - x;
}

// One stable pass over digit (key >> shift) & (2^nbits - 1), nbits <= RBITS.
// XQ: digit_base is qbase[8][kLsdMaxRadix], ticket the 8 queue tickets (at
// a stride of 32 words), next_hist the next pass's [8][kLsdMaxRadix] counts;
// qd divides an output position by the queue span (tpq tiles).
template <class Src, int RBITS, bool PACKED, bool XQ = false>
__global__ __launch_bounds__((lsd_block<PACKED, RBITS, XQ>()), 4) void k_lsd(Src src, uint64_t n, uint32_t shift, uint32_t nbits,
                                                   const uint32_t* __restrict__ digit_base,
                                                   uint64_t* __restrict__ states, uint32_t* __restrict__ ticket,
                                                   uint32_t epoch, uint64_t* __restrict__ out_keys,
                                                   uint32_t* __restrict__ out_vals, uint32_t* __restrict__ err,
                                                   unsigned long long* __restrict__ prof, uint32_t nshift,
                                                   uint32_t nnbits, uint32_t* __restrict__ next_hist,
                                                   QDiv qd = QDiv{}, uint32_t tpq = 0) {
    constexpr int BLOCK = lsd_block<PACKED, RBITS, XQ>();
    constexpr int ITEMS = lsd_items<PACKED, RBITS, XQ>();
    constexpr int WAVES = BLOCK / kWave;
    constexpr int RADIX = 1 << RBITS;
    constexpr int RWAVES = RADIX / kWave;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE <= 65535 && WTILE <= 65535, "16-bit tile offsets");
    static_assert(BLOCK >= RADIX, "one thread per digit");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_vals[PACKED ? 1 : TILE];
    __shared__ uint16_t s_wcnt[WAVES][RADIX];   // per-wave digit counts, then wave offsets
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile[2];
    // the next pass's digit totals of this workgroup's tiles (XQ: per queue)
    constexpr int NH = XQ ? 8 * kLsdMaxRadix : kLsdMaxRadix;
    __shared__ uint32_t s_nh[NH];

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    const uint32_t mask = (1u << nbits) - 1u;
    const uint32_t nmask = (1u << nnbits) - 1u;
    for (int i = dg; i < NH; i += BLOCK) s_nh[i] = 0;
    const uint64_t tiles_all = (n + TILE - 1) / TILE;
    // XQ: this workgroup's queue and its tiles [t0, t1) (tile ids are global)
    const uint32_t xq = XQ ? (blockIdx.x & 7u) : 0u;
    const uint64_t t0 = XQ ? std::min<uint64_t>((uint64_t)xq * tpq, tiles_all) : 0ull;
    const uint64_t tiles = XQ ? std::min<uint64_t>(t0 + tpq, tiles_all) : tiles_all;   // the end of the tiles taken
    if constexpr (XQ) {
        ticket += xq * 32;
        digit_base += xq * kLsdMaxRadix;
    }
    const uint64_t tag = (uint64_t)(epoch & kEpochMask) << 48;
    uint32_t* const wc32 = reinterpret_cast<uint32_t*>(&s_wcnt[0][0]);
    if (dg == 0) s_tile[0] = atomicAdd(ticket, 1u);
    for (int i = dg; i < WAVES * RADIX / 2; i += BLOCK) wc32[i] = 0;
    __syncthreads();
    uint64_t t = t0 + (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[0]);
    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    // clamped loads (pairs past the end are never ranked)
    auto load = [&](uint64_t tt, uint64_t* kk, uint32_t* vv) {
        const uint64_t tb = tt * TILE;
        const uint32_t last = (uint32_t)min(n - 1 - tb, (uint64_t)(TILE - 1));
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const uint64_t e = tb + (le < last ? le : last);
            if constexpr (has_raw<Src>::value)
                kk[j] = src.raw(e);
            else
                kk[j] = src.key(e);
            if constexpr (!PACKED) vv[j] = src.val(e);
        }
    };
    if (t < tiles) load(t, k, v);
    uint32_t par = 0;
    // SA_LSD_PROF (diagnostic builds): thread 0's clock64 spans per phase
    uint64_t tacc[5] = {0, 0, 0, 0, 0}, tlast = SA_LSD_PROF ? clock64() : 0;
    auto stamp = [&](int q) {
        if constexpr (SA_LSD_PROF != 0) {
            const uint64_t now = clock64();
            tacc[q] += now - tlast;
            tlast = now;
        }
    };
    while (t < tiles) {
        const uint64_t tb = t * TILE;
        const uint32_t valid = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);
        // rank in input order: items (j, lane) of wave w are its slice's
        // positions j * 64 + lane; dr = digit << 16 | rank in the wave's run
        uint32_t dr[ITEMS];
        uint16_t* wc = s_wcnt[wave];
        if constexpr (has_raw<Src>::value) {
            const uint32_t last = valid - 1;
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                const uint32_t le = wave * WTILE + j * kWave + lane;
                k[j] = src.finish(k[j], tb + (le < last ? le : last));
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const bool ok = le < valid;
            if (!XQ && next_hist && ok) atomicAdd(&s_nh[(uint32_t)(k[j] >> nshift) & nmask], 1u);
            const uint32_t d = ok ? (uint32_t)(k[j] >> shift) & mask : (uint32_t)RADIX;
            uint64_t peers = __ballot(ok);
            for (uint32_t b = 0; b < nbits; ++b) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bal = __ballot(bit);
                peers &= bit ? bal : ~bal;
            }
            const uint32_t cnt = ok ? (uint32_t)wc[d] : 0u;
            const uint32_t below = (uint32_t)__popcll(peers & lanemask_lt());
            if (ok && below == 0) wc[d] = (uint16_t)(cnt + (uint32_t)__popcll(peers));
            dr[j] = (d << 16) | (cnt + below);
        }
        __syncthreads();
        stamp(0);
        uint32_t tile_cnt = 0;
        if (dg < (uint32_t)RADIX) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                const uint32_t x = s_wcnt[w][dg];
                s_wcnt[w][dg] = (uint16_t)tile_cnt;
                tile_cnt += x;
            }
            st_store(&states[t * RADIX + dg], (t == t0 ? kStPrefix : kStAgg) | tag | tile_cnt);
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
        stamp(1);
        if (dg < (uint32_t)RADIX) {
            // (XQ: over the queue's own tiles, t0 first)
            const uint64_t excl =
                tile_lookback<RADIX, false, SA_LSD_LOOK>(states + t0 * RADIX, t - t0, dg, tile_cnt, tag, err);
            s_gofs[dg] = digit_base[dg] + (uint32_t)excl;
        }
        // the next tile's ticket only now (see k_split), its loads in flight
        // during the staging and the writes
        if (dg == 0) s_tile[par ^ 1u] = atomicAdd(ticket, 1u);
        __syncthreads();
        stamp(2);
        const uint64_t tn = t0 + (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[par ^ 1u]);
        uint64_t kn[ITEMS];
        uint32_t vn[ITEMS];
        load(tn < tiles ? tn : tiles - 1, kn, vn);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t d = dr[j] >> 16;
            if (d < (uint32_t)RADIX) {
                const uint32_t pos = s_start[d] + s_wcnt[wave][d] + (dr[j] & 0xFFFFu);
                s_keys[pos] = k[j];
                if constexpr (!PACKED) s_vals[pos] = v[j];
            }
        }
        __syncthreads();
        stamp(3);
        for (int i = dg; i < WAVES * RADIX / 2; i += BLOCK) wc32[i] = 0;   // the next tile ranks after a barrier
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t q = j * BLOCK + dg;
            if (q < valid) {
                const uint64_t key = s_keys[q];
                const uint32_t dd = (uint32_t)(key >> shift) & mask;
                const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
                if (g < n) {
                    out_keys[g] = key;
                    if constexpr (!PACKED) out_vals[g] = s_vals[q];
                    // XQ: the next pass's digit in the queue of this output position
                    if (XQ && next_hist) atomicAdd(&s_nh[qd.q(g) * kLsdMaxRadix + ((uint32_t)(key >> nshift) & nmask)], 1u);
                }
            }
        }
        __syncthreads();
        stamp(4);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            k[j] = kn[j];
            if constexpr (!PACKED) v[j] = vn[j];
        }
        t = tn;
        par ^= 1u;
    }
    if constexpr (SA_LSD_PROF != 0)
        if (dg == 0)
            for (int q = 0; q < 5; ++q) atomicAdd(prof + q, (unsigned long long)tacc[q]);
    if (next_hist) {
        __syncthreads();
        if constexpr (XQ) {
            for (uint32_t i = dg; i < (uint32_t)NH; i += BLOCK)
                if ((i & (kLsdMaxRadix - 1)) <= nmask && s_nh[i]) atomicAdd(&next_hist[i], s_nh[i]);
        } else {
            for (uint32_t i = dg; i <= nmask; i += BLOCK)
                if (s_nh[i]) atomicAdd(&next_hist[i], s_nh[i]);
        }
    }
}

// The reference schedule's first ranks (as k_init_rank_dense: rank[i] =
// dense code of text[i], manber_myers.c:88-92) with round 1's first-digit
// counts per XCD queue of its LSD passes: item i's key is rank[i] << w |
// rank[i + 1] (0 past the end, SrcRankPk), its digit (key >> dshift) & dmask,
// its queue qd.q(i) -- so round 1 reads no histogram pass (k_lsd_hist over
// n rank pairs).  A workgroup's 1024 positions per step lie in one queue but
// for the step that crosses a queue border; counts flushed per workgroup.
__global__ __launch_bounds__(kBlock) void k_init_rank_hist(const uint8_t* __restrict__ text, uint64_t n,
                                                           const uint16_t* __restrict__ code,
                                                           uint32_t* __restrict__ rank, uint32_t w, uint32_t dshift,
                                                           uint32_t dmask, QDiv qd, uint32_t* __restrict__ qh) {
    constexpr int RUN = 16;   // positions per thread and step: one 16-byte text load
    __shared__ uint16_t s_code[256];
    __shared__ uint32_t s_h[8 * kLsdMaxRadix];
    s_code[threadIdx.x] = code[threadIdx.x];
    for (uint32_t i = threadIdx.x; i < 8 * kLsdMaxRadix; i += kBlock) s_h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * RUN;
    for (uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * RUN; i < n; i += stride) {
        uint32_t r[RUN + 1];
        if (i + RUN + 1 <= n && (((uintptr_t)(text + i)) & 15) == 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(text + i);
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int y = 0; y < 4; ++y) r[4 * q + y] = s_code[(wv[q] >> (8 * y)) & 0xFFu];
            r[RUN] = s_code[text[i + RUN]];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<uint4*>(rank + i + 4 * q) = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
        } else {
#pragma unroll
            for (int j = 0; j <= RUN; ++j) r[j] = i + j < n ? (uint32_t)s_code[text[i + j]] : 0u;
            for (uint64_t j = i; j < n && j < i + RUN; ++j) rank[j] = r[j - i];
        }
        // one queue for the thread's 16 positions unless they cross a border
        const uint32_t q0 = qd.q(i), q1 = qd.q(i + RUN - 1);
#pragma unroll
        for (int j = 0; j < RUN; ++j)
            if (i + j < n) {
                const uint32_t q = q0 == q1 ? q0 : qd.q(i + j);
                atomicAdd(&s_h[q * kLsdMaxRadix + ((((r[j] << w) | r[j + 1]) >> dshift) & dmask)], 1u);
            }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 8 * kLsdMaxRadix; i += kBlock)
        if (s_h[i]) atomicAdd(&qh[i], s_h[i]);
}

// SA from the sorted items of a PACKED final round
__global__ __launch_bounds__(kBlock) void k_items_to_sa(const uint64_t* __restrict__ items, uint64_t n,
                                                        uint32_t ib, uint32_t* __restrict__ sa) {
    const uint64_t m = (1ull << ib) - 1ull;
    for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (uint64_t)gridDim.x * kBlock)
        sa[e] = (uint32_t)(items[e] & m);
}

}  // namespace sa
