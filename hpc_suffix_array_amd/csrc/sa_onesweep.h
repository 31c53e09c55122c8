// sa_onesweep.h -- single-pass LSD radix passes with decoupled look-back
// (the per-pass sort of one doubling round, replacing the two stable
// counting passes of radix_sort_suffixes_seq, manber_myers.c:37-48).
//
// Per sort:
//   k_global_hist  one read of the pass-0 source -> digit totals of EVERY
//                  pass (the multiset of keys is the same in all passes)
//                  (k_pack_text computes them itself for the packed round 1)
//   k_digit_base   exclusive scan of each pass's 256 totals
// Per pass (one launch, one tile per workgroup, tile ids from an atomic
// ticket so a tile only ever waits on tiles that are already running):
//   1. load the tile, rank it stably per wave (match-any from ballots)
//   2. publish the tile's per-digit count (AGGREGATE) in its state words
//   3. look back over predecessors, summing AGGREGATEs until an INCLUSIVE
//      prefix; publish this tile's INCLUSIVE prefix
//   4. stage the tile digit-sorted in LDS, write each digit run to
//      digit_base[d] + exclusive prefix + offset in run
// State words are 64-bit agent-scope atomics holding {status, epoch, count}:
// the data is its own flag (MI355X_MICROARCH.md "R2" granule), so no fences;
// the epoch makes a stale word from an earlier pass read as "not ready".
#pragma once
#include "sa_kernels.h"

namespace sa {

constexpr uint64_t kStAgg = 1ull << 62;
constexpr uint64_t kStPrefix = 2ull << 62;
constexpr uint32_t kEpochBits = 14;
constexpr uint32_t kEpochMask = (1u << kEpochBits) - 1u;
constexpr uint64_t kCountMask = (1ull << 48) - 1ull;
constexpr uint32_t kMaxPasses = 8;
constexpr uint32_t kSpinLimit = 1u << 26;
constexpr int kOsBlock = 1024;   // product shape of k_onesweep
constexpr int kOsItems = 4;

__device__ __forceinline__ uint64_t st_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Adds one wave's keys (one per active lane, the active lanes a prefix of
// the wave) to the LDS digit histograms: per pass, only the first lane of
// each run of equal digits across neighbouring lanes adds the run's length.
// Random digits cost one atomic per lane as before; sorted-like keys (the
// high digits of a degenerate text's unsorted-set rounds) one per run instead
// of 64 colliding atomics on one bin (k_materialize 13.1 ms per 2^30 keys).
__device__ __forceinline__ void hist_add_runs(uint32_t (*s_h)[kRadix], uint64_t k, uint32_t passes) {
    const uint32_t lane = lane_id();
    const uint32_t nact = (uint32_t)__popcll(__ballot(1));
    const uint64_t above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t d = (uint32_t)(k >> (8 * p)) & 0xFFu;
        const uint32_t dl = __shfl_up(d, 1, 64);
        const bool head = lane == 0 || dl != d;
        const uint64_t hm = __ballot(head) & above;
        const uint32_t next = hm ? (uint32_t)__ffsll((long long)hm) - 1u : nact;
        if (head) atomicAdd(&s_h[p][d], next - lane);
    }
}

// digit histograms of all `passes` 8-bit digits of the source keys
template <class Src>
__global__ __launch_bounds__(kBlock) void k_global_hist(Src src, uint64_t n, uint32_t passes,
                                                        uint32_t* __restrict__ ghist) {
    __shared__ uint32_t s_h[kMaxPasses][kRadix];
    for (int i = threadIdx.x; i < (int)(kMaxPasses * kRadix); i += kBlock) (&s_h[0][0])[i] = 0;
    __syncthreads();
    for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (uint64_t)gridDim.x * kBlock) {
        hist_add_runs(s_h, src.key(e), passes);
    }
    __syncthreads();
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t v = s_h[p][threadIdx.x];
        if (v) atomicAdd(&ghist[p * kRadix + threadIdx.x], v);
    }
}

// keys of a generated source written once (an unsorted-set round's keys cost
// a binary search each: computing them in both the histogram and the first
// scatter doubled that), with the digit totals of every pass
template <class Src>
__global__ __launch_bounds__(kBlock) void k_materialize(Src src, uint64_t n, uint32_t passes,
                                                        uint64_t* __restrict__ keys, uint32_t* __restrict__ ghist) {
    __shared__ uint32_t s_h[kMaxPasses][kRadix];
    for (int i = threadIdx.x; i < (int)(kMaxPasses * kRadix); i += kBlock) (&s_h[0][0])[i] = 0;
    __syncthreads();
    for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (uint64_t)gridDim.x * kBlock) {
        const uint64_t k = src.key(e);
        keys[e] = k;
        hist_add_runs(s_h, k, passes);
    }
    __syncthreads();
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t v = s_h[p][threadIdx.x];
        if (v) atomicAdd(&ghist[p * kRadix + threadIdx.x], v);
    }
}

// base[d] = sum of ghist[d'] for d' < d over `bins` <= 1024 entries (a pass
// of RBITS > 8 spans several 256-entry rows of the ghist / base layout)
__global__ __launch_bounds__(1024) void k_digit_base_wide(const uint32_t* __restrict__ ghist, uint32_t bins,
                                                          uint32_t* __restrict__ base) {
    __shared__ uint32_t s_tmp[16];
    const uint32_t i = threadIdx.x;
    const uint32_t x = i < bins ? ghist[i] : 0u;
    const uint32_t inc = wave_inclusive_sum(x);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t w = 0; w < wave_id(); ++w) off += s_tmp[w];
    if (i < bins) base[i] = off + inc - x;
}

// base[p][d] = sum of ghist[p][d'] for d' < d; one workgroup per pass
__global__ __launch_bounds__(kBlock) void k_digit_base(const uint32_t* __restrict__ ghist,
                                                       uint32_t* __restrict__ base) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint32_t p = blockIdx.x;
    base[p * kRadix + threadIdx.x] = block_exclusive_sum(ghist[p * kRadix + threadIdx.x], s_tmp, nullptr);
}

// RBITS: digit width (8, or 9 for the bucketed first round's high pass);
// digit_base and states are laid out with 1 << RBITS entries per tile.
template <class Src, int BLOCK, int ITEMS, int RBITS = 8>
__global__ __launch_bounds__(BLOCK) void k_onesweep(Src src, uint64_t n, uint32_t shift, uint32_t nbits,
                                                    const uint32_t* __restrict__ digit_base,
                                                    uint64_t* __restrict__ states, uint32_t* __restrict__ ticket,
                                                    uint32_t epoch, uint64_t* __restrict__ out_keys,
                                                    uint32_t* __restrict__ out_vals, uint32_t* __restrict__ err) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int RADIX = 1 << RBITS;
    constexpr int RWAVES = RADIX / kWave;   // waves holding one digit per thread
    static_assert(BLOCK >= RADIX, "one thread per digit");
    static_assert(TILE <= 65535, "16-bit tile offsets");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_vals[TILE];
    __shared__ uint16_t s_wcnt[WAVES][RADIX];   // per-wave digit counts, then wave offsets
    __shared__ uint16_t s_start[RADIX];         // digit run starts in the tile
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile;

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t mask = (1u << nbits) - 1u;
    if (threadIdx.x == 0) {
        uint32_t tk = atomicAdd(ticket, 1u);
        s_tile = tk;
    }
    for (int i = threadIdx.x; i < WAVES * RADIX; i += BLOCK) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t t = s_tile;
    const uint64_t tb = t * TILE;
    const uint32_t valid = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);

    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    uint32_t d[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint32_t le = wave * WTILE + j * kWave + lane;
        const bool ok = le < valid;
        k[j] = ok ? src.key(tb + le) : 0ull;
        v[j] = ok ? src.val(tb + le) : 0u;
        d[j] = ok ? src_digit(src, k[j], shift, mask, 0) : RADIX;
    }
    uint32_t r[ITEMS];
    uint16_t* wc = s_wcnt[wave];
    {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const bool ok = d[j] < (uint32_t)RADIX;
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
            if (ok && below == 0) wc[d[j]] = (uint16_t)(cnt + (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();

    const uint32_t dg = threadIdx.x;   // digit owned by this thread (dg < RADIX)
    uint32_t tile_cnt = 0;
    if (dg < (uint32_t)RADIX) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const uint32_t x = s_wcnt[w][dg];
            s_wcnt[w][dg] = (uint16_t)tile_cnt;
            tile_cnt += x;
        }
        const uint64_t tag = (uint64_t)(epoch & kEpochMask) << 48;
        st_store(&states[t * RADIX + dg], (t == 0 ? kStPrefix : kStAgg) | tag | tile_cnt);
    }
    // tile layout: exclusive scan of the per-digit counts (threads >= 256 add 0)
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
    // look back (one thread per digit)
    if (dg < (uint32_t)RADIX) {
        uint64_t excl = 0;
        if (t > 0) {
            // read kLook predecessors per step (independent loads: one
            // fabric round trip per kLook tiles instead of per tile)
            constexpr int kLook = 4;
            int64_t tp = (int64_t)t - 1;
            uint32_t spins = 0;
            const uint32_t ep_now = epoch & kEpochMask;
            while (tp >= 0) {
                uint64_t sv[kLook];
#pragma unroll
                for (int i = 0; i < kLook; ++i)
                    sv[i] = (tp - i >= 0) ? st_load(&states[(uint64_t)(tp - i) * RADIX + dg]) : 0ull;
                int used = 0;
                bool done = false;
#pragma unroll
                for (int i = 0; i < kLook; ++i) {
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
            const uint64_t tag = (uint64_t)(epoch & kEpochMask) << 48;
            st_store(&states[t * RADIX + dg], kStPrefix | tag | ((excl + tile_cnt) & kCountMask));
        }
        s_gofs[dg] = digit_base[dg] + (uint32_t)excl;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (d[j] < (uint32_t)RADIX) {
            const uint32_t pos = s_start[d[j]] + s_wcnt[wave][d[j]] + r[j];
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
            const uint32_t dd = src_digit(src, key, shift, mask, 0);
            const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
            if (g < n) {
                out_keys[g] = key;
                out_vals[g] = s_vals[q];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Chunked stable scatter with a one-tile register prefetch (reduce-then-scan
// radix, the alternative to k_onesweep): the workgroup walks its chunk's
// tiles in order, so its running per-digit offsets (from k_hist + k_scan_rows)
// replace the look-back, and the next tile's loads are in flight while the
// current tile is ranked, staged and written.  BLOCK x ITEMS = kTile, so the
// chunking and the histogram layout are those of k_hist.
// ---------------------------------------------------------------------------
template <class Src, int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK, BLOCK / 128) void k_scatter_pipe(Src src, Chunking ch, uint32_t shift,
                                                                    uint32_t nbits,
                                                                    const uint32_t* __restrict__ hist,
                                                                    const uint32_t* __restrict__ totals,
                                                                    uint64_t* __restrict__ out_keys,
                                                                    uint32_t* __restrict__ out_vals) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int WTILE = kWave * ITEMS;
    static_assert(TILE == kTile, "chunking and histograms assume kTile");
    static_assert(BLOCK >= kRadix, "one thread per digit");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_vals[TILE];
    __shared__ uint16_t s_wcnt[WAVES][kRadix];
    __shared__ uint16_t s_start[kRadix];
    __shared__ uint32_t s_run[kRadix];
    __shared__ uint32_t s_tmp[kWaves];

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t mask = (1u << nbits) - 1u;
    const uint32_t c = blockIdx.x;
    const uint32_t dg = threadIdx.x;
    // running global offset of each digit for this chunk
    {
        const uint32_t x = dg < (uint32_t)kRadix ? totals[dg] : 0u;
        const uint32_t inc = wave_inclusive_sum(x);
        if (lane == kWave - 1 && wave < (uint32_t)kWaves) s_tmp[wave] = inc;
        __syncthreads();
        uint32_t off = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) off += (w < (int)wave) ? s_tmp[w] : 0u;
        if (dg < (uint32_t)kRadix) s_run[dg] = off + inc - x + hist[(uint64_t)dg * ch.chunks + c];
    }
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    uint64_t k[ITEMS], kn[ITEMS];
    uint32_t v[ITEMS], vn[ITEMS];
    auto load = [&](uint64_t tb, uint64_t* kk, uint32_t* vv) {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t e = tb + wave * WTILE + j * kWave + lane;
            const bool ok = e < e1;
            kk[j] = ok ? src.key(e) : 0ull;
            vv[j] = ok ? src.val(e) : 0u;
        }
    };
    if (e0 < e1) load(e0, k, v);
    for (uint64_t tb = e0; tb < e1; tb += TILE) {
        const uint32_t valid = (uint32_t)((e1 - tb) < (uint64_t)TILE ? (e1 - tb) : (uint64_t)TILE);
        if (tb + TILE < e1) load(tb + TILE, kn, vn);      // in flight during this tile
        for (int i = threadIdx.x; i < WAVES * kRadix; i += BLOCK) (&s_wcnt[0][0])[i] = 0;
        __syncthreads();
        uint32_t d[ITEMS], r[ITEMS];
        uint16_t* wc = s_wcnt[wave];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const bool ok = le < valid;
            d[j] = ok ? (uint32_t)(k[j] >> shift) & mask : kRadix;
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
            if (ok && below == 0) wc[d[j]] = (uint16_t)(cnt + (uint32_t)__popcll(peers));
        }
        __syncthreads();
        uint32_t tile_cnt = 0;
        if (dg < (uint32_t)kRadix) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                const uint32_t x = s_wcnt[w][dg];
                s_wcnt[w][dg] = (uint16_t)tile_cnt;
                tile_cnt += x;
            }
        }
        {
            const uint32_t x = (dg < (uint32_t)kRadix) ? tile_cnt : 0u;
            const uint32_t inc = wave_inclusive_sum(x);
            if (lane == kWave - 1 && wave < (uint32_t)kWaves) s_tmp[wave] = inc;
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) off += (w < (int)wave) ? s_tmp[w] : 0u;
            if (dg < (uint32_t)kRadix) s_start[dg] = (uint16_t)(off + inc - x);
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            if (d[j] < (uint32_t)kRadix) {
                const uint32_t pos = s_start[d[j]] + s_wcnt[wave][d[j]] + r[j];
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
                const uint64_t g = (uint64_t)s_run[dd] + (q - s_start[dd]);
                if (g < ch.n) {
                    out_keys[g] = key;
                    out_vals[g] = s_vals[q];
                }
            }
        }
        __syncthreads();
        if (dg < (uint32_t)kRadix) s_run[dg] += tile_cnt;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            k[j] = kn[j];
            v[j] = vn[j];
        }
    }
}

}  // namespace sa
