// sa_split.h -- the two bucket passes of the bucketed first round
// (sa_round1.h) as persistent single-pass scatters: the counting passes of
// radix_sort_suffixes_seq (manber_myers.c:15-34) over the bucket digits.
//
// Differences from k_onesweep (sa_onesweep.h), measured in
// microbench_radix.hip (2^30 pairs, 8-bit digits: 10.3 -> 7.1 ms):
//   * 8192-pair tiles (1024 x 8): half the look-back work and state traffic,
//     digit runs twice as long (fewer partial-line writes);
//   * ranks from one LDS atomic per pair instead of per-wave match-any
//     ballots; the first pass need not be stable (the local sort orders each
//     window by (key, suffix) completely), the second must keep the order of
//     the first pass's digit only, which it does by ranking one previous
//     digit value at a time (a tile of bucket-ordered input spans one or two
//     of them), falling back to stable ballots when a tile spans more;
//   * persistent workgroups that take tiles from the ticket in order and
//     issue the next tile's loads right after ranking the current one, so
//     they are in flight during the look-back, the LDS staging and the writes.
// Tile ids still come from the ticket, so a tile waits only on tiles whose
// workgroups already run: a workgroup's prefetched tile is always later than
// its current one, hence the smallest unfinished tile is always being
// processed and the look-back cannot deadlock.
#pragma once
#include <type_traits>
#include "sa_bucket.h"
#include "sa_onesweep.h"

// When the bucket passes take the next tile's ticket (A/B at 2^30 DNA):
// pass 1 takes it after the digit staging and loads the next tile's text
// after the claims (the loads right behind the ticket: 5.34 -> 5.71 ms,
// slower); pass 2 takes it at the start of the unit, not after the claims
// (5.885 -> 5.83 ms)
// diagnostic: per-phase clock64 spans of k_split_seg printed by two
// workgroups (scatter 36 %, write 22 %, base wait 18 %, ranking 12 %, claims
// 12 % at 2^30 DNA).  Batching the per-item LDS reads of the scatter and
// write loops (one wait instead of one per item) raised VGPR spills 4 -> 17
// and made both passes slower (5.9 -> 7.2 ms, 5.5 -> 6.3 ms): reverted.
// Letting the second pass's stores stay in flight into the next unit's
// ranking (unconditional stores + an explicit wait after the prologue's
// loads, so the loop-top wait counts only loads; the early ticket's atomic
// kept off the compiler's atomic optimizer) was slower too (5.91 -> 6.0-6.3
// ms, profiles/r02_ah_ab_seg_nodrain_reverted.txt): the pass is not waiting
// on its store acknowledgements.
// First-pass writes unconditional in count (a slot past the tile's pairs
// re-writing the last pair) so that the next tile's staging would not wait
// for them: 4.09 -> 4.08 ms, within noise (profiles/r02_ar_ab_text_staging.txt;
// the loop-top wait stays vmcnt(0) for the claims' branches anyway), dropped.
// Packed items staged whole in the second pass (digit from the item's top
// bits, no 16-bit digit array): 4.646 -> 4.650 ms, and 14 pairs per lane with
// the LDS so saved spill (5.16 ms): profiles/r02_au_ab_pk_digit_in_item.txt.
// The first pass's early ticket kept off the atomic optimizer and held in a
// register until the claims (no wait for it, nor drain of wave 0, before the
// staging barrier) was slower: 4.09 -> 4.50 ms
// (profiles/r02_ax_ab_text_ticket_deferred.txt).
// Reading every pair's LDS slot before the staging writes (no read-wait-write
// chain per pair) was slower in the first pass (4.19 -> 4.28 ms) and equal in
// the second (profiles/r02_ao_ab_batched_slots_reverted.txt).
// Claims issued before the LDS staging and waited for after it, then the
// segment count and base wait (the order of the first pass's late claims):
// 4.915 -> 4.95 ms (profiles/r02_am_ab_seg_late_claims_reverted.txt; the
// publish branch before the writes made the compiler wait for every store).
#ifndef SA_SEG_PROF
#define SA_SEG_PROF 0
#endif
#ifndef SA_TEXT_PROF
#define SA_TEXT_PROF 0
#endif

namespace sa {

constexpr int kSpBlock = 1024;
constexpr int kSpItems = 8;
constexpr int kSpTile = kSpBlock * kSpItems;   // 8192 pairs
constexpr int kSpWaves = kSpBlock / kWave;

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, kWave));
    return x;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, kWave));
    return x;
}

// Decoupled look-back of digit dg for tile t (the tile's AGGREGATE is
// already published): sums predecessors' counts, kLook state words per
// step, until an INCLUSIVE prefix; publishes this tile's own prefix.
template <int RADIX, bool PROF = false, int kLook = 4>
__device__ __forceinline__ uint64_t tile_lookback(uint64_t* __restrict__ states, uint64_t t, uint32_t dg,
                                                  uint32_t tile_cnt, uint64_t tag, uint32_t* __restrict__ err,
                                                  uint32_t* steps = nullptr) {
    uint64_t excl = 0;
    if (t == 0) return 0;
    const uint32_t ep_now = (uint32_t)(tag >> 48) & kEpochMask;
    int64_t tp = (int64_t)t - 1;
    uint32_t spins = 0;
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
        if constexpr (PROF) {
            steps[0] += 1;
            steps[1] += used == 0;
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
    return excl;
}

// One pass over digit (src.digit(key, shift, RADIX - 1)).  STABLE: pairs of
// equal digit keep the order of their previous-pass digit
// src.digit(key, lshift, lmask) (the input is ordered by it); otherwise their
// order is arbitrary.
template <class Src, int RBITS, bool STABLE, bool PROF = false, int ITEMS = kSpItems>
__global__ __launch_bounds__(kSpBlock) void k_split(Src src, uint64_t n, uint32_t shift, uint32_t lshift,
                                                    uint32_t lmask, const uint32_t* __restrict__ digit_base,
                                                    uint64_t* __restrict__ states, uint32_t* __restrict__ ticket,
                                                    uint32_t epoch, uint64_t* __restrict__ out_keys,
                                                    uint32_t* __restrict__ out_vals, uint32_t* __restrict__ err) {
    constexpr int RADIX = 1 << RBITS;
    constexpr int RWAVES = RADIX / kWave;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int TILE = kSpBlock * ITEMS;
    static_assert(TILE <= 16384, "ranks in 14 bits, run starts in 16");
    static_assert(kSpBlock >= RADIX, "one thread per digit");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_vals[TILE];
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile[2];
    __shared__ uint32_t s_nx[3];   // STABLE: the next previous-digit value to rank (rotating)

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    const uint32_t mask = RADIX - 1;
    const uint64_t tiles = (n + TILE - 1) / TILE;
    const uint64_t tag = (uint64_t)(epoch & kEpochMask) << 48;
    if (dg == 0) {
        s_tile[0] = atomicAdd(ticket, 1u);
        s_nx[0] = s_nx[1] = s_nx[2] = ~0u;
    }
    if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;
    __syncthreads();
    uint64_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[0]);
    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    // clamped, unpredicated loads (pairs past the end are never ranked)
    // (tile numbers come through LDS: readfirstlane keeps the tile base in
    // scalar registers, so each load is a scalar base + 32-bit lane offset)
    auto load = [&](uint64_t tt, uint64_t* kk, uint32_t* vv) {
        const uint64_t tb = tt * TILE;
        const uint32_t last = (uint32_t)min(n - 1 - tb, (uint64_t)(TILE - 1));
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const uint64_t e = tb + (le < last ? le : last);
            kk[j] = src.key(e);
            vv[j] = src.val(e);
        }
    };
    if (t < tiles) load(t, k, v);
    uint32_t par = 0;
    // PROF (microbenchmarks only): per-phase clock64 spans of thread 0
    // accumulated into err[2..11] as u64
    uint64_t tacc[5] = {0, 0, 0, 0, 0}, tlast = PROF ? clock64() : 0;
    uint32_t lbsteps[2] = {0, 0};   // look-back steps, steps that found nothing ready
    auto stamp = [&](int q) {
        if constexpr (PROF) {
            const uint64_t now = clock64();
            tacc[q] += now - tlast;
            tlast = now;
        }
    };
    while (t < tiles) {
        const uint64_t tb = t * TILE;
        const uint32_t valid = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);
        // dr[j] = digit << 16 | rank in the tile's digit run (< 2^14; digit RADIX: no pair)
        uint32_t dr[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            dr[j] = (le < valid ? src_digit(src, k[j], shift, mask, 0) : (uint32_t)RADIX) << 16;
        }
        if constexpr (!STABLE) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j)
                if ((dr[j] >> 16) < (uint32_t)RADIX) dr[j] |= atomicAdd(&s_cnt[dr[j] >> 16], 1u);
            __syncthreads();
        } else {
            // ranks in rounds, one previous-digit value per round, in
            // increasing order and only the values present in the tile: all
            // pairs of value l take their ranks before any pair of a larger
            // value.  Round r also finds the next value (its minimum over the
            // block lands in s_nx[r % 3]; thread 0 clears the slot round r + 1
            // will use, last read before round r - 1's barrier).  Round 0 only
            // finds the smallest value.  A tile of bucket-ordered input holds
            // one or two values, so typically two or three rounds.
            uint32_t cur = ~0u;
            for (uint32_t r = 0;; ++r) {
                uint32_t nx = ~0u;
#pragma unroll
                for (int j = 0; j < ITEMS; ++j) {
                    if ((dr[j] >> 16) < (uint32_t)RADIX) {
                        const uint32_t l = src_digit(src, k[j], lshift, lmask, 0);
                        if (l == cur) dr[j] |= atomicAdd(&s_cnt[dr[j] >> 16], 1u);
                        else if ((cur == ~0u || l > cur) && l < nx) nx = l;
                    }
                }
                nx = wave_min_u32(nx);
                if (lane == 0 && nx != ~0u) atomicMin(&s_nx[r % 3], nx);
                if (dg == 0) s_nx[(r + 1) % 3] = ~0u;
                __syncthreads();
                cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_nx[r % 3]);
                if (cur == ~0u) break;
            }
        }
        stamp(0);
        uint32_t tile_cnt = 0;
        if (dg < (uint32_t)RADIX) {
            tile_cnt = s_cnt[dg];
            st_store(&states[t * RADIX + dg], (t == 0 ? kStPrefix : kStAgg) | tag | tile_cnt);
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
            const uint64_t excl = tile_lookback<RADIX, PROF>(states, t, dg, tile_cnt, tag, err, lbsteps);
            s_gofs[dg] = digit_base[dg] + (uint32_t)excl;
        }
        // the next tile: its ticket is taken only now (a tile is processed
        // soon after its ticket, so successors seldom find it unpublished),
        // its loads are in flight during the staging and the writes (past
        // the last tile: the last again, unused; one program point for every
        // wave, so nothing waits for them at a branch join)
        if (dg == 0) s_tile[par ^ 1u] = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint64_t tn = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[par ^ 1u]);
        uint64_t kn[ITEMS];
        uint32_t vn[ITEMS];
        load(tn < tiles ? tn : tiles - 1, kn, vn);
        stamp(2);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t d = dr[j] >> 16;
            if (d < (uint32_t)RADIX) {
                const uint32_t pos = s_start[d] + (dr[j] & 0x3FFFu);
                s_keys[pos] = k[j];
                s_vals[pos] = v[j];
            }
        }
        __syncthreads();
        if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;   // the next tile's atomics come after the next barrier
        if (STABLE && dg < 3u) s_nx[dg] = ~0u;
        stamp(3);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t q = j * kSpBlock + dg;
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
        __syncthreads();
        stamp(4);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            k[j] = kn[j];
            v[j] = vn[j];
        }
        t = tn;
        par ^= 1u;
    }
    if constexpr (PROF) {
        if (dg == 0)
            for (int q = 0; q < 5; ++q) atomicAdd(reinterpret_cast<unsigned long long*>(err + 2) + q, tacc[q]);
        if (dg < (uint32_t)RADIX) {
            atomicAdd(reinterpret_cast<unsigned long long*>(err + 12), (unsigned long long)lbsteps[0]);
            atomicAdd(reinterpret_cast<unsigned long long*>(err + 14), (unsigned long long)lbsteps[1]);
        }
    }
}

// ---------------------------------------------------------------------------
// The first bucket pass straight from the text (no key1 round trip through
// HBM): each lane computes key1 of ITEMS consecutive positions (Horner for
// the first, rolling updates of D and of the remainder for the rest) from
// dense digits staged in LDS, and the pair (key1, position) is scattered by
// the bucket's low kLoBits.  The order within a digit is arbitrary (LDS
// atomics), so the lane -> position mapping is free, and so is the order of
// the tiles within a digit: each tile claims its place from a per-digit
// cursor (no look-back).  The digit totals come from k_bucket_hist; the
// second pass's totals are counted here.  The next tile's text (the tile +
// a K - 1 byte halo, as 32-bit words) is loaded while the current one is
// staged and written.
// ---------------------------------------------------------------------------
// Launched as BLOCK 512 x 12 items, two workgroups per CU (SA_TEXT_BLOCK):
// one workgroup's scatter overlaps the other's staging and barriers, 4.09 ->
// 3.62 ms at 1 GiB DNA over one 1024 x 12 workgroup per CU (an early version
// measured the opposite, 5.5 -> 6.3 ms; 256 x 12: 6.6 ms, 512 x 8: 5.0 ms)
// POW2: sigma a power of two -- D and the remainder roll by shifts and masks
// and the bucket is a bit field of D (no multiplications)
// Bucket range (range-partitioned build, sa_dist.h): only positions whose
// bucket lies in [blo, bhi) are kept, digits of the local bucket bk - blo;
// m = the number kept (the output's length).  One GPU: [0, 2^bb), m = n.
// PK8 (POW2): each pair leaves as ONE 64-bit
// item -- the second pass's digit (the local bucket's high hb bits) on top, then
// key1 below its bucket (key1 - Dmin(bucket) << rb: the bits of D under the
// bucket and low) and the position in the low ib bits, so the pass writes 8
// bytes per suffix instead of 12 (key1 + position) and the second pass reads
// 8 (SrcPk8).  Needs hb + (lg sigma^s - bb + rb) + ib <= 64 (plan_pk8).
// DNA: the text's alphabet is exactly {A, C, G, T}; their dense digits
// 0..3 are ((b >> 1) ^ (b >> 2)) & 3 of the byte b (0x41 0x43 0x47 0x54 ->
// 0 1 2 3), four bytes of a word at once, instead of four LDS byte-map reads
#ifndef SA_DNA_SWAR
#define SA_DNA_SWAR 1
#endif
// SA_TEXT_FULL: whole tiles of the whole bucket range take the key loop
// without per-item tests (its LDS atomics unpredicated): 3.54 -> 3.27-3.37
// ms at 1 GiB DNA; the staging and write loops alone made no difference
// (profiles/r04_n_ab_full_tiles.txt)
#ifndef SA_TEXT_IDENT
#define SA_TEXT_IDENT 1   // sigma = 256: keys from byte windows (k_split_text<.., IDENT>)
#endif
#ifndef SA_TEXT_FULL
#define SA_TEXT_FULL 1
#endif
// IDENT (sigma = 256, every byte present, K <= 8): the dense digit is the
// byte itself -- staged without the byte map, and each position's D and
// remainder are bit fields of the big-endian 8-byte window at it (two
// alignbyte + bswap of the lane's staged words) instead of a roll by bytes
// R32 (!POW2, sigma^R < 2^32: alnum, ascii127): the remainder rolls in 32
// bits (one v_mul_lo_u32 per step instead of a 64-bit multiply)
template <int ITEMS, int BLOCK = kSpBlock, bool POW2 = false, bool PK8 = false, bool DNA = false, bool IDENT = false,
          bool R32 = false>
__global__ __launch_bounds__(BLOCK, 2048 / BLOCK) void k_split_text(const uint8_t* __restrict__ text, uint64_t n,
                                                         const uint16_t* __restrict__ code, BucketSpec b,
                                                         const uint32_t* __restrict__ digit_base,
                                                         uint32_t* __restrict__ ticket, uint64_t* __restrict__ out_keys,
                                                         uint32_t* __restrict__ out_vals,
                                                         uint32_t* __restrict__ ghist_hi, uint32_t* __restrict__ cursor,
                                                         uint64_t m, uint32_t blo, uint32_t bhi,
                                                         const uint32_t* __restrict__ seg_end = nullptr,
                                                         uint32_t* __restrict__ ovf = nullptr, uint32_t pk_hb = 0,
                                                         uint32_t pk_ib = 0, uint32_t stripes = 1) {
    // stripes > 1 (padded segments only): digit d's segment is cut into
    // `stripes` equal sub-segments and workgroup w claims in sub-segment
    // w % stripes from its own cursor cursor[(w % stripes) * RADIX + d]:
    // device-scope atomics on one address serialise at ~19 ns each
    // (microbench_claims.hip), and 256 cursors shared by every tile took a
    // claim per tile and digit.  1 GiB DNA, interleaved A/B: 1 stripe 4.01 /
    // 4.02 ms, 8 stripes 3.70 / 3.70 (tiles assigned statically instead of
    // by the ticket: 3.80 / 3.91; 2 or 4 stripes static 4.16 / 4.22).
    // PK8 over a non-power-of-two alphabet (NP2): key1 below its bucket is
    // key1 - (Dmin(b) << rb), D - Dmin(b) from the bucket's fraction of D cmul
    // (a per-item gather of a table of Dmin(b) made the pass 4.4 ->
    // 7.4 ms at 1 GiB alnum: profiles/r06_k_ab_alnum_no_eonly_no_pk8.txt)
    constexpr bool NP2 = PK8 && !POW2;
    constexpr int RADIX = kLoRadix;
    constexpr int RWAVES = RADIX / kWave;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int kHalo = kMaxK;                        // >= K - 1 bytes past the tile
    constexpr int NW = (TILE + kHalo) / 4;              // staged text words
    constexpr int WPT = (NW + BLOCK - 1) / BLOCK; // per lane
    static_assert(ITEMS % 4 == 0 && kHalo % 4 == 0 && TILE <= 65535, "word staging, 16-bit tile offsets");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint16_t s_idx[TILE];                    // tile offset; PK8: the pair's digit
    __shared__ uint32_t s_dcw[NW + 8];                  // dense digits, 4 per word (0 past the end; + slack)
    // DNA: the digits packed 2 bits each, one byte per staged word (the first
    // digit on top), so a lane's 32 symbols from l0 are three word reads and
    // each position's key1 a shift of that window (no Horner start, no
    // per-position byte extraction); the host launches it when K + ITEMS - 1 <= 32
    __shared__ uint32_t s_pkw[DNA ? (NW + 3) / 4 + 4 : 1];
    __shared__ uint8_t s_map[256];
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile[2];
    __shared__ uint32_t s_kept;
    __shared__ uint32_t s_hhi[1024];   // the second pass's digit totals (local bucket >> kLoBits)
    __shared__ uint32_t s_gend[RADIX]; // padded segments: the end of digit d's segment
    const uint8_t* s_dc = reinterpret_cast<const uint8_t*>(s_dcw);
    const uint32_t bspan = bhi - blo;
    bool over = false;

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    const uint64_t tiles = (n + TILE - 1) / TILE;
    const uint32_t K = b.s + b.R;
    const uint32_t stripe = blockIdx.x % stripes;
    uint32_t sbase = 0;               // this workgroup's sub-segment start in digit dg
    for (uint32_t i = dg; i < 1024u; i += BLOCK) s_hhi[i] = 0;
    if (seg_end && dg < (uint32_t)RADIX) {
        const uint32_t lo = digit_base[dg], hi = seg_end[dg], sc = (hi - lo) / stripes;
        sbase = lo + stripe * sc;
        s_gend[dg] = stripe + 1 == stripes ? hi : sbase + sc;
    }
    cursor += stripe * RADIX;
    if (dg < 256u) {
        const uint32_t cv = code[dg];
        s_map[dg] = (uint8_t)(cv ? cv - 1u : 0u);
    }
    if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;
    if (dg == 0) s_tile[0] = atomicAdd(ticket, 1u);
    __syncthreads();
    uint64_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[0]);
    // raw text words dg, dg + 1024, ... of the tile + halo; bytes at or past
    // n are never read
    auto load4 = [&](uint64_t pos) -> uint32_t {
        if (pos + 4 <= n && (((uintptr_t)(text + pos)) & 3) == 0) return *reinterpret_cast<const uint32_t*>(text + pos);
        uint32_t w = 0;
        for (int q = 0; q < 4; ++q)
            if (pos + q < n) w |= (uint32_t)text[pos + q] << (8 * q);
        return w;
    };
    uint32_t raw[WPT];
    auto load = [&](uint64_t tt) {
        const uint64_t tb = tt * TILE;
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
            // words past NW (unused) re-read word NW - 1: no zero written
            // into a register a load may still be filling
            const uint32_t w = dg + i * BLOCK;
            raw[i] = load4(tb + 4ull * (w < (uint32_t)NW ? w : (uint32_t)NW - 1u));
        }
    };
    if (t < tiles) load(t);
    uint32_t par = 0;
    // tile-level range tests as 32-bit tile-index compares (scalar): in 64
    // bits they went to VALU with a hoisted 64-bit constant that spilled to
    // scratch, and every reload waited for the previous tile's stores
    const uint32_t t_whole = n >= 4ull * NW ? (uint32_t)((n - 4ull * NW) / TILE + 1) : 0u;   // tb + 4 NW <= n
    const uint32_t t_int = n >= (uint64_t)TILE + K ? (uint32_t)((n - TILE - K) / TILE + 1) : 0u;   // tb + TILE + K <= n
    const uint32_t t_last = (uint32_t)(tiles - 1);
#if SA_TEXT_PROF
    // diagnostic build (-DSA_TEXT_PROF=1): clock64 spans of thread 0 per phase
    uint64_t pacc[5] = {0, 0, 0, 0, 0}, plast = clock64();
#define TEXT_STAMP(k)                               \
    if (dg == 0) {                                  \
        const uint64_t now_ = clock64();            \
        pacc[k] += now_ - plast;                    \
        plast = now_;                               \
    }
#else
#define TEXT_STAMP(k)
#endif
    while (t < tiles) {
        const uint64_t tb = t * TILE;
        const uint32_t valid = (uint32_t)t < t_last ? (uint32_t)TILE : (uint32_t)(n - tb);
        // dense digits (0 past the end); a tile whose staged words lie inside
        // the text maps its four bytes with four independent LDS reads (the
        // per-byte bounds test made them a chain of branches and waits)
        const bool whole = (uint32_t)t < t_whole;   // uniform
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
            const uint32_t w = dg + i * BLOCK;
            if (w < (uint32_t)NW) {
                uint32_t o = 0;
                if (whole) {
                    if constexpr (DNA)
                        o = ((raw[i] >> 1) ^ (raw[i] >> 2)) & 0x03030303u;
                    else if constexpr (IDENT)
                        o = raw[i];
                    else
                        o = (uint32_t)s_map[raw[i] & 0xFFu] | ((uint32_t)s_map[(raw[i] >> 8) & 0xFFu] << 8) |
                            ((uint32_t)s_map[(raw[i] >> 16) & 0xFFu] << 16) | ((uint32_t)s_map[raw[i] >> 24] << 24);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint64_t pos = tb + 4ull * w + q;
                        o |= (pos < n ? (uint32_t)s_map[(raw[i] >> (8 * q)) & 0xFFu] : 0u) << (8 * q);
                    }
                }
                s_dcw[w] = o;
                if constexpr (DNA)
                    reinterpret_cast<uint8_t*>(s_pkw)[w] =
                        (uint8_t)(((o & 3u) << 6) | ((o >> 4) & 0x30u) | ((o >> 14) & 0xCu) | (o >> 24));
            }
        }
        // the next tile's ticket now: its round trip overlaps this tile's key
        // computation (no look-back depends on the ticket order); its text
        // loads wait until after the claims (loading right here was slower)
        if (dg == 0) s_tile[par ^ 1u] = atomicAdd(ticket, 1u);
        __syncthreads();
        TEXT_STAMP(0)
        // key1 of positions tb + ITEMS dg + j (D < 64 sigma 2^bb <= 2^32 rolls
        // in 32 bits; the remainder in 64)
        const bool full0 = SA_TEXT_FULL && valid == (uint32_t)TILE && blo == 0 && bspan == (1u << b.bb);
        uint64_t k[ITEMS];
        uint32_t dr[ITEMS];
        {
            const uint32_t l0 = ITEMS * dg;
            uint32_t D = 0;
            using RT = typename std::conditional<R32 && !POW2, uint32_t, uint64_t>::type;
            RT r = 0;
            // POW2: lg = log2 sigma; D < 2^(lg s) <= 2^32, r < 2^(lg R)
            const uint32_t lg = POW2 ? (uint32_t)__builtin_ctz(b.sigma) : 0u;
            const uint32_t dmask = POW2 ? (lg * b.s >= 32 ? ~0u : (1u << (lg * b.s)) - 1u) : 0u;
            const uint64_t rmask = POW2 ? ((1ull << (lg * b.R)) - 1ull) : 0ull;
            const uint32_t bksh = POW2 ? lg * b.s - b.bb : 0u;   // bucket = D >> (lg s - bb)
            // interior low = r mulR + addR (BucketSpec: compact or not)
            const uint64_t mulR = b.cmp == 2 ? 1u : b.cmp ? 2u : b.R + 1u, addR = b.cmp == 2 ? 0u : b.cmp ? 1u : b.s + b.R;
            uint64_t win = 0;   // DNA: symbols l0 .. l0 + 31, the first on top
            uint32_t wid[IDENT ? ITEMS / 4 + 2 : 1];   // IDENT: the lane's staged words from l0
            if constexpr (IDENT) {
#pragma unroll
                for (int q = 0; q < ITEMS / 4 + 2; ++q) wid[q] = s_dcw[l0 / 4 + q];
            } else if constexpr (DNA) {
                const uint32_t bo = l0 / 4, sh = bo & 3u;   // l0 % 4 == 0: one packed byte per 4 symbols
                const uint32_t w0 = s_pkw[bo >> 2], w1 = s_pkw[(bo >> 2) + 1], w2 = s_pkw[(bo >> 2) + 2];
                win = ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, sh)) << 32) |
                      __builtin_bswap32(__builtin_amdgcn_alignbyte(w2, w1, sh));
            } else if constexpr (POW2) {
                for (uint32_t q = 0; q < b.s; ++q) D = (D << lg) | s_dc[l0 + q];
                for (uint32_t q = 0; q < b.R; ++q) r = (r << lg) | s_dc[l0 + b.s + q];
            } else {
                for (uint32_t q = 0; q < b.s; ++q) D = D * b.sigma + s_dc[l0 + q];
                for (uint32_t q = 0; q < b.R; ++q) r = r * (RT)b.sigma + s_dc[l0 + b.s + q];
            }
            const bool interior = (uint32_t)t < t_int;   // every suffix of the tile has >= K symbols
            const bool full = full0 && interior;        // uniform
            // the digits leaving D (l0 ..), moving from the remainder into D
            // (l0 + s ..) and entering the remainder (l0 + K ..)
            uint32_t xo[ITEMS / 4], xm[ITEMS / 4], xn[ITEMS / 4];
            if constexpr (!DNA && !IDENT) {
                lds_bytes<ITEMS>(s_dcw, l0, xo);
                lds_bytes<ITEMS>(s_dcw, l0 + b.s, xm);
                lds_bytes<ITEMS>(s_dcw, l0 + K, xn);
            }
            const uint32_t dsh = 64u - 2u * b.s, rsh = 64u - 2u * K;
            // FULL: a whole tile of the whole bucket range, every position
            // kept (no per-item tests)
            auto keyloop = [&](auto fullc) {
            constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                if constexpr (DNA) {
                    const uint64_t x = win << (2 * j);
                    D = (uint32_t)(x >> dsh);
                    r = (x >> rsh) & rmask;
                } else if constexpr (IDENT) {
                    const uint64_t x =
                        ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(wid[j / 4 + 1], wid[j / 4], j % 4)) << 32) |
                        __builtin_bswap32(__builtin_amdgcn_alignbyte(wid[j / 4 + 2], wid[j / 4 + 1], j % 4));
                    D = (uint32_t)(x >> (64u - 8u * b.s));
                    r = (x >> (64u - 8u * K)) & rmask;
                } else if (j > 0) {
                    const uint32_t xi = byte_at<ITEMS>(xm, j - 1);
                    if constexpr (POW2) {
                        D = ((D << lg) | xi) & dmask;
                        r = ((r << lg) | byte_at<ITEMS>(xn, j - 1)) & rmask;
                    } else {
                        D = (D - byte_at<ITEMS>(xo, j - 1) * (uint32_t)b.pow_s1) * b.sigma + xi;
                        r = (r - (RT)xi * (RT)b.powR1) * (RT)b.sigma + byte_at<ITEMS>(xn, j - 1);
                    }
                }
                // (past the end L wraps: never ranked; FULL tiles are interior)
                const uint64_t low = (FULL || interior) ? (uint64_t)r * mulR + addR : bucket_low(b, r, n - (tb + l0 + j));
                k[j] = ((uint64_t)D << b.rb) | low;
                // (a non-power-of-two sigma has sigma^s > 2^16 = 2^bb at least,
                // so cmul = 2^48 / sigma^s < 2^32: one 32 x 32 multiply)
                const uint32_t bk = POW2 ? (D >> bksh) : (uint32_t)(((uint64_t)D * (uint32_t)b.cmul) >> b.bsh);
                const uint32_t lb = bk - blo;
                if constexpr (FULL) {
                    const uint32_t d = lb & (RADIX - 1);
                    dr[j] = (d << 16) | atomicAdd(&s_cnt[d], 1u);
                    atomicAdd(&s_hhi[lb >> kLoBits], 1u);
                } else {
                    const bool ok = l0 + j < valid && lb < bspan;
                    const uint32_t d = ok ? (lb & (RADIX - 1)) : (uint32_t)RADIX;
                    dr[j] = (d << 16) | (ok ? atomicAdd(&s_cnt[d], 1u) : 0u);
                    if (ok) atomicAdd(&s_hhi[lb >> kLoBits], 1u);
                }
            }
            };
            if (full) keyloop(std::true_type{});
            else keyloop(std::false_type{});
        }
        __syncthreads();
        TEXT_STAMP(1)
        uint32_t tile_cnt = 0;
        // the claim, waited for after the LDS staging (claims were 15 % of the
        // pass before; no zero initialisation: a register write there is a write-after-write on
        // the previous tile's pending claim, and the compiler drained every
        // memory operation for it)
        uint32_t clm, dbase;
        if (dg < (uint32_t)RADIX) {
            // (the lane's addresses rebuilt here from an opaque copy of dg: hoisted
            // out of the loop they spilled to scratch, and each reload waited
            // for every store of the previous tile)
            uint32_t dgo = dg;
            asm volatile("" : "+v"(dgo));
            tile_cnt = s_cnt[dgo];
            s_cnt[dgo] = 0;
            // the pass need not be stable, so a tile's place in each digit
            // is claimed from a cursor (one atomic round trip, whatever the
            // other tiles do) instead of a look-back
            dbase = seg_end ? sbase : digit_base[dgo];
            clm = tile_cnt ? atomicAdd(&cursor[dgo], tile_cnt) : 0u;
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
            if (dg == (uint32_t)RADIX - 1) s_kept = off + inc;   // pairs kept in this tile
        }
        // the next tile's text loads
        __syncthreads();
        TEXT_STAMP(2)
        const uint64_t tn = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[par ^ 1u]);
        load(tn < tiles ? tn : tiles - 1);
        // PK8: the item is built here, not in the key loop (its extra live
        // values there spilled 19 VGPRs): the second pass's digit (the
        // bucket's high bits; one GPU: local = global bucket), key1 below its
        // bucket, the position
        const uint32_t kbsh = b.rb + ((PK8 && POW2) ? (uint32_t)__builtin_ctz(b.sigma) * b.s - b.bb : 0u);
        const uint64_t remmask = (PK8 && POW2) ? (1ull << kbsh) - 1ull : 0ull;
        // NP2: D - Dmin(bucket) = the values of D below D in its bucket =
        // floor(f / cmul), f = D cmul mod 2^bsh (the bucket's fraction; f <
        // 2^31): by a double reciprocal, corrected by one integer step
        const double icm = NP2 ? 1.0 / (double)b.cmul : 0.0;
        const uint64_t fmask = (1ull << b.bsh) - 1ull;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t d = dr[j] >> 16;
            if (d < (uint32_t)RADIX) {
                const uint32_t pos = s_start[d] + (dr[j] & 0xFFFFu);
                if constexpr (NP2) {   // (D < 2^32, cmul < 2^32: 32 x 32 multiplies)
                    const uint32_t cm32 = (uint32_t)b.cmul;
                    const uint64_t prod = (uint64_t)(uint32_t)(k[j] >> b.rb) * cm32;
                    const uint32_t bk = (uint32_t)(prod >> b.bsh);
                    const uint32_t f = (uint32_t)(prod & fmask);
                    uint32_t rd = (uint32_t)((double)f * icm);
                    rd = ((uint64_t)rd * cm32 > f) ? rd - 1u : rd;
                    rd = ((uint64_t)(rd + 1u) * cm32 <= f) ? rd + 1u : rd;
                    const uint32_t hi = (bk - blo) >> kLoBits;   // local bucket
                    const uint64_t rel = ((uint64_t)rd << b.rb) | (k[j] & ((1ull << b.rb) - 1ull));
                    s_keys[pos] = ((uint64_t)hi << (64u - pk_hb)) | (rel << pk_ib) | (tb + ITEMS * dg + j);
                    s_idx[pos] = (uint16_t)d;
                } else if constexpr (PK8) {
                    const uint32_t hi = ((uint32_t)(k[j] >> kbsh) - blo) >> kLoBits;   // local bucket
                    s_keys[pos] = ((uint64_t)hi << (64u - pk_hb)) | ((k[j] & remmask) << pk_ib) |
                                  (tb + ITEMS * dg + j);
                    s_idx[pos] = (uint16_t)d;
                } else {
                    s_keys[pos] = k[j];
                    s_idx[pos] = (uint16_t)(ITEMS * dg + j);
                }
            }
        }
        // the claims' round trips overlapped the staging (only the writes
        // need the tile's places)
        if (dg < (uint32_t)RADIX) s_gofs[dg] = dbase + clm;
        __syncthreads();
        TEXT_STAMP(3)
        const uint32_t kept = s_kept;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t q = j * BLOCK + dg;
            if (q < kept) {
                const uint64_t key = s_keys[q];
                uint32_t dd;
                if constexpr (PK8) {
                    dd = s_idx[q];
                } else {
                    // POW2: the bucket is a bit field of key1 (no 64-bit multiply)
                    const uint32_t bq = POW2 ? (uint32_t)(key >> (b.rb + (uint32_t)__builtin_ctz(b.sigma) * b.s - b.bb))
                                             : (uint32_t)(((key >> b.rb) * b.cmul) >> b.bsh);
                    dd = (bq - blo) & (RADIX - 1);
                }
                const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
                if (seg_end ? g < s_gend[dd] : g < m) {
                    out_keys[g] = key;
                    if constexpr (!PK8) out_vals[g] = (uint32_t)(tb + s_idx[q]);
                } else {
                    over = true;
                }
            }
        }
        __syncthreads();
        TEXT_STAMP(4)
        t = tn;
        par ^= 1u;
    }
    for (uint32_t i = dg; i < 1024u; i += BLOCK)
        if (s_hhi[i]) atomicAdd(&ghist_hi[i], s_hhi[i]);
    if (over && ovf) atomicOr(ovf, 1u);
#if SA_TEXT_PROF
    if (dg == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
        printf("k_split_text wg %u clk: stage %llu keys %llu claims %llu scatter %llu write %llu\n", blockIdx.x,
               (unsigned long long)pacc[0], (unsigned long long)pacc[1], (unsigned long long)pacc[2],
               (unsigned long long)pacc[3], (unsigned long long)pacc[4]);
#endif
#undef TEXT_STAMP
}

// ---------------------------------------------------------------------------
// The first bucket pass of one rank's bucket range in the range-partitioned
// build (sa_dist.h) from the range's records (key1, position) that
// k_bucket_hist<LIST> compacted: a rank of G keeps ~n/G of the text's
// suffixes, and rolling key1 over every position of the text inside this
// pass cost k_split_text 2.9 of a 5.0 ms first round at G = 8.  Ranking,
// claims and the scatter by the low kLoBits of the local bucket are those of
// k_split_text.
// ---------------------------------------------------------------------------
// PK8: packed 8-byte items as k_split_text<.., PK8> writes them
template <int ITEMS, int BLOCK = kSpBlock, bool PK8 = false>
__global__ __launch_bounds__(BLOCK, 2048 / BLOCK) void k_split_list(BucketSpec b, const uint64_t* __restrict__ lkeys,
                                                         const uint32_t* __restrict__ lpos, uint64_t m, uint32_t blo,
                                                         const uint32_t* __restrict__ digit_base,
                                                         uint32_t* __restrict__ ticket, uint64_t* __restrict__ out_keys,
                                                         uint32_t* __restrict__ out_vals,
                                                         uint32_t* __restrict__ ghist_hi, uint32_t* __restrict__ cursor,
                                                         uint32_t pk_hb = 0, uint32_t pk_ib = 0,
                                                         const uint32_t* __restrict__ reg_cnt = nullptr,
                                                         uint32_t reg_cap = 0) {
    // reg_cnt (k_bucket_hist<.., LM = 3>'s records): kRecStripes regions of
    // reg_cap records, region r holding reg_cnt[r kRecCurStride] from r reg_cap; the
    // units are cut per region.  Else m records from 0.
    constexpr int RADIX = kLoRadix;
    constexpr int RWAVES = RADIX / kWave;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE <= 65535, "16-bit tile offsets");
    __shared__ uint64_t s_keys[TILE];
    __shared__ uint32_t s_pos[TILE];   // PK8: the pair's digit
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[RWAVES];
    __shared__ uint32_t s_tile[2];
    __shared__ uint32_t s_hhi[1024];   // the second pass's digit totals (local bucket >> kLoBits)
    __shared__ uint32_t s_ubase[kRecStripes + 1];   // regions: units before region r
    static_assert(BLOCK >= (int)kRecStripes && kRecStripes == kWave, "one wave numbers the regions");

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    for (uint32_t i = dg; i < 1024u; i += BLOCK) s_hhi[i] = 0;
    if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;
    if (dg == 0) s_tile[0] = atomicAdd(ticket, 1u);
    if (reg_cnt && wave == 0) {
        const uint32_t c = min(reg_cnt[lane * kRecCurStride], reg_cap);
        const uint32_t x = (c + TILE - 1) / TILE;
        const uint32_t inc = wave_inclusive_sum(x);
        s_ubase[lane] = inc - x;
        if (lane == kWave - 1) s_ubase[kRecStripes] = inc;
    }
    __syncthreads();
    const uint64_t tiles = reg_cnt ? (uint64_t)s_ubase[kRecStripes] : (m + TILE - 1) / TILE;
    // unit -> its first record and size
    auto locate = [&](uint64_t u, uint64_t& tb, uint32_t& valid) {
        if (!reg_cnt) {
            tb = u * TILE;
            valid = (uint32_t)((m - tb) < (uint64_t)TILE ? (m - tb) : (uint64_t)TILE);
            return;
        }
        uint32_t a = 0, z = kRecStripes;   // last region r with s_ubase[r] <= u
        while (z - a > 1) {
            const uint32_t mid = (a + z) / 2;
            if (s_ubase[mid] <= (uint32_t)u) a = mid;
            else z = mid;
        }
        const uint32_t i0 = ((uint32_t)u - s_ubase[a]) * TILE;
        tb = (uint64_t)a * reg_cap + i0;
        const uint32_t c = min(reg_cnt[a * kRecCurStride], reg_cap) - i0;
        valid = c < (uint32_t)TILE ? c : (uint32_t)TILE;
    };
    uint64_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[0]);
    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    auto load = [&](uint64_t tb, uint32_t valid, uint64_t* kk, uint32_t* vv) {   // clamped, unpredicated (see k_split)
        const uint32_t last = valid - 1;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const uint64_t e = tb + (le < last ? le : last);
            kk[j] = lkeys[e];
            vv[j] = lpos[e];
        }
    };
    uint64_t tb = 0;
    uint32_t valid = 1;
    if (t < tiles) {
        locate(t, tb, valid);
        load(tb, valid, k, v);
    }
    uint32_t par = 0;
    while (t < tiles) {
        uint32_t dr[ITEMS];
        // whole tiles take the ranking without per-item tests
        auto rank = [&](auto wholec) {
            constexpr bool WHOLE = decltype(wholec)::value;
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                const uint32_t le = wave * WTILE + j * kWave + lane;
                const bool ok = WHOLE || le < valid;
                const uint32_t lb = bucket_of(k[j], b.rb, b.cmul, b.bsh) - blo;
                const uint32_t d = ok ? (lb & (RADIX - 1)) : (uint32_t)RADIX;
                dr[j] = (d << 16) | (ok ? atomicAdd(&s_cnt[d], 1u) : 0u);
                if (ok) atomicAdd(&s_hhi[lb >> kLoBits], 1u);
            }
        };
        if (valid == (uint32_t)TILE) rank(std::true_type{});   // uniform
        else rank(std::false_type{});
        __syncthreads();
        uint32_t tile_cnt = 0;
        if (dg < (uint32_t)RADIX) {
            tile_cnt = s_cnt[dg];
            s_cnt[dg] = 0;
            s_gofs[dg] = digit_base[dg] + (tile_cnt ? atomicAdd(&cursor[dg], tile_cnt) : 0u);
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
        if (dg == 0) s_tile[par ^ 1u] = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint64_t tn = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[par ^ 1u]);
        uint64_t kn[ITEMS];
        uint32_t vn[ITEMS];
        uint64_t tbn;
        uint32_t validn;
        locate(tn < tiles ? tn : tiles - 1, tbn, validn);
        load(tbn, validn, kn, vn);
        const uint32_t kbsh = b.rb + (PK8 ? (uint32_t)__builtin_ctz(b.sigma) * b.s - b.bb : 0u);
        const uint64_t remmask = PK8 ? (1ull << kbsh) - 1ull : 0ull;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t d = dr[j] >> 16;
            if (d < (uint32_t)RADIX) {
                const uint32_t q = s_start[d] + (dr[j] & 0xFFFFu);
                if constexpr (PK8) {
                    const uint32_t hi = ((uint32_t)(k[j] >> kbsh) - blo) >> kLoBits;
                    s_keys[q] = ((uint64_t)hi << (64u - pk_hb)) | ((k[j] & remmask) << pk_ib) | v[j];
                    s_pos[q] = d;
                } else {
                    s_keys[q] = k[j];
                    s_pos[q] = v[j];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t q = j * BLOCK + dg;
            if (q < valid) {
                const uint64_t key = s_keys[q];
                const uint32_t dd =
                    PK8 ? s_pos[q] : (bucket_of(key, b.rb, b.cmul, b.bsh) - blo) & (RADIX - 1);
                const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
                if (g < m) {
                    out_keys[g] = key;
                    if constexpr (!PK8) out_vals[g] = s_pos[q];
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
        tb = tbn;
        valid = validn;
        par ^= 1u;
    }
    for (uint32_t i = dg; i < 1024u; i += BLOCK)
        if (s_hhi[i]) atomicAdd(&ghist_hi[i], s_hhi[i]);
}

// ---------------------------------------------------------------------------
// The second bucket pass without a look-back.  Its input is ordered by the
// first pass's digit l (the bucket's low kLoBits): segment l of the input is
// [lo_base[l], lo_base[l + 1]).  The pass must keep l's order only, and
// within a segment all pairs share l, so work units never straddle segments
// (the tile grid is cut at segment boundaries) and a unit of segment l
// claims its place per high digit h from a per-(l, h) atomic cursor.  Where
// segment l starts inside digit h -- base(h, l) = base(h) + the count of h
// in segments < l -- is published by the last unit of segment l - 1 to
// claim (done[l - 1] counts claims) once base(h, l - 1) is known: a chain of
// one hop per segment (256 per pass) instead of a look-back per tile.  A
// unit waits only for base(., l); claims never wait, so the chain always
// advances.  No fences (a device-scope release writes back the L2: 10x
// slower): a claim's atomic has returned before its unit counts itself
// done, and base words carry their own ready bit (bit 32).
// segw (zeroed before the pass): cur u32[256][RADIX] | base u64[256][RADIX]
// | done u32[256].  Output: one 64-bit word per pair, bucket-relative
// (bucket_dmin, sa_bucket.h): w = (key1 - (Dmin(b) << rb)) << ib | idx --
// 8 B written (and read by the local sort) instead of 12.
// ---------------------------------------------------------------------------
constexpr uint32_t kSegs = kLoRadix;
constexpr uint32_t kMaxStripes = 8;   // first-pass cursor stripes (k_split_text)
constexpr uint64_t segw_words(int radix) { return 3ull * kSegs * radix + kSegs; }
// the bucket starts live after the widest pass's segment words
constexpr uint64_t kBstartOff = segw_words(1024);
constexpr uint64_t kBstartWords = (1ull << 18) + 1;

// (BLOCK 512 x 10 items, two workgroups per CU, measured slower: 7.2 -> 9.1 ms;
// again with PK8 items, 512 x 12 (SA_SEG_BLOCK=512): 4.64 -> 6.27 ms.
// Whole packed items staged (digit from their top bits, no s_dig) with the
// next unit's loads issued after the staging into the same registers, so
// that 14 or 16 items per lane fit: 12 / 14 / 16 items 5.07 / 5.20 / 6.4 ms
// against 4.68 for this kernel, profiles/r04_b_ab_seg_late.txt -- the loads
// must be in flight through the base wait and the staging, and larger units
// do not make the 512-way writes faster.)
// Also measured slower (profiles/r04_i_ab_seg_whole.txt): whole packed items
// staged (digit from the top bits, no s_dig) with 16 / 14 / 12 items per lane
// and the next unit's loads split around the staging: 5.72 / 4.94 / 4.89 ms
// against 4.68-4.95 -- although 32-item runs write faster than 24-item ones
// in isolation (microbench_runs.hip, profiles/r04_e_microbench_runs.txt).
// ---------------------------------------------------------------------------
// XQ: per-XCD queues and output regions (round 5).  Workgroup w runs on XCD
// w mod 8 (workgroups are dealt to the 8 XCDs round robin), so queue q =
// w mod 8 takes the units u = 8 t + q from its own ticket, and its units'
// items go to region q of the output: region q is in bucket order (h, l)
// over queue q's items only, each digit h in a sub-region of capacity
// cap(h) = tot(h) / 8 + tot(h) / 128 + kXqSlack (a queue holds every 8th
// unit of every segment, so its share of a digit is tot(h) / 8 within a few
// hundred items on any text whose digit-h items spread over the units).
// Every queue keeps its own cursors, bases and segment chain: a unit waits
// only for units of its own queue, and the runs that end next to one
// another in a sub-region were written by the same XCD, whose L2 merges the
// partial lines at their ends -- the write pattern that held the pass at
// 0.46 of the HBM peak (microbench_seg.hip: one region 4.97 ms, per-XCD
// regions 3.61 ms at 2^30 items, profiles/r05_b_microbench_seg.txt).  A
// queue whose digit outgrows its sub-region sets words[9] (err2); the round
// then runs the pass again without XQ.  k_bucket_starts_xq derives the
// exact bucket starts and each bucket's chunk per region; the local sort
// loads a one-bucket window from its 8 chunks.
// ---------------------------------------------------------------------------
constexpr uint32_t kXqSlack = 2048;     // per (queue, digit) sub-region slack
constexpr uint32_t kXqTicketStride = 32;   // one 128-byte line per queue ticket
struct SegXq {
    uint32_t* cur = nullptr;           // [kXq][kSegs][RADIX] claim cursors
    uint64_t* sbase = nullptr;         // [kXq][kSegs][RADIX] published bases (bit 32: ready)
    uint32_t* done = nullptr;          // [kXq][kSegs] claims per segment
    uint32_t* tickets = nullptr;       // [kXq] at kXqTicketStride
    const uint32_t* dh = nullptr;      // [RADIX + 1] digit sub-region starts inside a region (dh[RADIX]: its size)
    uint32_t cap = 0;                  // output capacity (items)
    uint32_t* err2 = nullptr;          // a sub-region overflowed
};
// words of the XQ workspace for a radix (cursors, bases, done, tickets)
constexpr uint64_t xq_words(int radix) { return 3ull * kXq * kSegs * radix + kXq * kSegs + kXq * kXqTicketStride; }

template <class Src, int RBITS, int ITEMS, int BLOCK = kSpBlock, bool XQ = false>
__global__ __launch_bounds__(BLOCK, 2048 / BLOCK) void k_split_seg(Src src, uint64_t n, uint32_t shift,
                                                        const uint32_t* __restrict__ lo_base,
                                                        const uint32_t* __restrict__ digit_base,
                                                        uint32_t* __restrict__ segw, uint32_t* __restrict__ ticket,
                                                        uint32_t ib, uint64_t* __restrict__ out_w,
                                                        uint32_t* __restrict__ err,
                                                        const uint32_t* __restrict__ seg_cnt = nullptr,
                                                        const uint32_t* __restrict__ dense_lo = nullptr,
                                                        uint32_t stripes = 1, SegXq xq = SegXq{}) {
    constexpr int RADIX = 1 << RBITS;
    constexpr int RWAVES = RADIX / kWave;
    constexpr int WTILE = kWave * ITEMS;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(BLOCK >= RADIX && (int)kSegs <= BLOCK, "one thread per digit / segment");
    static_assert((int)(kSegs * kMaxStripes) <= 2 * BLOCK, "two sub-segments per thread in the unit numbering");
    static_assert(TILE <= 65535, "16-bit tile offsets");
    __shared__ uint64_t s_keys[TILE];   // bucket-relative items, digit-sorted
    __shared__ uint16_t s_dig[TILE];
    __shared__ uint32_t s_dmin[RADIX];  // Dmin of bucket (h, l)
    __shared__ uint32_t s_cnt[RADIX];
    __shared__ uint16_t s_start[RADIX];
    __shared__ uint32_t s_gofs[RADIX];
    __shared__ uint32_t s_tmp[(BLOCK / kWave)];
    __shared__ uint32_t s_ubase[kSegs * kMaxStripes + 1];   // units before sub-segment q (exclusive scan)
    __shared__ uint32_t s_tile[2];
    __shared__ uint32_t s_last;
    __shared__ uint32_t s_claim[RADIX];
    // XQ: this workgroup's queue (= its XCD) and the queue's own cursors,
    // bases, claim counts and ticket
    const uint32_t xqq = XQ ? (blockIdx.x & (kXq - 1)) : 0u;
    uint32_t* const cur = XQ ? xq.cur + (uint64_t)xqq * kSegs * RADIX : segw;
    uint64_t* const sbase = XQ ? xq.sbase + (uint64_t)xqq * kSegs * RADIX
                               : reinterpret_cast<uint64_t*>(segw + (uint64_t)kSegs * RADIX);
    uint32_t* const done = XQ ? xq.done + xqq * kSegs : segw + 3ull * kSegs * RADIX;
    if constexpr (XQ) ticket = xq.tickets + xqq * kXqTicketStride;
    const uint64_t gcap = XQ ? (uint64_t)xq.cap : n;
    const uint32_t xrs = XQ ? xq.dh[RADIX] : 0u;   // region size
    constexpr uint64_t kReady = 1ull << 32;

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    const uint32_t mask = RADIX - 1;
    // sub-segment q = l * stripes + s of the input (s < stripes; one per
    // segment unless the first pass striped its cursors): [lo, hi) with
    // lo = lo_base[l] + s * ((lo_base[l + 1] - lo_base[l]) / stripes) and,
    // padded (seg_cnt), hi = lo + seg_cnt[s * kSegs + l]; unpadded, segment l
    // is [lo_base[l], the next segment's start).  dense_lo: the pairs before
    // segment l (0: every earlier segment is empty)
    const uint32_t nsub = kSegs * stripes;
    auto sub_lo = [&](uint32_t q) -> uint64_t {
        const uint32_t l = q / stripes, sidx = q % stripes;
        if (stripes == 1) return lo_base[l];
        return (uint64_t)lo_base[l] + sidx * ((lo_base[l + 1] - lo_base[l]) / stripes);
    };
    auto sub_hi = [&](uint32_t q) -> uint64_t {
        const uint32_t l = q / stripes, sidx = q % stripes;
        if (seg_cnt) return sub_lo(q) + seg_cnt[sidx * kSegs + l];
        return l + 1 < kSegs ? (uint64_t)lo_base[l + 1] : n;
    };
    const uint32_t* const dlo = dense_lo ? dense_lo : lo_base;
    // unit numbering: sub-segment by sub-segment (nsub <= BLOCK * 2)
    {
        uint32_t x0 = 0, x1 = 0;
        const uint32_t q0 = 2 * dg, q1 = 2 * dg + 1;
        if (q0 < nsub) x0 = (uint32_t)((sub_hi(q0) - sub_lo(q0) + TILE - 1) / TILE);
        if (q1 < nsub) x1 = (uint32_t)((sub_hi(q1) - sub_lo(q1) + TILE - 1) / TILE);
        const uint32_t x = x0 + x1;
        const uint32_t inc = wave_inclusive_sum(x);
        if (lane == kWave - 1) s_tmp[wave] = inc;
        __syncthreads();
        uint32_t off = 0;
        for (uint32_t w = 0; w < wave; ++w) off += s_tmp[w];
        if (q0 < nsub) s_ubase[q0] = off + inc - x;
        if (q1 < nsub) s_ubase[q1] = off + inc - x1;
        if (q1 + 1 >= nsub && q0 < nsub) s_ubase[nsub] = off + inc;
    }
    if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;
    if (dg == 0) s_tile[0] = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t units = s_ubase[nsub];
    // XQ: units u < U of this queue (u mod 8 = xqq); a ticket t is unit 8 t + xqq
    auto qcount = [&](uint32_t U) -> uint32_t { return XQ ? (U + (kXq - 1) - xqq) / kXq : U; };
    auto unit_of = [&](uint32_t t) -> uint32_t { return XQ ? t * kXq + xqq : t; };
    // units of segment l (all its sub-segments; XQ: of this queue)
    auto units_of = [&](uint32_t l) -> uint32_t {
        return qcount(s_ubase[(l + 1) * stripes]) - qcount(s_ubase[l * stripes]);
    };
    // unit -> (segment, first position, size)
    auto locate = [&](uint32_t u, uint32_t& l, uint64_t& tb, uint32_t& valid) {
        uint32_t a = 0, b = nsub;   // last q with s_ubase[q] <= u (units of empty sub-segments are skipped)
        while (b - a > 1) {
            const uint32_t mid = (a + b) / 2;
            if (s_ubase[mid] <= u) a = mid;
            else b = mid;
        }
        l = a / stripes;
        tb = sub_lo(a) + (uint64_t)(u - s_ubase[a]) * TILE;
        const uint64_t e = sub_hi(a);
        valid = (uint32_t)(e - tb < (uint64_t)TILE ? e - tb : (uint64_t)TILE);
    };
    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    auto load = [&](uint64_t tb, uint32_t valid, uint64_t* kk, uint32_t* vv) {
        const uint32_t last = valid - 1;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const uint64_t e = tb + (le < last ? le : last);
            kk[j] = src.key(e);
            vv[j] = Src::kPk8 ? 0u : src.val(e);
        }
    };
    uint32_t u = unit_of((uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[0]));
    uint32_t l = 0, valid = 0;
    uint64_t tb = 0;
    if (u < units) {
        locate(u, l, tb, valid);
        load(tb, valid, k, v);
    }
    uint32_t par = 0;
#if SA_SEG_PROF
    // diagnostic build (-DSA_SEG_PROF=1): clock64 spans of thread 0 per phase
    uint64_t pacc[7] = {0, 0, 0, 0, 0, 0, 0}, plast = clock64();
#define SEG_STAMP(k)                                \
    if (dg == 0) {                                  \
        const uint64_t now_ = clock64();            \
        pacc[k] += now_ - plast;                    \
        plast = now_;                               \
    }
#else
#define SEG_STAMP(k)
#endif
    while (u < units) {
        // the next unit's ticket: its round trip overlaps the ranking and
        // claims (read after the claims' barrier)
        if (dg == 0) s_tile[par ^ 1u] = atomicAdd(ticket, 1u);
        // ranks within the unit (any order: one segment, one value of l)
        // (full units without per-item bounds tests: no faster,
        // profiles/r04_n_ab_full_tiles.txt)
        uint32_t dr[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t le = wave * WTILE + j * kWave + lane;
            const uint32_t d = le < valid ? src_digit(src, k[j], shift, mask, 0) : (uint32_t)RADIX;
            dr[j] = (d << 16) | (d < (uint32_t)RADIX ? atomicAdd(&s_cnt[d], 1u) : 0u);
        }
        __syncthreads();
        SEG_STAMP(0)
        // claim this unit's place in (l, h); count the claim for segment l
        // (the claim's return value is stored first: it has been performed)
        uint32_t tile_cnt = 0;
        if (dg < (uint32_t)RADIX) {
            tile_cnt = s_cnt[dg];
            s_claim[dg] = tile_cnt ? atomicAdd(&cur[(uint64_t)l * RADIX + dg], tile_cnt) : 0u;
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
        SEG_STAMP(1)
        if (dg == 0) s_last = atomicAdd(&done[l], 1u) == units_of(l) - 1 ? 1u : 0u;
        // base(h, l): digit_base when every earlier segment is empty, else
        // published (with its ready bit) by segment l - 1's last claimer
        if (dg < (uint32_t)RADIX) {
            uint32_t bh;
            if (XQ ? qcount(s_ubase[l * stripes]) == 0 : dlo[l] == 0) {
                // the first segment of the (queue's) items: the digit's start
                // (XQ: its sub-region in the queue's region)
                bh = XQ ? xqq * xrs + xq.dh[dg] : digit_base[dg];
            } else {
                uint64_t w;
                uint32_t spins = 0;
                while (((w = __hip_atomic_load(&sbase[(uint64_t)l * RADIX + dg], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) & kReady) == 0) {
                    if (++spins > kSpinLimit) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                bh = (uint32_t)w;
            }
            s_gofs[dg] = bh + s_claim[dg];
            if constexpr (XQ) {   // the run must end inside the digit's sub-region
                if (tile_cnt && (uint64_t)bh + s_claim[dg] + tile_cnt > (uint64_t)xqq * xrs + xq.dh[dg + 1])
                    atomicOr(xq.err2, 1u);
            }
            s_claim[dg] = bh;
            if constexpr (!Src::kPk8) s_dmin[dg] = bucket_dmin(((dg << kLoBits) | l) + src.bofs, src.cmul, src.bsh);
        }
        __syncthreads();
        SEG_STAMP(2)
        if (s_last) {
            // every claim of segment l has been performed: publish base(., l')
            // for the next segment and the empty ones after it
            if (dg < (uint32_t)RADIX) {
                const uint32_t tot = __hip_atomic_load(&cur[(uint64_t)l * RADIX + dg], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                for (uint32_t l2 = l + 1; l2 < kSegs; ++l2) {
                    __hip_atomic_store(&sbase[(uint64_t)l2 * RADIX + dg], kReady | (uint64_t)(s_claim[dg] + tot),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (units_of(l2) > 0) break;
                }
            }
        }
        // the next unit's loads (see k_split)
        __syncthreads();
        const uint32_t un = unit_of((uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile[par ^ 1u]));
        SEG_STAMP(3)
        uint32_t ln = l, validn = valid;
        uint64_t tbn = tb;
        if (un < units) locate(un, ln, tbn, validn);
        uint64_t kn[ITEMS];
        uint32_t vn[ITEMS];
        load(tbn, validn, kn, vn);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t d = dr[j] >> 16;
            if (d < (uint32_t)RADIX) {
                const uint32_t pos = s_start[d] + (dr[j] & 0xFFFFu);
                if constexpr (Src::kPk8)   // the item below its digit (shift = 64 - hb)
                    s_keys[pos] = k[j] & ((1ull << shift) - 1ull);
                else
                    s_keys[pos] = ((k[j] - ((uint64_t)s_dmin[d] << src.rb)) << ib) | v[j];
                s_dig[pos] = (uint16_t)d;
            }
        }
        __syncthreads();
        SEG_STAMP(4)
        if (dg < (uint32_t)RADIX) s_cnt[dg] = 0;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint32_t q = j * BLOCK + dg;
            if (q < valid) {
                const uint32_t dd = s_dig[q];
                const uint64_t g = (uint64_t)s_gofs[dd] + (q - s_start[dd]);
                if (g < gcap) out_w[g] = s_keys[q];
            }
        }
        __syncthreads();
        SEG_STAMP(5)
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            k[j] = kn[j];
            v[j] = vn[j];
        }
        u = un;
        l = ln;
        tb = tbn;
        valid = validn;
        par ^= 1u;
    }
#if SA_SEG_PROF
    if (dg == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
        printf("k_split_seg wg %u clk: rank %llu claim %llu base %llu ticket+load %llu scatter %llu write %llu\n",
               blockIdx.x, (unsigned long long)pacc[0], (unsigned long long)pacc[1], (unsigned long long)pacc[2],
               (unsigned long long)pacc[3], (unsigned long long)pacc[4], (unsigned long long)pacc[5]);
#endif
#undef SEG_STAMP
}

// bucket b = (h << kLoBits) | l starts at base(h, l) in the second pass's
// output (= SA order of round 1): digit_base[h] while every segment before
// l is empty, else the value k_split_seg published.  bstart[2^bb] = n; the
// bucket's smallest D is bdmin[b].  The local sort rebuilds key1 from the
// bucket-relative items with them; the sparse rank look-ups of later rounds
// search key1 only inside the bucket.
// (local buckets b of a range starting at global bucket bofs: Dmin of b + bofs)
template <int RADIX>
__global__ __launch_bounds__(kBlock) void k_bucket_starts(const uint32_t* __restrict__ lo_base,
                                                          const uint32_t* __restrict__ digit_base,
                                                          const uint32_t* __restrict__ segw, uint64_t n,
                                                          uint64_t cmul, uint32_t bsh, uint32_t* __restrict__ bstart,
                                                          uint32_t* __restrict__ bdmin, uint32_t bofs) {
    const uint64_t* sbase = reinterpret_cast<const uint64_t*>(segw + (uint64_t)kSegs * RADIX);
    const uint32_t nb = (uint32_t)RADIX << kLoBits;
    for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b <= nb; b += gridDim.x * kBlock) {
        if (b == nb) {
            bstart[b] = (uint32_t)n;
            continue;
        }
        const uint32_t h = b >> kLoBits, l = b & (kSegs - 1);
        bstart[b] = lo_base[l] == 0 ? digit_base[h] : (uint32_t)sbase[(uint64_t)l * RADIX + h];
        bdmin[b] = bucket_dmin(b + bofs, cmul, bsh);
    }
}

// XQ digit sub-regions: dh[h] = sum of cap(h') for h' < h, dh[RADIX] = the
// region size, from the digit totals tot (one workgroup of 1024 threads;
// RADIX <= 1024).  exact_caps (tests): cap = tot / 8, no slack, so that a
// queue overflows and the round takes the exact pass.
__global__ __launch_bounds__(1024) void k_xq_dh(const uint32_t* __restrict__ tot, uint32_t radix, uint32_t exact_caps,
                                                uint32_t* __restrict__ dh) {
    __shared__ uint32_t s_tmp[1024 / kWave];
    const uint32_t t = threadIdx.x;
    uint32_t cap = 0;
    if (t < radix) {
        const uint32_t x = tot[t];
        cap = exact_caps ? x / kXq : x / kXq + x / 128u + kXqSlack;
    }
    const uint32_t inc = wave_inclusive_sum(cap);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t w = 0; w < wave_id(); ++w) off += s_tmp[w];
    if (t < radix) dh[t] = off + inc - cap;
    if (t == radix - 1) dh[radix] = off + inc;
}

// XQ bucket tables: one workgroup per high digit h, one thread per segment
// l (bucket b = h << kLoBits | l).  Queue q's count of bucket b is its final
// cursor cur[q][l][h]; its chunk starts at q rs + dh[h] + the queue's counts
// of (l' < l, h), and the bucket starts (exact, SA order) at digit_base[h] +
// the counts of (l' < l, h) of all queues.  pc / pn: [kXq][nb] chunk starts
// and counts; bstart[nb] = n.
template <int RADIX>
__global__ __launch_bounds__(kLoRadix) void k_bucket_starts_xq(const uint32_t* __restrict__ digit_base,
                                                               const uint32_t* __restrict__ cur,
                                                               const uint32_t* __restrict__ dh,
                                                               uint64_t n, uint64_t cmul, uint32_t bsh,
                                                               uint32_t* __restrict__ bstart,
                                                               uint32_t* __restrict__ bdmin, uint32_t* __restrict__ pc,
                                                               uint32_t* __restrict__ pn, uint32_t bofs) {
    static_assert(kSegs == kLoRadix && kLoRadix % kWave == 0, "one thread per segment");
    __shared__ uint32_t s_tmp[kLoRadix / kWave];
    const uint32_t nb = (uint32_t)RADIX << kLoBits;
    const uint32_t h = blockIdx.x, l = threadIdx.x;
    const uint32_t b = (h << kLoBits) | l;
    auto excl = [&](uint32_t x) {   // exclusive scan over the workgroup's segments
        const uint32_t inc = wave_inclusive_sum(x);
        __syncthreads();
        if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
        __syncthreads();
        uint32_t off = 0;
        for (uint32_t w = 0; w < wave_id(); ++w) off += s_tmp[w];
        return off + inc - x;
    };
    const uint32_t rs = dh[RADIX];
    uint32_t tot = 0;
#pragma unroll 1
    for (uint32_t q = 0; q < kXq; ++q) {
        const uint32_t c = cur[((uint64_t)q * kSegs + l) * RADIX + h];
        tot += c;
        pn[(uint64_t)q * nb + b] = c;
        pc[(uint64_t)q * nb + b] = q * rs + dh[h] + excl(c);
    }
    bstart[b] = digit_base[h] + excl(tot);
    bdmin[b] = bucket_dmin(b + bofs, cmul, bsh);
    if (b == 0) bstart[nb] = (uint32_t)n;
}

}  // namespace sa
