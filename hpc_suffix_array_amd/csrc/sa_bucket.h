// sa_bucket.h -- bucketed first round of the packed schedule: two global
// radix passes over a 16-bit bucket of each suffix's prefix, then one
// workgroup sorts each bucket window in LDS.
//
// The first round sorts every suffix by its first K symbols (it replaces
// rounds h = 1 .. K/2 of manber_myers.c:97-125).  A full LSD sort of a
// 47-bit key is six 24-byte-per-suffix passes over HBM; here the key is
// laid out so that its order is (bucket, rest):
//
//   D(i)   = sum_{t<s} dc(i+t) sigma^(s-1-t)     dense s-symbol prefix,
//            dc = code - 1 (codes 1..sigma), 0 past the end
//   low(i) = L - 1                        if L = n - i < s  (shorter than s)
//            s + E(i) (R+1) + min(R, L-s)  otherwise, E(i) = the next R symbols
//            as dense digits dc (0 past the end) and min(R, L-s) how many of
//            them precede the end
//   key1(i) = D(i) << rb | low(i)
//
// key1 orders suffixes exactly as their first K = s + R symbols (end
// smallest) and two suffixes get equal key1 iff those K symbols are equal.
// The end digit is clamped onto the smallest symbol's digit, so a suffix
// that ends inside a window shares its dense value with the suffixes that
// continue it with the smallest symbol; the count of symbols before the end
// (for L < s: L - 1 < s, below every longer suffix) puts it, and shorter
// ones first, ahead of them.  Both fields are dense, so for random text the
// 16-bit bucket = (D * cmul) >> 32 (sigma^s >= 2^16) and the top bits of
// low are near-uniform.
//
//   k_bucket_hist     text -> the first pass's digit totals (low kLoBits)
//   k_split_text      first pass (sa_split.h): key1 computed per tile from
//                     the text, scattered by the low kLoBits of the bucket
//                     (unstable, atomic cursors; also counts the high bits)
//   k_split           second pass: stable by the high bb - kLoBits bits
//                     (SrcBucketKeys; look-back)
//   k_window_starts   window j starts at the first bucket boundary >= j*W
//   k_window_list     the non-empty windows and the largest (the host
//                     checks it against the LDS capacity; oversize windows
//                     fall back to the full LSD sort)
//   k_bucket_sort     one workgroup per window: counting scatter into
//                     sub-buckets + register sorting networks over
//                     key1 - min(window) (idx packed below) -> sorted key1 +
//                     SA written coalesced, and the round-1 groups
//   k_bucket_sort_lsd windows with clustered keys: LSD passes in LDS
//   k_wscan_* + k_u_gather  the unsorted set in SA order
#pragma once
#include "sa_kernels.h"

namespace sa {

// local sort workgroup: 8 waves x 18 suffixes per lane; 72 KiB of LDS and
// <= 128 VGPRs, so two workgroups share a CU and one's loads and stores
// overlap the other's sorting (1024 x 9 ran one per CU: 11.1 -> 8.3 ms at
// 2^30 in microbench_bucket)
#ifndef SA_BS_BLOCK
#define SA_BS_BLOCK 512
#endif
constexpr int kBsBlock = SA_BS_BLOCK;
#ifndef SA_BS_ITEMS
#define SA_BS_ITEMS 18
#endif
constexpr int kBsItems = SA_BS_ITEMS;
constexpr int kBsCap = kBsBlock * kBsItems;  // 9216 suffixes per window
constexpr uint32_t kWinStride = 1024;        // nominal window spacing W
// persistent workgroups per CU of the fixed-span local sort (k_bucket_sort)
#ifndef SA_BS_WPC
#define SA_BS_WPC 2
#endif
constexpr uint32_t kBsWpc = SA_BS_WPC;
#ifndef SA_BS_GRID
#define SA_BS_GRID (1u << 22)
#endif
// one workgroup per window: the dispatcher balances the windows (a grid
// of 1024 workgroups looping over them: 7.90 ms at 2^30, 8192: 7.58,
// one per window: 7.40; interleaved A/B on one box)
constexpr uint32_t kBsGrid = SA_BS_GRID;
constexpr uint64_t kBucketMinN = 1ull << 20; // auto: bucketed first round from 1 Mi suffixes
// bucket digits: the first pass (unstable, atomic cursors) takes the low
// kLoBits, the second (stable, look-back) the remaining bb - kLoBits (9 + 8
// at 2^30: 7.1 + 8.2 ms, 8 + 9: 6.0 + 9.0 ms)
constexpr uint32_t kLoBits = 8;
constexpr uint32_t kLoRadix = 1u << kLoBits;

__device__ __forceinline__ uint32_t bucket_of(uint64_t key1, uint32_t rb, uint64_t cmul, uint32_t bsh) {
    return (uint32_t)(((key1 >> rb) * cmul) >> bsh);
}

// smallest D of bucket b (D * cmul >> bsh is monotone: d0 = floor(b 2^bsh /
// cmul) has bucket <= b and d0 + 1 bucket >= b).  Bucket-relative items
// (second pass output) are w = (key1 - (Dmin(b) << rb)) << ib | idx, which
// fits 64 bits by plan_bucketed's span + rb + ib <= 64.
__device__ __forceinline__ uint32_t bucket_dmin(uint32_t b, uint64_t cmul, uint32_t bsh) {
    const uint64_t d0 = ((uint64_t)b << bsh) / cmul;
    return (uint32_t)((((d0 * cmul) >> bsh) == b) ? d0 : d0 + 1);
}

// radix source of the second bucket pass (digits of bucket_of(key))
// (digits of the LOCAL bucket, bucket_of(key) - bofs: bofs = the first bucket
// of this rank's range in the range-partitioned build, 0 on one GPU)
struct SrcBucketKeys {
    const uint64_t* __restrict__ keys;
    const uint32_t* __restrict__ vals;
    uint32_t rb, bsh;
    uint64_t cmul;
    uint32_t bofs;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return keys[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return vals[e]; }
    static constexpr bool kPk8 = false;
    __device__ __forceinline__ uint32_t digit(uint64_t k, uint32_t shift, uint32_t mask) const {
        return ((bucket_of(k, rb, cmul, bsh) - bofs) >> shift) & mask;
    }
};

// radix source of the second bucket pass over the first pass's packed items
// (k_split_text<.., PK8>): the digit is the item's top hb bits (shift 64 -
// hb), and the item below them is already the bucket-relative output word
struct SrcPk8 {
    const uint64_t* __restrict__ items;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return items[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t) const { return 0u; }
    static constexpr bool kPk8 = true;
};

// NW consecutive bytes of an LDS byte array (viewed as words) starting at
// byte `off` (any alignment), as NW / 4 words: one word read per output
// word + 1, then v_alignbyte (the per-byte ds_read_u8 of a rolling update
// cost more than its arithmetic)
template <int NB>
__device__ __forceinline__ void lds_bytes(const uint32_t* __restrict__ w32, uint32_t off, uint32_t (&out)[NB / 4]) {
    static_assert(NB % 4 == 0, "whole words");
    const uint32_t base = off >> 2, sh = off & 3u;
    uint32_t w[NB / 4 + 1];
#pragma unroll
    for (int q = 0; q <= NB / 4; ++q) w[q] = w32[base + q];
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) out[q] = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
}
template <int NB>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&v)[NB / 4], int j) {
    return (v[j >> 2] >> (8 * (j & 3))) & 0xFFu;
}

// ---------------------------------------------------------------------------
// Digit totals of the first bucket pass straight from the text: the bucket
// depends on D (the first s dense digits, < 2^32: plan_bucketed) only, so
// each lane rolls D in 32 bits over 16 consecutive positions; an LDS
// histogram of the low kLoBits -> ghist[0 .. kLoRadix) (the high bits are
// counted by the first pass itself, k_split_text).  Grid-stride over
// 4096-position tiles.
// ---------------------------------------------------------------------------
// POW2: sigma a power of two (shifts and masks, the bucket a bit field of D)
// Bucket range (the range-partitioned build, sa_dist.h): only positions in
// [p0, p1) whose bucket lies in [blo, bhi) are counted, by their LOCAL bucket
// bk - blo; the single-GPU build passes [0, n) and [0, 2^bb).
// COARSE: the histogram is of (bucket >> cshift) over kCoarse 64-bit bins
// (ghist then points at uint64 words) instead of the low kLoBits of the local
// bucket (the cut plan of sa_dist.h).
constexpr uint32_t kCoarseBits = 12;
constexpr uint32_t kCoarse = 1u << kCoarseBits;

// LM (list mode), for the record-driven first pass (k_split_list) of one
// rank's bucket range: the suffixes counted are written as compacted records
// (key1 -> lkeys, position -> lpos), key1 computed from the LDS-staged digits
// for the kept positions only (~1/G of them).  Two launches over the same
// grid: LM = 1 histograms and counts each workgroup's kept positions (wg[]),
// an exclusive scan (k_exscan_u32) turns the counts into offsets, LM = 2
// writes each workgroup's records from its offset (no claims: a claim per
// 4096-position tile on one counter serialised; LM = 1 keeps the plain
// histogram's occupancy).
// LM = 3: one launch instead of LM = 1 + LM = 2 -- the records of a tile go
// to one of kRecStripes regions of rcap records (stripe = workgroup mod
// kRecStripes; the grid a multiple of it, so a stripe takes every
// kRecStripes-th tile of the text), their place claimed per tile from the
// stripe's cursor wg[stripe]; the low-digit histogram as LM = 1.  A stripe
// whose records outgrow rcap sets *rovf and writes none past it (the caller
// re-runs with LM = 1 + 2).
// IDENT: sigma = 256 (every byte value present), so the dense digit is the
// byte itself: no LDS byte map (configs[3]'s byte256 text: each rank scans
// the whole 4 GiB text twice)
// DNA (POW2): the text's alphabet is exactly {A, C, G, T}: dense digits by
// ((b >> 1) ^ (b >> 2)) & 3 per byte, four at once (as k_split_text)
constexpr uint32_t kRecStripes = 64;
constexpr uint32_t kXq = 8;   // second-pass queues = XCDs (sa_split.h SegXq, XqWin below)
constexpr uint32_t kRecCurStride = 64;   // words between stripe cursors (atomics on one line serialise)
// record slots of a range of m suffixes: the striped regions' 1/8 margin and
// two tiles of slack per stripe
constexpr uint64_t rec_capacity(uint64_t m) { return m + m / 8 + kRecStripes * (2ull * kTile + 1); }
template <bool POW2 = false, bool COARSE = false, int LM = 0, bool IDENT = false, bool DNA = false>
__global__ __launch_bounds__(kBlock) void k_bucket_hist(const uint8_t* __restrict__ text, uint64_t n,
                                                        const uint16_t* __restrict__ code, BucketSpec b,
                                                        uint32_t* __restrict__ ghist, uint64_t p0, uint64_t p1,
                                                        uint32_t blo, uint32_t bhi,
                                                        uint64_t* __restrict__ lkeys = nullptr,
                                                        uint32_t* __restrict__ lpos = nullptr,
                                                        uint32_t* __restrict__ wg = nullptr, uint32_t rcap = 0,
                                                        uint32_t* __restrict__ rovf = nullptr) {
    constexpr bool REC = LM == 2 || LM == 3;   // records written
    constexpr int RUN = kTile / kBlock;   // 16
    constexpr uint32_t NB = COARSE ? kCoarse : kLoRadix;
    __shared__ uint32_t s_tmp[kWaves];
    // LM = 2: the tile's kept positions (tile offsets), compacted
    __shared__ uint16_t s_rp[REC ? kTile : 1];
    __shared__ uint32_t s_claim;
    __shared__ uint8_t s_map[256];
    __shared__ __attribute__((aligned(16))) uint32_t s_dcw[(kTile + kMaxK) / 4 + 8];   // dense digits, 4 per word (+ slack)
    uint8_t* s_dc = reinterpret_cast<uint8_t*>(s_dcw);
    __shared__ uint32_t s_hlo[NB];
    // DNA records: the tile's digits packed 2 bits each, 16 per word (the
    // first on top) + the halo, so a record's K <= 32 symbols are three word
    // reads instead of K byte reads
    constexpr bool PKD = DNA && REC;
    __shared__ uint32_t s_pk[PKD ? kBlock + kMaxK / 16 + 2 : 1];
    {
        const uint32_t cv = code[threadIdx.x];
        s_map[threadIdx.x] = (uint8_t)(cv ? cv - 1u : 0u);
    }
    for (uint32_t i = threadIdx.x; i < NB; i += kBlock) s_hlo[i] = 0;
    const uint32_t sig = b.sigma, ps1 = (uint32_t)b.pow_s1;
    const uint32_t shh = b.bsh;
    const uint32_t cshift = b.bb > kCoarseBits ? b.bb - kCoarseBits : 0u;
    const uint32_t bspan = bhi - blo;
    __syncthreads();
    const uint64_t tiles = (p1 - p0 + kTile - 1) / kTile;
    uint32_t kept_lane = 0;                        // LM = 1: this lane's kept positions
    uint32_t run = LM == 2 ? wg[blockIdx.x] : 0u;  // LM = 2: the workgroup's next record slot
    const uint32_t stripe = blockIdx.x % kRecStripes;  // LM = 3
    const uint64_t rbase = (uint64_t)stripe * rcap;
    // the next tile's 16 text bytes per lane (and the halo byte of lanes <
    // kMaxK) are loaded while the current tile is counted: clamped to the
    // last tile, unconditional (a conditional load is waited for at the join)
    auto fetch = [&](uint64_t tt2, uint4& v, uint32_t& hv) {
        const uint64_t tb2 = p0 + tt2 * kTile;
        const uint64_t i2 = tb2 + (uint64_t)threadIdx.x * RUN;
        v = (i2 + RUN <= n && (((uintptr_t)(text + i2)) & 15) == 0) ? *reinterpret_cast<const uint4*>(text + i2)
                                                                     : make_uint4(0u, 0u, 0u, 0u);
        const uint64_t h2 = tb2 + kTile + threadIdx.x;
        hv = (threadIdx.x < (uint32_t)kMaxK && h2 < n) ? (uint32_t)text[h2] : 0u;
    };
    uint4 cv = make_uint4(0u, 0u, 0u, 0u);
    uint32_t chv = 0;
    if (blockIdx.x < tiles) fetch(blockIdx.x, cv, chv);
    for (uint64_t tt = blockIdx.x; tt < tiles; tt += gridDim.x) {
        const uint64_t tb = p0 + tt * kTile;
        uint4 nv;
        uint32_t nhv;
        const uint64_t tn = tt + gridDim.x;
        // LM = 3 issues the prefetch after its claim: a claim issued behind
        // the prefetch could only be waited for together with it
        if constexpr (LM != 3) fetch(tn < tiles ? tn : tiles - 1, nv, nhv);
        {
            const uint64_t i = tb + (uint64_t)threadIdx.x * RUN;
            uint32_t w[4];
            if (i + RUN <= n && (((uintptr_t)(text + i)) & 15) == 0) {
                const uint4 v = cv;
                w[0] = v.x;
                w[1] = v.y;
                w[2] = v.z;
                w[3] = v.w;
                if constexpr (DNA) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) w[q] = ((w[q] >> 1) ^ (w[q] >> 2)) & 0x03030303u;
                } else if constexpr (!IDENT) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t o = 0;
#pragma unroll
                        for (int y = 0; y < 4; ++y) o |= (uint32_t)s_map[(w[q] >> (8 * y)) & 0xFFu] << (8 * y);
                        w[q] = o;
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t o = 0;
                    for (int y = 0; y < 4; ++y) {
                        const uint64_t p = i + 4 * q + y;
                        o |= (p < n ? (uint32_t)s_map[text[p]] : 0u) << (8 * y);
                    }
                    w[q] = o;
                }
            }
            *reinterpret_cast<uint4*>(s_dc + threadIdx.x * RUN) = make_uint4(w[0], w[1], w[2], w[3]);
            if constexpr (PKD) {
                uint32_t pk = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t x = w[q];   // four digits 0..3, the first in the low byte
                    const uint32_t v = ((x & 3u) << 6) | ((x >> 4) & 0x30u) | ((x >> 14) & 0xCu) | (x >> 24);
                    pk |= v << (24 - 8 * q);
                }
                s_pk[threadIdx.x] = pk;
            }
            if (threadIdx.x < (uint32_t)kMaxK) {   // wave 0, every lane
                const uint64_t h = tb + kTile + threadIdx.x;
                const uint32_t hd = (h < n) ? (IDENT ? chv : (uint32_t)s_map[chv]) : 0u;
                s_dc[kTile + threadIdx.x] = (uint8_t)hd;
                if constexpr (PKD) {
                    // the halo's packed words: 16 lanes' digits OR-ed together
                    static_assert(kMaxK == kWave, "the halo is wave 0's");
                    uint32_t v = hd << (30 - 2 * (threadIdx.x & 15u));
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) v |= (uint32_t)__shfl_xor((int)v, o, kWave);
                    if ((threadIdx.x & 15u) == 0) s_pk[kBlock + threadIdx.x / 16] = v;
                    if (threadIdx.x < 2) s_pk[kBlock + kMaxK / 16 + threadIdx.x] = 0;
                }
            }
        }
        __syncthreads();
        const uint32_t l0 = threadIdx.x * RUN;
        uint32_t D = 0;
        const uint32_t lg = POW2 ? (uint32_t)__builtin_ctz(sig) : 0u;
        const uint32_t dmask = POW2 ? (lg * b.s >= 32 ? ~0u : (1u << (lg * b.s)) - 1u) : 0u;
        const uint32_t bksh = POW2 ? lg * b.s - b.bb : 0u;
        // the digits leaving (positions l0 .. l0 + 15) and entering (l0 + s ..)
        uint32_t xo[RUN / 4], xi[RUN / 4];
        // PKD: the lane's 32 symbols from l0 as one 64-bit word (its packed
        // word and the next); position l0 + j's bucket is bits [2j, 2j + bb)
        // from the top (bb <= 2s: the bucket is a bit field of D)
        uint64_t wpk = 0;
        // IDENT (sigma = 256, digit = byte): the lane's 20 bytes from l0 as
        // five aligned words; position l0 + j's bucket is the top bb bits of
        // the big-endian word at byte j (bb <= 32, a bit field of D)
        uint32_t wid[IDENT ? 5 : 1];
        if constexpr (IDENT) {
#pragma unroll
            for (int q = 0; q < 5; ++q) wid[q] = s_dcw[l0 / 4 + q];
        } else if constexpr (PKD) {
            wpk = ((uint64_t)s_pk[threadIdx.x] << 32) | s_pk[threadIdx.x + 1];
        } else {
            for (uint32_t q = 0; q < b.s; ++q) D = POW2 ? ((D << lg) | s_dc[l0 + q]) : D * sig + s_dc[l0 + q];
            lds_bytes<RUN>(s_dcw, l0, xo);
            lds_bytes<RUN>(s_dcw, l0 + b.s, xi);
        }
        const uint32_t pksh = 64u - b.bb;
        uint32_t keep = 0;   // LIST: bit j = position l0 + j is in the range
        // whole tiles inside [p0, p1) take the loop without the position test
        auto count = [&](auto wholec) {
            constexpr bool WHOLE = decltype(wholec)::value;
#pragma unroll
            for (int j = 0; j < RUN; ++j) {
                if (!PKD && !IDENT && j > 0) {
                    if constexpr (POW2) D = ((D << lg) | byte_at<RUN>(xi, j - 1)) & dmask;
                    else D = (D - byte_at<RUN>(xo, j - 1) * ps1) * sig + byte_at<RUN>(xi, j - 1);
                }
                if (WHOLE || tb + l0 + j < p1) {
                    uint32_t bk;
                    if constexpr (IDENT)
                        bk = __builtin_bswap32(__builtin_amdgcn_alignbyte(wid[j / 4 + 1], wid[j / 4], j % 4)) >> (32u - b.bb);
                    else
                        bk = PKD ? (uint32_t)((wpk << (2 * j)) >> pksh)
                             : POW2 ? (D >> bksh)
                                    : (uint32_t)(((uint64_t)D * b.cmul) >> shh);
                    if constexpr (COARSE) {
                        atomicAdd(&s_hlo[bk >> cshift], 1u);
                    } else {
                        const uint32_t lb = bk - blo;
                        if (lb < bspan) {
                            if (LM != 2) atomicAdd(&s_hlo[lb & (kLoRadix - 1)], 1u);
                            keep |= 1u << j;
                        }
                    }
                }
            }
        };
        if (tb + kTile <= p1) count(std::true_type{});   // uniform
        else count(std::false_type{});
        if (LM == 1) kept_lane += (uint32_t)__popc(keep);
        if constexpr (REC) {
            // the tile's kept positions compacted into LDS in order, then one
            // thread per record computes key1 from the staged digits (only
            // ~1/G of the positions) and writes it coalesced
            uint32_t tot;
            uint32_t off = block_exclusive_sum((uint32_t)__popc(keep), s_tmp, &tot);
            // (the claim's round trip overlaps the compaction)
            uint32_t clm = 0;
            if (LM == 3 && threadIdx.x == 0 && tot) clm = atomicAdd(&wg[stripe * kRecCurStride], tot);
            if constexpr (LM == 3) fetch(tn < tiles ? tn : tiles - 1, nv, nhv);
            while (keep) {
                const int j = __builtin_ctz(keep);
                keep &= keep - 1;
                s_rp[off++] = (uint16_t)(l0 + j);
            }
            if (LM == 3 && threadIdx.x == 0) s_claim = clm;
            __syncthreads();
            if constexpr (LM == 3) {
                const uint32_t cl = s_claim;
                if (cl + tot > rcap) {   // uniform: the stripe is full
                    if (threadIdx.x == 0) atomicOr(rovf, 1u);
                    tot = 0;
                }
            }
            const uint64_t rb = LM == 3 ? rbase + s_claim : (uint64_t)run;
            const uint32_t K = b.s + b.R;
            for (uint32_t t = threadIdx.x; t < tot; t += kBlock) {
                const uint32_t l = s_rp[t];
                uint32_t Dk = 0;
                uint64_t r = 0;
                if (PKD && K <= 32) {   // uniform
                    const uint32_t wi = l >> 4, off = 2u * (l & 15u);
                    const uint64_t a = s_pk[wi], bw = s_pk[wi + 1], cw = s_pk[wi + 2];
                    uint64_t win = ((a << 32) | bw) << off;
                    if (off) win |= cw >> (32u - off);
                    Dk = (uint32_t)(win >> (64u - 2u * b.s));
                    r = (win >> (64u - 2u * K)) & ((1ull << (2u * b.R)) - 1ull);
                } else {
                    for (uint32_t q = 0; q < b.s; ++q) Dk = POW2 ? ((Dk << lg) | s_dc[l + q]) : Dk * sig + s_dc[l + q];
                    for (uint32_t q = b.s; q < K; ++q) r = POW2 ? ((r << lg) | s_dc[l + q]) : r * sig + s_dc[l + q];
                }
                lkeys[rb + t] = ((uint64_t)Dk << b.rb) | bucket_low(b, r, n - (tb + l));
                lpos[rb + t] = (uint32_t)(tb + l);
            }
            if (LM == 2) run += tot;
        }
        cv = nv;
        chv = nhv;
        __syncthreads();
    }
    if (LM == 1) {
        uint32_t tot;
        block_exclusive_sum(kept_lane, s_tmp, &tot);
        if (threadIdx.x == 0) wg[blockIdx.x] = tot;
    }
    for (uint32_t i = threadIdx.x; i < NB; i += kBlock) {
        if (!s_hlo[i]) continue;
        if constexpr (COARSE)   // 64-bit bins (all-reduced as int64 by the caller)
            atomicAdd(reinterpret_cast<unsigned long long*>(ghist) + i, (unsigned long long)s_hlo[i]);
        else
            atomicAdd(&ghist[i], s_hlo[i]);
    }
}

// exclusive scan of cnt u32 entries into out (one workgroup of kBlock lanes,
// 16 entries per lane per step, carried across steps)
__global__ __launch_bounds__(kBlock) void k_exscan_u32(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint32_t cnt) {
    __shared__ uint32_t s_tmp[kWaves];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < cnt; base += kBlock * 16) {
        uint32_t v[16], sum = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t i = base + threadIdx.x * 16 + k;
            v[k] = i < cnt ? in[i] : 0u;
            sum += v[k];
        }
        uint32_t tot;
        uint32_t off = block_exclusive_sum(sum, s_tmp, &tot) + carry;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t i = base + threadIdx.x * 16 + k;
            if (i < cnt) out[i] = off;
            off += v[k];
        }
        carry += tot;
    }
}

// ---------------------------------------------------------------------------
// The same window starts from the bucket start table (bstart[0 .. nb],
// non-decreasing, bstart[nb] = n): ws[j] = the first bucket start >= j*W,
// a binary search in a 512 KiB table instead of a gallop over the keys;
// wb[j] = that bucket.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_window_starts_tab(const uint32_t* __restrict__ bstart, uint32_t nb,
                                                              uint64_t n, uint64_t nw, uint32_t* __restrict__ ws,
                                                              uint32_t* __restrict__ wb) {
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j <= nw; j += (uint64_t)gridDim.x * kBlock) {
        const uint64_t x = j * kWinStride;
        if (x >= n) {
            ws[j] = (uint32_t)n;
            wb[j] = nb;
            continue;
        }
        uint32_t lo = 0, len = nb + 1;   // lower_bound(bstart, x)
        while (len > 0) {
            const uint32_t half = len >> 1;
            if (bstart[lo + half] < x) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        ws[j] = bstart[lo];
        wb[j] = lo;   // the window's first bucket (its buckets: [wb[j], wb[j + 1]))
    }
}

// ---------------------------------------------------------------------------
// window starts over the bucket-sorted keys: ws[j] = first g >= j*W with
// g == 0, g == n or bucket(g) != bucket(g-1) (gallop, then bisect); j <= nw.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_window_starts(const uint64_t* __restrict__ keys, uint64_t n,
                                                          uint64_t nw, uint32_t rb, uint64_t cmul, uint32_t bsh,
                                                          uint32_t* __restrict__ ws) {
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j <= nw; j += (uint64_t)gridDim.x * kBlock) {
        const uint64_t x = j * kWinStride;
        uint64_t res;
        if (x >= n) {
            res = n;
        } else if (x == 0) {
            res = 0;
        } else {
            const uint32_t bx = bucket_of(keys[x - 1], rb, cmul, bsh);
            if (bucket_of(keys[x], rb, cmul, bsh) != bx) {
                res = x;
            } else {
                uint64_t lo = x, hi, step = 1;   // bucket(lo) == bx
                for (;;) {
                    hi = lo + step;
                    if (hi >= n) {
                        hi = n;
                        break;
                    }
                    if (bucket_of(keys[hi], rb, cmul, bsh) != bx) break;
                    lo = hi;
                    step *= 2;
                }
                while (hi - lo > 1) {   // first index in (lo, hi] past bucket bx (n counts)
                    const uint64_t mid = lo + (hi - lo) / 2;
                    if (bucket_of(keys[mid], rb, cmul, bsh) != bx) hi = mid;
                    else lo = mid;
                }
                res = hi;
            }
        }
        ws[j] = (uint32_t)res;
    }
}

// Non-empty windows -> list (any order: windows are independent), their
// number -> words[7] (one atomic per workgroup), the largest -> words[5].
__global__ __launch_bounds__(kBlock) void k_window_list(const uint32_t* __restrict__ ws, uint64_t nw,
                                                        uint32_t* __restrict__ list, uint32_t* __restrict__ words) {
    __shared__ uint32_t s_n[kWaves], s_base;
    __shared__ uint32_t s_mx[kWaves];
    const uint32_t lane = lane_id(), wave = wave_id();
    const uint64_t per = ((nw + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
    const uint64_t j0 = (uint64_t)blockIdx.x * per, j1 = j0 + per < nw ? j0 + per : nw;
    // the workgroup's non-empty windows first, then its one claim (a claim
    // per 256 windows serialised 4096 atomics on one word: 60 us at 2^30)
    uint32_t mx = 0, cnt = 0;
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += kBlock) {
        const uint32_t d = ws[j + 1] - ws[j];
        mx = d > mx ? d : mx;
        cnt += d != 0;
    }
    uint32_t tot;
    uint32_t off = block_exclusive_sum(cnt, s_n, &tot);
    if (threadIdx.x == 0) s_base = tot ? atomicAdd(&words[7], tot) : 0u;
    __syncthreads();
    off += s_base;
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += kBlock)
        if (ws[j + 1] != ws[j]) list[off++] = (uint32_t)j;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(mx, o, kWave);
        mx = y > mx ? y : mx;
    }
    if (lane == 0) s_mx[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int x = 0; x < kWaves; ++x) t = s_mx[x] > t ? s_mx[x] : t;
        if (t) atomicMax(&words[5], t);
    }
}

// ---------------------------------------------------------------------------
// Padded first-pass segments (one GPU, 2^26 <= n <= 2^31): instead of the
// exact digit totals of k_bucket_hist (one more read of the text, 0.48 ms at
// 2^30), the low-digit totals are estimated from one position per 2^ssh
// (pseudo-random inside each block, so a periodic text cannot alias the
// stride) and each digit's segment of the first pass's output gets the
// Poisson upper bound S (k + 4 sqrt k + 16) (1 + 1/32) slots.  The first
// pass claims within its segment and flags a claim past the segment's end
// (words[11]); the host then runs the round again with the exact totals.
// The second pass reads segment l as [start(l), start(l) + count(l)).
// ---------------------------------------------------------------------------
template <bool POW2>
__global__ __launch_bounds__(kBlock) void k_bucket_sample(const uint8_t* __restrict__ text, uint64_t n,
                                                          const uint16_t* __restrict__ code, BucketSpec b,
                                                          uint32_t ssh, uint32_t* __restrict__ ghist) {
    __shared__ uint8_t s_map[256];
    __shared__ uint32_t s_h[kLoRadix];
    {
        const uint32_t cv = code[threadIdx.x];
        s_map[threadIdx.x] = (uint8_t)(cv ? cv - 1u : 0u);
    }
    for (uint32_t i = threadIdx.x; i < kLoRadix; i += kBlock) s_h[i] = 0;
    __syncthreads();
    const uint32_t lg = POW2 ? (uint32_t)__builtin_ctz(b.sigma) : 0u;
    const uint32_t bksh = POW2 ? lg * b.s - b.bb : 0u;
    const uint64_t ns = n >> ssh;   // whole blocks only
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < ns; i += (uint64_t)gridDim.x * kBlock) {
        uint32_t hsh = (uint32_t)i * 0x9E3779B1u;
        hsh ^= hsh >> 15;
        hsh *= 0x85EBCA6Bu;
        hsh ^= hsh >> 13;
        const uint64_t p = (i << ssh) + (hsh >> (32 - ssh));
        // the s <= 32 bytes (sigma^s <= 2^32, plan_bucketed) loaded before any
        // is used: a load-use chain per byte took 0.106 ms for the 2^20
        // samples of 1 GiB DNA, 0.064 batched (profiles/r05_al_ab_sample_loads_*.txt)
        uint32_t raw[32];
#pragma unroll
        for (uint32_t q = 0; q < 32; ++q)
            raw[q] = (q < b.s && p + q < n) ? (uint32_t)text[p + q] : 256u;
        uint32_t D = 0;
#pragma unroll
        for (uint32_t q = 0; q < 32; ++q) {
            if (q < b.s) {
                const uint32_t c = raw[q] < 256u ? (uint32_t)s_map[raw[q]] : 0u;
                D = POW2 ? ((D << lg) | c) : D * b.sigma + c;
            }
        }
        const uint32_t bk = POW2 ? (D >> bksh) : (uint32_t)(((uint64_t)D * b.cmul) >> b.bsh);
        atomicAdd(&s_h[bk & (kLoRadix - 1)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kLoRadix; i += kBlock)
        if (s_h[i]) atomicAdd(&ghist[i], s_h[i]);
}

// sample counts -> padded segment starts pstart[0 .. kLoRadix] (one workgroup)
// (a total above `limit`, the buffers' capacity -- not expected: the bound
// sums to < 1.1 n -- gives every segment 0 slots: the first pass overflows
// and the round re-runs with the exact totals)
__global__ __launch_bounds__(kLoRadix) void k_pad_starts(const uint32_t* __restrict__ samples, uint32_t ssh,
                                                         uint32_t slack_off, uint32_t limit,
                                                         uint32_t* __restrict__ pstart) {
    __shared__ uint32_t s_tmp[kLoRadix / kWave];
    const uint32_t k = samples[threadIdx.x];
    const float bound = slack_off ? (float)k : (float)k + 4.0f * sqrtf((float)k) + 16.0f;
    uint64_t cap = (uint64_t)bound << ssh;
    cap = slack_off ? cap : cap + (cap >> 5);
    cap = (cap + 63) & ~63ull;
    const uint32_t c32 = (uint32_t)cap;   // host: n <= 2^31, total < 2^32
    const uint32_t inc = wave_inclusive_sum(c32);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t w = 0; w < wave_id(); ++w) off += s_tmp[w];
    __syncthreads();
    if (threadIdx.x == kLoRadix - 1) s_tmp[0] = off + inc;
    __syncthreads();
    const bool fits = s_tmp[0] <= limit;
    pstart[threadIdx.x] = fits ? off + inc - c32 : 0u;
    if (threadIdx.x == kLoRadix - 1) pstart[kLoRadix] = fits ? off + inc : 0u;
}

// ---------------------------------------------------------------------------
// Local sort of each listed window [ws[j], ws[j+1]) (whole buckets, at most
// CAP suffixes).  w = (key1 - min) << ib | idx (ib = bit width of n - 1) is
// unique per suffix, so no step has to be stable:
//   1. counting scatter on the top kSubBits of the key span: LDS histogram
//      (16-bit counters packed in pairs, atomics), scan, atomic cursors ->
//      s_w holds 2^kSubBits sub-buckets of a few suffixes each (random text);
//   2. each suffix counts the smaller keys of its sub-bucket (its rank in
//      it), then all move to their final slots;
//   3. s_w is written out in order: sorted key1 and SA, coalesced.
// A window with a sub-bucket above kMaxSub (many equal or clustered keys) is
// appended to `skew` (count in words[10]) and left to k_bucket_sort_lsd.
// err bit 0: window larger than the LDS tile; bit 1: key span too wide.
// ---------------------------------------------------------------------------
#ifndef SA_SUB_BITS
#define SA_SUB_BITS 11
#endif
constexpr int kSubBits = SA_SUB_BITS;
constexpr int kSubBuckets = 1 << kSubBits;
constexpr uint32_t kMaxSub = 64;
constexpr int kRetryWord = 13;   // words[]: fixed-span windows for the measured-span launch

// where the second pass's bucket-relative items (k_split_seg) sit: window j
// holds buckets [wb[j], wb[j + 1]); bucket b starts at bstart[b] and its
// smallest D is bdmin[b]
struct BucketRel {
    const uint32_t* __restrict__ wb;
    const uint32_t* __restrict__ bstart;
    const uint32_t* __restrict__ bdmin;
    uint32_t rb;
    // bit width of the largest bucket-relative key of one
    // bucket (0: measure each window's span)
    uint32_t bits1 = 0;
};

// window j's items -> registers as w = (key1 - min) << ib | idx, with key1 =
// (Dmin(bucket) << rb) + (item >> ib); false (and the error flag) when the
// key span does not fit beside the index bits.  s_bk: 2 x 32 words of LDS
// (the bucket starts and Dmin of a window of up to 32 buckets).
template <int BLOCK, int ITEMS>
__device__ __forceinline__ bool load_window(const uint64_t* __restrict__ w_in, const BucketRel& br, uint32_t j,
                                            uint64_t a, uint32_t m, uint32_t ib, uint64_t (&w)[ITEMS], uint64_t& mn,
                                            uint32_t& bits, uint64_t (*s_red)[BLOCK / kWave],
                                            uint32_t (*s_bk)[32], uint32_t* __restrict__ err, bool* fixed = nullptr) {
    if (fixed) *fixed = false;
    constexpr int WAVES = BLOCK / kWave;
    constexpr int WT = kWave * ITEMS;
    const uint32_t wave = wave_id(), lane = lane_id();
    const uint64_t imask = (ib >= 64) ? ~0ull : ((1ull << ib) - 1ull);
    const uint32_t b0 = br.wb[j], nbk = br.wb[j + 1] - b0;   // uniform
    uint32_t dmin0 = 0;
    if (nbk == 1) {
        dmin0 = br.bdmin[b0];
    } else if (nbk <= 32) {
        if (threadIdx.x < nbk) {
            s_bk[0][threadIdx.x] = br.bstart[b0 + threadIdx.x];
            s_bk[1][threadIdx.x] = br.bdmin[b0 + threadIdx.x];
        }
        __syncthreads();
    }
    // bucket of position p: the last of the window's buckets starting <= p
    auto dmin_of = [&](uint64_t p) -> uint32_t {
        if (nbk == 1) return dmin0;
        if (nbk <= 32) {
            uint32_t lo = 0;
            for (uint32_t step = 16; step; step >>= 1)
                if (lo + step < nbk && s_bk[0][lo + step] <= p) lo += step;
            return s_bk[1][lo];
        }
        uint32_t lo = b0, len = nbk;   // last b in [b0, b0 + nbk) with bstart[b] <= p
        while (len > 1) {
            const uint32_t half = len >> 1;
            if (br.bstart[lo + half] <= p) {
                lo += half;
                len -= half;
            } else {
                len = half;
            }
        }
        return br.bdmin[lo];
    };
    uint64_t mx = 0;
    mn = ~0ull;
    if (nbk == 1 && br.bits1) {
        // one bucket whose keys fill the plan's span (the compact layout):
        // the items are w already, the sub-buckets split the whole span --
        // no min / max reduction, no barrier
        const uint32_t l0 = wave * WT + lane;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const uint32_t le = l0 + i * kWave;
            w[i] = w_in[a + (le < m ? le : m - 1)];
        }
        bits = br.bits1;
        mn = (uint64_t)dmin0 << br.rb;
        if (fixed) *fixed = true;
        // the caller's zeroing of the sub-bucket counters must be done before
        // any wave counts (the min / max path's barrier did this; the loads
        // stay in flight across it)
        __syncthreads();
        return true;
    }
    if (nbk == 1) {
        // one bucket (the common case from 2^29 suffixes): the items are
        // (key1 - Dmin) << ib | idx already, so w = item - (min's key part
        // << ib) -- one 64-bit subtract per suffix, min / max on the items
        const uint32_t l0 = wave * WT + lane;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const uint32_t le = l0 + i * kWave;
            const uint64_t x = w_in[a + (le < m ? le : m - 1)];
            w[i] = x;
            mn = x < mn ? x : mn;
            mx = x > mx ? x : mx;
        }
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) {
            const uint64_t y0 = __shfl_xor(mn, o, kWave), y1 = __shfl_xor(mx, o, kWave);
            mn = y0 < mn ? y0 : mn;
            mx = y1 > mx ? y1 : mx;
        }
        if (lane == 0) {
            s_red[0][wave] = mn;
            s_red[1][wave] = mx;
        }
        __syncthreads();
#pragma unroll
        for (int x = 0; x < WAVES; ++x) {
            mn = s_red[0][x] < mn ? s_red[0][x] : mn;
            mx = s_red[1][x] > mx ? s_red[1][x] : mx;
        }
        const uint64_t mrel = mn >> ib, span = (mx >> ib) - mrel;
        bits = span ? 64u - (uint32_t)__clzll(span) : 0u;
        const uint64_t base = mrel << ib;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) w[i] -= base;
        mn = ((uint64_t)dmin0 << br.rb) + mrel;
        return true;
    }
    uint32_t v[ITEMS];
    // unpredicated loads (slots past m re-read the last suffix: no per-item
    // exec masks, which cost SGPRs and spills at 128 VGPRs); later phases
    // skip those slots by le < m
    const uint32_t l0 = wave * WT + lane;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t le = l0 + i * kWave;
        const uint64_t e = a + (le < m ? le : m - 1);
        const uint64_t x = w_in[e];
        v[i] = (uint32_t)(x & imask);
        w[i] = ((uint64_t)dmin_of(e) << br.rb) + (x >> ib);
        mn = w[i] < mn ? w[i] : mn;
        mx = w[i] > mx ? w[i] : mx;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const uint64_t y0 = __shfl_xor(mn, o, kWave), y1 = __shfl_xor(mx, o, kWave);
        mn = y0 < mn ? y0 : mn;
        mx = y1 > mx ? y1 : mx;
    }
    if (lane == 0) {
        s_red[0][wave] = mn;
        s_red[1][wave] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < WAVES; ++x) {
        mn = s_red[0][x] < mn ? s_red[0][x] : mn;
        mx = s_red[1][x] > mx ? s_red[1][x] : mx;
    }
    bits = (mx - mn) ? 64u - (uint32_t)__clzll(mx - mn) : 0u;
    if (bits + ib > 64) {   // uniform over the block
        if (threadIdx.x == 0) atomicOr(err, 2u);
        return false;
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) w[i] = ((w[i] - mn) << ib) | v[i];
    return true;
}

// ksh = 0: every sorted key1 to keys_out[p]; else only the key1 of every
// 2^ksh-th SA position p, to keys_out[p >> ksh] (the sparse rank look-ups
// search these samples, then the last 2^ksh slots by key1 rebuilt from SA and
// text: lower_bound_sampled in sa_kernels.h) -- 0.5 instead of 8 bytes per
// suffix written
template <int BLOCK, int ITEMS>
__device__ __forceinline__ void store_window(const uint64_t* __restrict__ s_w, uint64_t a, uint32_t m, uint32_t ib,
                                             uint64_t mn, uint64_t* __restrict__ keys_out,
                                             uint32_t* __restrict__ sa_out, uint32_t ksh) {
    constexpr int WT = kWave * ITEMS;
    const uint32_t wave = wave_id(), lane = lane_id();
    const uint64_t imask = (ib >= 64) ? ~0ull : ((1ull << ib) - 1ull);
    const uint64_t smask = (1ull << ksh) - 1ull;
#pragma unroll 2
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t le = wave * WT + i * kWave + lane;
        if (le < m) {
            const uint64_t x = s_w[le];
            const uint64_t p = a + le;
            if ((p & smask) == 0) keys_out[p >> ksh] = (x >> ib) + mn;
            sa_out[p] = (uint32_t)(x & imask);
        }
    }
}

// ---------------------------------------------------------------------------
// Round-1 segments of a sorted window (replaces k_seg_count + k_seg_write of
// the LSD first round, which re-read every sorted key twice): a window holds
// whole groups, so its heads (key differs from the previous: the re-rank of
// manber_myers.c:101-110), singletons and unsorted members (U) are found in
// LDS.  For every U member x at SA position p: rank[x] = (its group's head
// position) + 1, its member bit, and (p, x, local U-group id) at its
// window-local U index in tmp; cnt_u[j] / cnt_g[j] = the window's U members
// and U groups (scanned and gathered in SA order by k_scan_windows +
// k_u_gather).  Returns (heads, U, U groups) to thread 0.
// s_pre: WAVES * ITEMS u64 of scratch LDS (per-row running values).
// ---------------------------------------------------------------------------
struct SegOut {
    uint32_t* rank;
    uint32_t* member;
    uint64_t rank_off;   // global SA position of this rank's first suffix (0 on one GPU)
    uint32_t* tmp_pos;
    uint32_t* tmp_idx;
    uint32_t* tmp_g;
    uint32_t* cnt_u;
    uint32_t* cnt_g;
    uint32_t ksh;   // sorted key1 written for every 2^ksh-th SA position only (store_window)
    // non-null (range-partitioned build): each unsorted member's rank goes to
    // tmp_rank at its window-local U index instead of rank[x] -- the compact
    // rank map's slots are known only once the member bitmap is complete, so
    // k_u_gather places them
    uint32_t* tmp_rank = nullptr;
    // 0: k_bucket_sort writes no key1 samples (one GPU: round 2 keys by key1
    // from the text, SrcUKey1; a later round that searches the samples has
    // them rebuilt first by k_key1_samples)
    uint32_t samples = 1;
};

template <int BLOCK, int ITEMS>
__device__ __forceinline__ void window_segments(const uint64_t* __restrict__ s_w, uint64_t* __restrict__ s_pre,
                                                uint64_t (*s_red)[BLOCK / kWave], uint64_t a, uint32_t m, uint32_t ib,
                                                uint32_t j, const SegOut& so, uint64_t& tot_h, uint64_t& tot_u,
                                                uint64_t& tot_g) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int WT = kWave * ITEMS;
    const uint32_t wave = wave_id(), lane = lane_id();
    // head / unsorted / unsorted-head masks of row rb0 (s = rb0 + lane)
    auto masks = [&](uint32_t rb0, uint64_t& mh, uint64_t& mu, uint64_t& muh) {
        const uint32_t le = rb0 + lane;
        const bool ok = le < m;
        const uint32_t lc = ok ? le : m - 1;   // three independent LDS reads, no branches
        const uint64_t cur = s_w[lc] >> ib;
        const uint64_t prv = s_w[lc ? lc - 1 : 0] >> ib;
        const uint64_t nxt = s_w[lc + 1 < m ? lc + 1 : lc] >> ib;
        const bool head = ok && (le == 0 || prv != cur);
        const bool nhead = ok && (le + 1 == m || nxt != cur);
        const bool in_u = ok && !(head && nhead);
        mh = __ballot(head);
        mu = __ballot(in_u);
        muh = __ballot(head && in_u);
    };
    // 1. per row: the wave's running (last head, U, U heads) before it; per
    // wave: which rows hold U members, and the totals
    int32_t last_h = -1;
    uint32_t nh = 0, nu = 0, ng = 0;
    uint32_t urows = 0;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t rb0 = wave * WT + i * kWave;
        if (rb0 >= m) break;   // uniform per wave
        uint64_t mh, mu, muh;
        masks(rb0, mh, mu, muh);
        if (lane == 0) s_pre[wave * ITEMS + i] = (uint64_t)(uint32_t)last_h | ((uint64_t)nu << 32) | ((uint64_t)ng << 48);
        if (mu) urows |= 1u << i;
        if (mh) last_h = (int32_t)(rb0 + 63 - __clzll(mh));
        nh += __popcll(mh);
        nu += __popcll(mu);
        ng += __popcll(muh);
    }
    if (lane == 0) {
        s_red[0][wave] = (uint64_t)(uint32_t)last_h | ((uint64_t)nh << 32);
        s_red[1][wave] = (uint64_t)nu | ((uint64_t)ng << 32);
    }
    __syncthreads();
    // 2. carries from the earlier waves, then only the rows holding U members
    int32_t cw = -1;
    uint32_t bu = 0, bg = 0, th = 0, tu = 0, tg = 0;
#pragma unroll
    for (int x = 0; x < WAVES; ++x) {
        const uint64_t v0 = s_red[0][x], v1 = s_red[1][x];
        if (x < (int)wave) {
            if ((int32_t)(uint32_t)v0 >= 0) cw = (int32_t)(uint32_t)v0;
            bu += (uint32_t)v1;
            bg += (uint32_t)(v1 >> 32);
        }
        th += (uint32_t)(v0 >> 32);
        tu += (uint32_t)v1;
        tg += (uint32_t)(v1 >> 32);
    }
    if (threadIdx.x == 0) {
        so.cnt_u[j] = tu;
        so.cnt_g[j] = tg;
        tot_h += th;
        tot_u += tu;
        tot_g += tg;
    }
    const uint64_t imask = (ib >= 64) ? ~0ull : ((1ull << ib) - 1ull);
    const uint64_t lt = lanemask_lt(), lem = lt | (1ull << lane);
    while (urows) {   // uniform per wave
        const uint32_t i = (uint32_t)__builtin_ctz(urows);
        urows &= urows - 1;
        const uint32_t rb0 = wave * WT + i * kWave;
        uint64_t mh, mu, muh;
        masks(rb0, mh, mu, muh);
        const uint64_t pre = s_pre[wave * ITEMS + i];
        const int32_t ph = (int32_t)(uint32_t)pre;
        const int32_t ch = ph >= 0 ? ph : cw;
        if ((mu >> lane) & 1ull) {
            const uint64_t hl = mh & lem;
            const uint32_t hpos = hl ? rb0 + 63 - (uint32_t)__clzll(hl) : (uint32_t)ch;
            const uint32_t ku = bu + (uint32_t)((pre >> 32) & 0xFFFFu) + (uint32_t)__popcll(mu & lt);
            const uint32_t kg = bg + (uint32_t)(pre >> 48) + (uint32_t)__popcll(muh & lem) - 1u;
            const uint32_t x = (uint32_t)(s_w[rb0 + lane] & imask);
            const uint32_t rv = (uint32_t)(so.rank_off + a + hpos + 1u);
            if (so.tmp_rank) so.tmp_rank[a + ku] = rv;
            else so.rank[x] = rv;
            atomicOr(&so.member[x >> 5], 1u << (x & 31));
            so.tmp_pos[a + ku] = (uint32_t)(a + rb0 + lane);
            so.tmp_idx[a + ku] = x;
            so.tmp_g[a + ku] = kg;
        }
    }
}

// per-workgroup totals of window_segments -> words[0..2] (D, m, G)
__device__ __forceinline__ void flush_totals(uint32_t* __restrict__ words, uint64_t th, uint64_t tu, uint64_t tg) {
    if (threadIdx.x == 0) {
        if (th) atomicAdd(&words[0], (uint32_t)th);
        if (tu) atomicAdd(&words[1], (uint32_t)tu);
        if (tg) atomicAdd(&words[2], (uint32_t)tg);
    }
}

// Exclusive scan in place of cnt_u[0..nw] and cnt_g[0..nw] (entry nw enters
// as 0 and leaves as the total), in blocks of kWsBlock entries:
// k_wscan_reduce (block sums) -> k_wscan_top (their scan, one workgroup) ->
// k_wscan_apply (each block rescanned from its offset).
constexpr int kWsPer = 8;
constexpr int kWsBlock = kBlock * kWsPer;   // 2048 entries per workgroup

__device__ __forceinline__ void wscan_load(const uint32_t* __restrict__ c, uint64_t nw, uint64_t b0, uint32_t (&x)[kWsPer],
                                           uint32_t& sum) {
    sum = 0;
#pragma unroll
    for (int k = 0; k < kWsPer; ++k) {
        const uint64_t i = b0 + threadIdx.x * kWsPer + k;
        x[k] = i <= nw ? c[i] : 0u;
        sum += x[k];
    }
}

__global__ __launch_bounds__(kBlock) void k_wscan_reduce(const uint32_t* __restrict__ cu, const uint32_t* __restrict__ cg,
                                                         uint64_t nw, uint32_t* __restrict__ part) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint64_t b0 = (uint64_t)blockIdx.x * kWsBlock;
    uint32_t x[kWsPer], su, sg, tu, tg;
    wscan_load(cu, nw, b0, x, su);
    wscan_load(cg, nw, b0, x, sg);
    block_exclusive_sum(su, s_tmp, &tu);
    block_exclusive_sum(sg, s_tmp, &tg);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = tu;
        part[2 * blockIdx.x + 1] = tg;
    }
}

__global__ __launch_bounds__(kBlock) void k_wscan_top(uint32_t* __restrict__ part, uint32_t blocks) {
    __shared__ uint32_t s_tmp[kWaves];
    uint32_t carry_u = 0, carry_g = 0;
    for (uint32_t b0 = 0; b0 < blocks; b0 += kBlock) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t u = b < blocks ? part[2 * b] : 0u, g = b < blocks ? part[2 * b + 1] : 0u;
        uint32_t tu, tg;
        const uint32_t eu = block_exclusive_sum(u, s_tmp, &tu) + carry_u;
        const uint32_t eg = block_exclusive_sum(g, s_tmp, &tg) + carry_g;
        if (b < blocks) {
            part[2 * b] = eu;
            part[2 * b + 1] = eg;
        }
        carry_u += tu;
        carry_g += tg;
    }
}

__global__ __launch_bounds__(kBlock) void k_wscan_apply(uint32_t* __restrict__ cu, uint32_t* __restrict__ cg, uint64_t nw,
                                                        const uint32_t* __restrict__ part) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint64_t b0 = (uint64_t)blockIdx.x * kWsBlock;
    for (int a = 0; a < 2; ++a) {
        uint32_t* c = a ? cg : cu;
        uint32_t x[kWsPer], sum;
        wscan_load(c, nw, b0, x, sum);
        uint32_t off = block_exclusive_sum(sum, s_tmp, nullptr) + part[2 * blockIdx.x + a];
#pragma unroll
        for (int k = 0; k < kWsPer; ++k) {
            const uint64_t i = b0 + threadIdx.x * kWsPer + k;
            if (i <= nw) c[i] = off;
            off += x[k];
        }
    }
}

// each listed window's U members from tmp (window-local order) to their
// compacted SA-order slots; one wave per window
// (so.tmp_rank: each member's rank also to rank[rm.slot(x)], the compact
// rank map of the range-partitioned build)
__global__ __launch_bounds__(kBlock) void k_u_gather(const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ words,
                                                     const uint32_t* __restrict__ ws, const uint32_t* __restrict__ ou,
                                                     const uint32_t* __restrict__ og, SegOut so,
                                                     uint32_t* __restrict__ u_pos, uint32_t* __restrict__ u_idx,
                                                     uint32_t* __restrict__ u_g, RankMap rm = RankMap{}) {
    const uint32_t nlist = words[7];
    const uint32_t lane = lane_id();
    for (uint64_t q = (uint64_t)blockIdx.x * kWaves + wave_id(); q < nlist; q += (uint64_t)gridDim.x * kWaves) {
        const uint32_t j = list[q];
        const uint32_t a = ws[j], o = ou[j], c = ou[j + 1] - o, g0 = og[j];
        for (uint32_t k = lane; k < c; k += kWave) {
            const uint32_t x = so.tmp_idx[a + k];
            u_pos[o + k] = so.tmp_pos[a + k];
            u_idx[o + k] = x;
            u_g[o + k] = so.tmp_g[a + k] + g0;
            if (so.tmp_rank) so.rank[rm.slot(x)] = so.tmp_rank[a + k];
        }
    }
}

// Exclusive popcount scan of a bitmap of nw words (the compact rank map's
// prefix, RankMap): k_popc_reduce (per-block popcount sums) -> k_popc_top
// (their exclusive scan, one workgroup) -> k_popc_apply (each block's words
// rescanned from its offset; one prefix word per 8 bitmap words).  kPcPer consecutive words per thread, moved as
// 16-byte vectors (bits and prefix are hipMalloc bases); kPcBlock words per
// block.  (8 scalar words per thread and a top scan of 256 sums per step:
// 0.24 ms for the 2^25 words of 1 GiB.)
constexpr int kPcPer = 16;
constexpr int kPcBlock = kBlock * kPcPer;   // 4096 words per workgroup

__device__ __forceinline__ void popc_load(const uint32_t* __restrict__ bits, uint64_t nw, uint64_t b0,
                                          uint32_t (&c)[kPcPer]) {
    if (b0 + kPcPer <= nw) {
#pragma unroll
        for (int q = 0; q < kPcPer / 4; ++q) {
            const uint4 v = reinterpret_cast<const uint4*>(bits + b0)[q];
            c[4 * q] = (uint32_t)__popc(v.x);
            c[4 * q + 1] = (uint32_t)__popc(v.y);
            c[4 * q + 2] = (uint32_t)__popc(v.z);
            c[4 * q + 3] = (uint32_t)__popc(v.w);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kPcPer; ++k) c[k] = b0 + k < nw ? (uint32_t)__popc(bits[b0 + k]) : 0u;
    }
}

__global__ __launch_bounds__(kBlock) void k_popc_reduce(const uint32_t* __restrict__ bits, uint64_t nw,
                                                        uint32_t* __restrict__ part) {
    __shared__ uint32_t s_tmp[kWaves];
    uint32_t c[kPcPer], sum = 0;
    popc_load(bits, nw, (uint64_t)blockIdx.x * kPcBlock + (uint64_t)threadIdx.x * kPcPer, c);
#pragma unroll
    for (int k = 0; k < kPcPer; ++k) sum += c[k];
    uint32_t tot;
    block_exclusive_sum(sum, s_tmp, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// one workgroup of kPcTop threads, each scanning a contiguous run of the
// block sums (one step for up to 16 K blocks)
constexpr int kPcTop = 1024;
__global__ __launch_bounds__(kPcTop) void k_popc_top(uint32_t* __restrict__ part, uint32_t blocks) {
    __shared__ uint32_t s_tmp[kPcTop / kWave];
    const uint32_t per = (blocks + kPcTop - 1) / kPcTop;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < blocks ? b0 + per : blocks;
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t b = b0; b < b1; ++b) sum += part[b];
    const uint32_t inc = wave_inclusive_sum(sum);
    if (lane_id() == kWave - 1) s_tmp[wave_id()] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
#pragma unroll
    for (int w = 0; w < kPcTop / kWave; ++w) run += w < (int)wave_id() ? s_tmp[w] : 0u;
#pragma unroll 8
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t v = part[b];
        part[b] = run;
        run += v;
    }
}

__global__ __launch_bounds__(kBlock) void k_popc_apply(const uint32_t* __restrict__ bits, uint64_t nw,
                                                       const uint32_t* __restrict__ part,
                                                       uint32_t* __restrict__ prefix) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint64_t b0 = (uint64_t)blockIdx.x * kPcBlock + (uint64_t)threadIdx.x * kPcPer;
    uint32_t c[kPcPer], sum = 0;
    popc_load(bits, nw, b0, c);
#pragma unroll
    for (int k = 0; k < kPcPer; ++k) sum += c[k];
    uint32_t run = block_exclusive_sum(sum, s_tmp, nullptr) + part[blockIdx.x];
    // one prefix word per 8-word block (RankMap)
    static_assert(kPcPer % 8 == 0, "whole 8-word blocks per thread");
#pragma unroll
    for (int q = 0; q < kPcPer / 8; ++q) {
        if (b0 + 8 * q < nw) prefix[(b0 >> 3) + q] = run;
#pragma unroll
        for (int k = 0; k < 8; ++k) run += c[8 * q + k];
    }
}

// Batcher's odd-even merge sort of N registers (N a power of two), fully
// unrolled: (N = 16) 63 compare-exchanges of u64.
template <int N>
__device__ __forceinline__ void sort_net(uint64_t (&v)[N]) {
#pragma unroll
    for (int p = 1; p < N; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; ++i)
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        const uint64_t x = v[i + j], y = v[i + j + k];
                        const bool sw = y < x;
                        v[i + j] = sw ? y : x;
                        v[i + j + k] = sw ? x : y;
                    }
}

// The same network on u32 keys: a compare-exchange is one v_min + one v_max.
template <int N>
__device__ __forceinline__ void sort_net32(uint32_t (&v)[N]) {
#pragma unroll
    for (int p = 1; p < N; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; ++i)
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        const uint32_t x = v[i + j], y = v[i + j + k];
                        v[i + j] = x < y ? x : y;
                        v[i + j + k] = x < y ? y : x;
                    }
}

constexpr int kNet = 16;   // sub-buckets up to this size are sorted in registers

// Sort one sub-bucket s_w[lo, lo + cnt) (cnt <= N) in registers: u32 sort
// keys = the key bits below the sub-bucket's (exact: equal <=> same group)
// over the slot, an N-input network, the items gathered by slot and written
// back; the sorted keys also give the groups: unsorted members (U, groups of
// two or more) and U groups added to nu / ng.
template <int N>
__device__ __forceinline__ void sort_sub(uint64_t* __restrict__ s_w, uint32_t lo, uint32_t cnt, uint32_t ib,
                                         uint32_t low_mask, uint32_t& nu, uint32_t& ng) {
    static_assert(N <= 16, "slot in 4 bits");
    uint32_t v[N];
#pragma unroll
    for (int t = 0; t < N; ++t)
        v[t] = (uint32_t)t < cnt ? (((uint32_t)(s_w[lo + t] >> ib) & low_mask) << 4) | (uint32_t)t : ~0u;
    sort_net32<N>(v);
    uint64_t x[N];
#pragma unroll
    for (int t = 0; t < N; ++t) x[t] = (uint32_t)t < cnt ? s_w[lo + (v[t] & 15u)] : 0ull;
    // bit t: slots t and t + 1 hold equal keys (one group)
    uint32_t eqm = 0;
#pragma unroll
    for (int t = 0; t + 1 < N; ++t) eqm |= ((v[t] ^ v[t + 1]) < 16u ? 1u : 0u) << t;
    eqm &= (1u << (cnt - 1)) - 1u;   // pairs inside the sub-bucket (1 <= cnt <= N)
#pragma unroll
    for (int t = 0; t < N; ++t)
        if ((uint32_t)t < cnt) s_w[lo + t] = x[t];
    nu += (uint32_t)__popc(eqm | (eqm << 1));
    ng += (uint32_t)__popc(eqm & ~(eqm << 1));
}

// a larger sub-bucket (rare on random text): insertion sort in LDS
__device__ __forceinline__ void sort_sub_lds(uint64_t* __restrict__ s_w, uint32_t lo, uint32_t hi, uint32_t ib,
                                             uint32_t& nu, uint32_t& ng) {
    for (uint32_t k = lo + 1; k < hi; ++k) {
        const uint64_t x = s_w[k];
        uint32_t y = k;
        while (y > lo && s_w[y - 1] > x) {
            s_w[y] = s_w[y - 1];
            --y;
        }
        s_w[y] = x;
    }
    uint64_t pr = ~0ull, cur = s_w[lo] >> ib;
    for (uint32_t k = lo; k < hi; ++k) {
        const uint64_t nx = k + 1 < hi ? (s_w[k + 1] >> ib) : ~0ull;
        const bool eqp = k > lo && pr == cur, eqn = k + 1 < hi && nx == cur;
        nu += (eqp || eqn) ? 1u : 0u;
        ng += (!eqp && eqn) ? 1u : 0u;
        pr = cur;
        cur = nx;
    }
}

// Instrumentation hook of k_bucket_sort: mark(k) at the end of phase k (0
// load, 1 histogram, 2 scan, 3 scatter, 4 sub-bucket sort, 5 U scan, 6 store;
// -1 = window start), flush(words) once per workgroup.  The library uses
// NoProbe (compiled away); microbench_bucket.hip passes a clock64() probe.
struct NoProbe {
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(uint32_t*) {}
};

template <int BLOCK, int ITEMS, class Probe = NoProbe>
__global__ __launch_bounds__(BLOCK, 4) void k_bucket_sort_wide(const uint64_t* __restrict__ keys_in, BucketRel br,
                                                       const uint32_t* __restrict__ ws,
                                                       const uint32_t* __restrict__ list, uint32_t* __restrict__ words,
                                                       uint32_t ib, uint64_t* __restrict__ keys_out,
                                                       uint32_t* __restrict__ sa_out, uint32_t* __restrict__ skew,
                                                       SegOut so, uint32_t* __restrict__ retry = nullptr,
                                                       uint32_t list_word = 7) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int CAP = BLOCK * ITEMS;
    constexpr int WT = kWave * ITEMS;
    __shared__ uint64_t s_w[CAP];
    __shared__ uint32_t s_cnt[kSubBuckets / 2];   // 16-bit counts, cursors, then ends; two per word
    __shared__ uint32_t s_tmp[WAVES];
    __shared__ uint32_t s_tmp2[WAVES];
    __shared__ uint64_t s_red[2][WAVES];
    __shared__ uint32_t s_bk[2][32];
    constexpr int WPT = kSubBuckets / 2 / BLOCK;   // counter words per thread
    static_assert(WPT >= 1 && WPT * 2 * BLOCK == kSubBuckets, "whole counter words per thread");

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    uint32_t* err = words + 6;
    const uint32_t nlist = words[list_word];
    auto end_of = [&](uint32_t sb) -> uint32_t { return (s_cnt[sb >> 1] >> (16 * (sb & 1))) & 0xFFFFu; };
    static_assert(WAVES * ITEMS * 8 <= kSubBuckets * 2, "per-row segment values fit in s_cnt");
    uint64_t th = 0, tu = 0, tg = 0;
    Probe probe;
    for (uint32_t q = blockIdx.x; q < nlist; q += gridDim.x) {
        probe.mark(-1);
        const uint32_t j = list[q];
        const uint64_t a = ws[j];
        const uint32_t m = (uint32_t)(ws[j + 1] - a);
        if (m > (uint32_t)CAP) {
            if (threadIdx.x == 0) atomicOr(err, 1u);
            continue;
        }
        for (int i = threadIdx.x; i < kSubBuckets / 2; i += BLOCK) s_cnt[i] = 0;
        uint64_t w[ITEMS];
        uint64_t mn;
        uint32_t bits;
        bool fixed;
        if (!load_window<BLOCK, ITEMS>(keys_in, br, j, a, m, ib, w, mn, bits, s_red, s_bk, err, &fixed)) {
            __syncthreads();
            continue;
        }
        probe.mark(0);
        uint32_t dsh = ib + (bits > (uint32_t)kSubBits ? bits - kSubBits : 0u);
        // 1. sub-bucket histogram (counts < 2^16: no carry between the halves)
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            if (wave * WT + i * kWave + lane < m) {
                const uint32_t sb = (uint32_t)(w[i] >> dsh) & (kSubBuckets - 1);
                atomicAdd(&s_cnt[sb >> 1], 1u << (16 * (sb & 1)));
            }
        }
        __syncthreads();
        probe.mark(1);
        // exclusive scan of the counts (2 WPT per thread, 16 bits each) and
        // their maximum
        uint32_t big = 0;
        {
            uint32_t c[2 * WPT], sum = 0, cm = 0;
#pragma unroll
            for (int x = 0; x < WPT; ++x) {
                const uint32_t pw = s_cnt[WPT * dg + x];
                c[2 * x] = pw & 0xFFFFu;
                c[2 * x + 1] = pw >> 16;
            }
#pragma unroll
            for (int x = 0; x < 2 * WPT; ++x) {
                sum += c[x];
                cm = c[x] > cm ? c[x] : cm;
            }
            const uint32_t inc = wave_inclusive_sum(sum);
#pragma unroll
            for (int o = kWave / 2; o > 0; o >>= 1) {
                const uint32_t y = __shfl_xor(cm, o, kWave);
                cm = y > cm ? y : cm;
            }
            if (lane == kWave - 1) s_tmp[wave] = inc;
            if (lane == 0) s_red[0][wave] = cm;
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int x = 0; x < WAVES; ++x) {
                off += (x < (int)wave) ? s_tmp[x] : 0u;
                big = (uint32_t)s_red[0][x] > big ? (uint32_t)s_red[0][x] : big;
            }
            uint32_t b = off + inc - sum;
#pragma unroll
            for (int x = 0; x < WPT; ++x) {
                const uint32_t b0 = b, b1 = b + c[2 * x];
                s_cnt[WPT * dg + x] = b0 | (b1 << 16);
                b = b1 + c[2 * x + 1];
            }
        }
        __syncthreads();
        probe.mark(2);
        if (big > kMaxSub) {   // uniform: clustered keys
            // a fixed-span window goes to the retry launch (its measured span
            // may spread the keys), else to the LSD kernel
            if (threadIdx.x == 0) {
                if (fixed && retry) retry[atomicAdd(&words[kRetryWord], 1u)] = j;
                else skew[atomicAdd(&words[10], 1u)] = j;
            }
            __syncthreads();
            continue;
        }
        // 2. scatter into sub-buckets (any order inside one) ...
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            if (wave * WT + i * kWave + lane < m) {
                const uint32_t sb = (uint32_t)(w[i] >> dsh) & (kSubBuckets - 1);
                const uint32_t old = atomicAdd(&s_cnt[sb >> 1], 1u << (16 * (sb & 1)));
                s_w[(old >> (16 * (sb & 1))) & 0xFFFFu] = w[i];
            }
        }
        __syncthreads();
        probe.mark(3);
        // ... then each thread sorts its 2 WPT consecutive sub-buckets: up to
        // kNet suffixes in registers (Batcher network), larger ones by
        // insertion in LDS.  Equal keys share a sub-bucket, so the sorted
        // sub-bucket also gives the groups: heads, unsorted members (U, groups
        // of two or more) and U heads, counted per thread in SA order.
        uint32_t nu = 0, ng = 0;
        uint32_t umask = 0;   // bit k: sub-bucket sb0 + k holds a group
        const uint32_t sb0 = 2 * WPT * dg;
        const uint32_t low_bits = bits > (uint32_t)kSubBits ? bits - kSubBits : bits;
        const uint32_t low_mask = low_bits >= 32 ? ~0u : ((1u << low_bits) - 1u);
        // the thread's four sub-buckets largest first: one of Poisson(~4.5)
        // sizes in 64 lanes exceeds 8 in most waves, but the second largest
        // of four rarely does, so iterations 2-4 mostly run the 8-input
        // network (wave-uniform choice) instead of the 16-input one
        static_assert(2 * WPT == 4, "four sub-buckets per thread");
        uint32_t order = 0;
        {
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t sb = sb0 + k;
                o[k] = ((end_of(sb) - (sb ? end_of(sb - 1) : 0u)) << 2) | (uint32_t)k;
            }
            sort_net32<4>(o);
#pragma unroll
            for (int k = 0; k < 4; ++k) order |= (o[3 - k] & 3u) << (2 * k);
        }
#pragma unroll 1
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t sb = sb0 + ((order >> (2 * i)) & 3u);
            const uint32_t lo = sb ? end_of(sb - 1) : 0u, hi = end_of(sb), cnt = hi - lo;
            const bool wide = __ballot(cnt > 8u) != 0ull;   // uniform
            // network sizes 4 / 8 / 12 / 16 by the wave's largest sub-bucket
            // of this rank (the largest of four is > 8 in almost every wave
            // but > 12 in about a fifth; the smallest is <= 4 in a third)
            const bool wide4 = __ballot(cnt > 4u) != 0ull, wide12 = __ballot(cnt > 12u) != 0ull;
            if (cnt == 0) continue;
            const uint32_t nu0 = nu;
            if (!wide4 && low_bits <= 28) sort_sub<4>(s_w, lo, cnt, ib, low_mask, nu, ng);
            else if (!wide && low_bits <= 28) sort_sub<8>(s_w, lo, cnt, ib, low_mask, nu, ng);
            else if (!wide12 && low_bits <= 28) sort_sub<12>(s_w, lo, cnt, ib, low_mask, nu, ng);
            else
            if (cnt <= (uint32_t)kNet && low_bits <= 28) sort_sub<kNet>(s_w, lo, cnt, ib, low_mask, nu, ng);
            else sort_sub_lds(s_w, lo, hi, ib, nu, ng);
            if (nu != nu0) umask |= 1u << (sb - sb0);
        }
        probe.mark(4);
        // exclusive U / U-group offsets of this thread's sub-buckets in the
        // window, and the window totals
        uint32_t bu, bg, th_w, tu_w, tg_w;
        {
            // nu, ng < 2^16 (a window holds <= kBsCap suffixes): one scan of
            // both; heads = singletons + U groups = m - U + G
            const uint32_t iug = wave_inclusive_sum(nu | (ng << 16));
            // its own LDS words: no barrier for the reads of the count scan's s_tmp
            uint32_t* const s_ug = s_tmp2;
            if (lane == kWave - 1) s_ug[wave] = iug;
            __syncthreads();
            uint32_t oug = 0, tug = 0;
#pragma unroll
            for (int x = 0; x < WAVES; ++x) {
                const uint32_t xug = s_ug[x];
                oug += (x < (int)wave) ? xug : 0u;
                tug += xug;
            }
            tu_w = tug & 0xFFFFu;
            tg_w = tug >> 16;
            th_w = m - tu_w + tg_w;
            bu = (oug & 0xFFFFu) + (iug & 0xFFFFu) - nu;
            bg = (oug >> 16) + (iug >> 16) - ng;
        }
        if (so.rank) {
            if (threadIdx.x == 0) {
                so.cnt_u[j] = tu_w;
                so.cnt_g[j] = tg_w;
                th += th_w;
                tu += tu_w;
                tg += tg_w;
            }
            // the unsorted members of this thread's sub-buckets (rare): rank =
            // group head position + 1, member bit, (p, x, U group) at their
            // window-local U index
            if (umask) {   // only the sub-buckets holding groups (never straddled)
                const uint64_t imask = (ib >= 64) ? ~0ull : ((1ull << ib) - 1ull);
                uint32_t ku = bu, kg = bg;
                for (uint32_t um = umask; um; um &= um - 1u) {
                    const uint32_t sb = sb0 + (uint32_t)__builtin_ctz(um);
                    const uint32_t lo = sb ? end_of(sb - 1) : 0u, hi = end_of(sb);
                    uint32_t head = lo;
                    uint64_t pr = ~0ull;
                    for (uint32_t k = lo; k < hi; ++k) {
                        const uint64_t x = s_w[k], r = x >> ib;
                        const uint64_t nx = k + 1 < hi ? (s_w[k + 1] >> ib) : ~0ull;
                        const bool eqp = k > lo && pr == r, eqn = k + 1 < hi && nx == r;
                        if (!eqp) head = k;
                        if (!eqp && eqn) ++kg;
                        if (eqp || eqn) {
                            const uint32_t xi = (uint32_t)(x & imask);
                            const uint32_t rv = (uint32_t)(so.rank_off + a + head + 1u);
                            if (so.tmp_rank) so.tmp_rank[a + ku] = rv;
                            else so.rank[xi] = rv;
                            atomicOr(&so.member[xi >> 5], 1u << (xi & 31));
                            so.tmp_pos[a + ku] = (uint32_t)(a + k);
                            so.tmp_idx[a + ku] = xi;
                            so.tmp_g[a + ku] = kg - 1u;
                            ++ku;
                        }
                        pr = r;
                    }
                }
            }
        }
        // (the U/G scan's barrier already follows every
        // thread's sort; the unsorted-set writes and the store only read s_w,
        // so the store need not wait for the few threads walking groups)
        probe.mark(5);
        store_window<BLOCK, ITEMS>(s_w, a, m, ib, mn, keys_out, sa_out, so.ksh);
        __syncthreads();   // s_w / s_cnt / s_red reuse by the next window
        probe.mark(6);
    }
    probe.flush(words);
    flush_totals(words, th, tu, tg);
}

// ---------------------------------------------------------------------------
// The fixed-span local sort over 32-bit LDS words.  For one-bucket windows of
// the compact layout (keys fill br.bits1 bits) the sub-bucket holds the top
// kSubBits of the key, so the bits below it (<= kLowMax) and the item's load
// slot (< 2^kSlotBits) fit one u32: the counting scatter writes that word,
// the sub-buckets are sorted as u32 words (networks without a gather by
// slot), and the store fetches the index of each sorted slot from a second
// LDS array (idx by load slot, written coalesced).  The register sort then
// needs 16 VGPRs instead of 48, which leaves room for the NEXT window's
// items: a workgroup takes windows from a ticket (dynamic, one ahead) and
// loads the next window right after scattering the current one into LDS,
// so the loads are in flight during the sort, the segments and the store.
// Windows: k_window_split lists the one-bucket windows with their headers
// (hdr, words[14]); the others, and windows whose keys cluster (a sub-bucket
// above kMaxSub), go to `retry` for k_bucket_sort_wide (measured span).
// ---------------------------------------------------------------------------
// This lane's first item slot of a window (wave-major rows of 64) as a value
// the compiler cannot hoist out of the window loop: kept live there, the
// ITEMS slot indices l0 + 64 i and the offsets derived from them took 36
// VGPRs and made the next window's loads spill
template <int ITEMS>
__device__ __forceinline__ uint32_t slot0() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return (t / kWave) * (kWave * ITEMS) + (t & (kWave - 1));
}

constexpr uint32_t kSlotBits = kBsCap > (1 << 14) ? 15 : 14;   // load slots of a window
constexpr uint32_t kSlotMask = (1u << kSlotBits) - 1u;
constexpr uint32_t kLowMax = 32 - kSlotBits;   // key bits below the sub-bucket
static_assert(kBsCap <= (1 << kSlotBits), "load slots in kSlotBits");
constexpr int kHdrWord = 14;                   // words[]: one-bucket windows listed by k_window_split
constexpr int kTicketWord = 15;                // words[]: k_bucket_sort's window ticket

// listed windows -> one-bucket windows with headers {j, a, m, Dmin} (fast:
// the fixed-span kernel runs) or the retry list (k_bucket_sort_wide)
// XQ (pc / pn: the per-region chunk starts and counts of k_bucket_starts_xq,
// [kXq][nb]): each one-bucket window's chunk header hx (load_items_xq).
__global__ __launch_bounds__(kBlock) void k_window_split(const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ ws, BucketRel br,
                                                         uint32_t* __restrict__ words, uint4* __restrict__ hdr,
                                                         uint32_t* __restrict__ retry, uint32_t fast,
                                                         const uint32_t* __restrict__ pc = nullptr,
                                                         const uint32_t* __restrict__ pn = nullptr, uint32_t nb = 0,
                                                         uint32_t* __restrict__ hx = nullptr, uint32_t crows = 0) {
    const uint32_t nlist = words[7];
    const uint32_t lane = lane_id();
    for (uint64_t q0 = (uint64_t)blockIdx.x * kBlock; q0 < nlist; q0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t q = q0 + threadIdx.x;
        uint32_t j = 0, b0 = 0;
        bool one = false;
        const bool ok = q < nlist;
        if (ok) {
            j = list[q];
            b0 = br.wb[j];
            one = fast && br.wb[j + 1] - b0 == 1u;
            // XQ: a chunk under 64 items could put two boundaries in one row
            // of 64 slots (k_window_rows): such windows take the wide kernel;
            // chunk rows (crows > 0: one chunk per row) need sum ceil(c / 64)
            // <= crows rows instead
            if (one && hx) {
                uint32_t nr = 0;
                for (uint32_t k = 0; k < kXq; ++k) {
                    const uint32_t c = pn[(uint64_t)k * nb + b0];
                    if (!crows && c && c < kWave) one = false;
                    nr += (c + kWave - 1) / kWave;
                }
                if (crows && nr > crows) one = false;
            }
        }
        const uint64_t m1 = __ballot(ok && one), m2 = __ballot(ok && !one);
        uint32_t base1 = 0, base2 = 0;
        if (lane == 0) {
            if (m1) base1 = atomicAdd(&words[kHdrWord], (uint32_t)__popcll(m1));
            if (m2) base2 = atomicAdd(&words[kRetryWord], (uint32_t)__popcll(m2));
        }
        base1 = (uint32_t)__shfl((int)base1, 0, kWave);
        base2 = (uint32_t)__shfl((int)base2, 0, kWave);
        if (ok && one) {
            const uint32_t a = ws[j];
            const uint32_t qi = base1 + (uint32_t)__popcll(m1 & lanemask_lt());
            hdr[qi] = make_uint4(j, a, ws[j + 1] - a, br.bdmin[b0]);
            if (hx) {
                uint32_t P = 0;
                for (uint32_t k = 0; k < kXq; ++k) {
                    const uint32_t c = pc[(uint64_t)k * nb + b0];
                    hx[(uint64_t)qi * 16 + k] = c - P;
                    if (k) hx[(uint64_t)qi * 16 + kXq - 1 + k] = P;
                    P += pn[(uint64_t)k * nb + b0];
                }
            }
        } else if (ok) {
            retry[base2 + (uint32_t)__popcll(m2 & lanemask_lt())] = j;
        }
    }
}

// XQ: the windows listed for k_bucket_sort_wide (by k_window_split: more
// than one bucket; by k_bucket_sort: keys that cluster) copied from their
// chunks in the per-XCD regions to their SA positions in `out` (which the
// wide / LSD window kernels then read), one workgroup per window; the chunks
// of bucket b in region k are [pc[k][b], pc[k][b] + pn[k][b]).
__global__ __launch_bounds__(kBlock) void k_window_gather(const uint32_t* __restrict__ list,
                                                          const uint32_t* __restrict__ words,
                                                          const uint32_t* __restrict__ ws,
                                                          const uint32_t* __restrict__ wb,
                                                          const uint32_t* __restrict__ pc,
                                                          const uint32_t* __restrict__ pn, uint32_t nb,
                                                          const uint64_t* __restrict__ in,
                                                          uint64_t* __restrict__ out) {
    const uint32_t nlist = words[kRetryWord];
    for (uint32_t qi = blockIdx.x; qi < nlist; qi += gridDim.x) {
        const uint32_t j = list[qi];
        uint64_t dst = ws[j];
        for (uint32_t b = wb[j]; b < wb[j + 1]; ++b) {
            for (uint32_t k = 0; k < kXq; ++k) {
                const uint32_t c = pn[(uint64_t)k * nb + b];
                const uint64_t src = pc[(uint64_t)k * nb + b];
                for (uint32_t t = threadIdx.x; t < c; t += kBlock) out[dst + t] = in[src + t];
                dst += c;
            }
        }
    }
}

// Sort one sub-bucket of u32 words s_k[lo, lo + cnt) (cnt <= N) in
// registers; equal key bits (above the slot) = one group: U members and U
// groups added to nu / ng
// LSV (local-sort variant, k_bucket_sort's VAR): bit 0 reads the N words
// unconditionally (s_k padded by kNet words; the words past the sub-bucket
// are masked by a select instead of an exec-masked load per word), bit 1
// writes back, for a sub-bucket without equal keys, the suffix index of
// each sorted word (s_x[slot]) instead of the word, so the store phase reads
// one sequential word per position (sub-buckets holding groups keep their
// sorted words for the U walk, which converts them).  Returns whether the
// sub-bucket holds a group.
template <int N, int LSV = 0>
__device__ __forceinline__ bool sort_sub_words(uint32_t* __restrict__ s_k, const uint32_t* __restrict__ s_x,
                                               uint32_t lo, uint32_t cnt, uint32_t& nu, uint32_t& ng) {
    uint32_t v[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        if constexpr (LSV & 1) {
            const uint32_t x = s_k[lo + t];
            v[t] = (uint32_t)t < cnt ? x : ~0u;
        } else {
            v[t] = (uint32_t)t < cnt ? s_k[lo + t] : ~0u;
        }
    }
    sort_net32<N>(v);
    uint32_t eqm = 0;
#pragma unroll
    for (int t = 0; t + 1 < N; ++t) eqm |= ((v[t] ^ v[t + 1]) <= kSlotMask ? 1u : 0u) << t;
    eqm &= (1u << (cnt - 1)) - 1u;
    if constexpr (LSV & 2) {
        if (eqm == 0u) {
            uint32_t xi[N];
#pragma unroll
            for (int t = 0; t < N; ++t) xi[t] = s_x[min(v[t] & kSlotMask, (uint32_t)kBsCap - 1u)];   // (padding: clamped)
#pragma unroll
            for (int t = 0; t < N; ++t)
                if ((uint32_t)t < cnt) s_k[lo + t] = xi[t];
            return false;
        }
    }
#pragma unroll
    for (int t = 0; t < N; ++t)
        if ((uint32_t)t < cnt) s_k[lo + t] = v[t];
    nu += (uint32_t)__popc(eqm | (eqm << 1));
    ng += (uint32_t)__popc(eqm & ~(eqm << 1));
    return eqm != 0u;
}

// a sub-bucket above kNet words (rare): insertion sort in LDS
__device__ __forceinline__ void sort_sub_words_lds(uint32_t* __restrict__ s_k, uint32_t lo, uint32_t hi, uint32_t& nu,
                                                   uint32_t& ng) {
    for (uint32_t k = lo + 1; k < hi; ++k) {
        const uint32_t x = s_k[k];
        uint32_t y = k;
        while (y > lo && s_k[y - 1] > x) {
            s_k[y] = s_k[y - 1];
            --y;
        }
        s_k[y] = x;
    }
    uint32_t pr = ~0u, cur = s_k[lo] >> kSlotBits;
    for (uint32_t k = lo; k < hi; ++k) {
        const uint32_t nx = k + 1 < hi ? (s_k[k + 1] >> kSlotBits) : ~0u;
        const bool eqp = k > lo && pr == cur, eqn = k + 1 < hi && nx == cur;
        nu += (eqp || eqn) ? 1u : 0u;
        ng += (!eqp && eqn) ? 1u : 0u;
        pr = cur;
        cur = nx;
    }
}

// The window's items into registers (slot le = l0 + 64 i; slots past m
// re-read the last item, see load_raw)
template <int ITEMS>
__device__ __forceinline__ void load_items(const uint64_t* __restrict__ w_in, uint64_t a, uint32_t m,
                                           uint64_t (&x)[ITEMS]) {
    const uint32_t l0 = slot0<ITEMS>();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t le = l0 + i * kWave;
        x[i] = w_in[a + (le < m ? le : m - 1)];
    }
}

// XQ windows (sa_split.h k_split_seg<.., XQ>): a one-bucket window's items
// are its bucket's chunks in the 8 per-XCD regions of the second pass's
// output.  Its header hx (16 words, k_window_split) holds, for chunk k,
// d[k] = (chunk start) - P_k and P_1..P_7 (P_k: the window slots before
// chunk k), so slot le reads w_in[d[k] + le] for the last k with P_k <= le.
// Its row table (k_window_rows) holds three words per row r of 64 slots
// (wave r / ITEMS, item r % ITEMS): d_a, d_b and split -- lanes below split
// read at d_a + le, the others at d_b + le (split 64: the row lies in one
// chunk; a window with a chunk under 64 items, whose rows could cross two
// boundaries, is not a fast window: k_window_split lists it for
// k_bucket_sort_wide).  Each wave loads its 18 rows' words into three VGPRs
// (lane i: row i) when it takes the next window's ticket and reads them by
// readlane at the prefetch point: a compare and a select per item on top of
// the contiguous load.  Measured alternatives (1 GiB DNA local sort, 3.5 ms
// over contiguous items): the table read at the prefetch point from memory
// 6.1 ms (a round trip before every load), staged through LDS 3.9 ms (the
// LDS store waited for the wave's previous stores), 18 scalar loads 4.2 ms
// (SGPR spills), a per-lane search of the header in a call for rows that
// cross a boundary 4.0 ms (the call waits for the loads in flight).
struct XqWin {
    const uint32_t* __restrict__ hx = nullptr;     // [hdr index][16]
    const uint32_t* __restrict__ rows = nullptr;   // [hdr index][3][rows per window]
};

// window slot le of chunk k: the last k with P_k <= le (P_0 = 0)
__device__ __forceinline__ uint32_t xq_offset(const uint32_t* __restrict__ hx, uint32_t le) {
    uint32_t off = hx[0];
#pragma unroll
    for (int k = 1; k < (int)kXq; ++k) off = hx[kXq - 1 + k] <= le ? hx[k] : off;
    return off;
}

// Chunk rows (CR, k_window_rows<true>): every row of 64 load slots reads ONE
// chunk -- the chunks' full rows first, in chunk order, then one partial row
// per chunk whose length is not a multiple of 64, then empty rows; the table
// holds per row its w_in index of lane 0 (t = 0) and its lanes holding items
// (t = 1: 64, the partial count or 0).  A load is then one uniform base and
// the lane (one readlane, no per-lane select or clamp: ~10 VALU per item
// fewer), at the price of up to 8 partial rows (k_window_split admits a
// window when sum ceil(chunk / 64) <= ROWS) whose idle lanes read up to 63
// items past their chunk, inside keys_u's slack, and are masked where the
// items are used.  The slots are no longer in window order; the sort does not
// need them to be.
template <int ITEMS>
__device__ __forceinline__ void load_items_cr(const uint64_t* __restrict__ w_in, const uint32_t (&rv)[3],
                                              uint64_t (&x)[ITEMS]) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)rv[0], i);
        x[i] = (w_in + base)[lane];
    }
}

// this wave's row words of a window: lane i < ITEMS holds word i of row
// (wave ITEMS + i) of table t (0: d_a, 1: d_b, 2: split; chunk rows: 0 base,
// 1 count)
template <int ITEMS, int ROWS>
__device__ __forceinline__ void load_rows_xq(const uint32_t* __restrict__ rows, uint32_t (&rv)[3]) {
    const uint32_t lane = lane_id();
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const uint32_t r = w * ITEMS + (lane < (uint32_t)ITEMS ? lane : 0u);
#pragma unroll
    for (int t = 0; t < 3; ++t) rv[t] = rows[t * ROWS + r];
}

template <int ITEMS>
__device__ __forceinline__ void load_items_xq(const uint64_t* __restrict__ w_in, const uint32_t (&rv)[3], uint32_t m,
                                              uint64_t (&x)[ITEMS]) {
    const uint32_t l0 = slot0<ITEMS>();
    const uint32_t lane = lane_id();
    const uint32_t last = m - 1;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t le = l0 + i * kWave;
        const uint32_t lc = le < m ? le : last;
        const uint32_t da = (uint32_t)__builtin_amdgcn_readlane((int)rv[0], i);
        const uint32_t db = (uint32_t)__builtin_amdgcn_readlane((int)rv[1], i);
        const uint32_t sp = (uint32_t)__builtin_amdgcn_readlane((int)rv[2], i);
        x[i] = w_in[(uint32_t)((lane < sp ? da : db) + lc)];
    }
}

// The row tables of the XQ one-bucket windows (k_window_split's headers
// words[kHdrWord], hx), one wave per window: row r covers slots [64 r,
// min(64 r + 63, m - 1)] (slots past m re-read item m - 1); at most one
// chunk boundary lies inside a row (k_window_split).
// CR: the chunk rows of load_items_cr instead.
template <bool CR>
__global__ __launch_bounds__(kBlock) void k_window_rows(const uint32_t* __restrict__ words, const uint4* __restrict__ hdr,
                                                        const uint32_t* __restrict__ hx, uint32_t nrows,
                                                        uint32_t* __restrict__ rows) {
    const uint32_t nh = words[kHdrWord];
    const uint32_t lane = lane_id();
    for (uint64_t q = (uint64_t)blockIdx.x * kWaves + wave_id(); q < nh; q += (uint64_t)gridDim.x * kWaves) {
        const uint32_t m = hdr[q].z;
        uint32_t hv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) hv[k] = hx[q * 16 + k];
        if constexpr (CR) {
            // chunk k: items [P_k, P_k+1) of the window at w_in[hv[k] + P_k ...]
            uint32_t st[kXq], cn[kXq], nfull = 0;
#pragma unroll
            for (int k = 0; k < (int)kXq; ++k) {
                const uint32_t p0 = k ? hv[kXq - 1 + k] : 0u, p1 = k + 1 < (int)kXq ? hv[kXq + k] : m;
                st[k] = hv[k] + p0;
                cn[k] = p1 - p0;
                nfull += cn[k] / kWave;
            }
            for (uint32_t r = lane; r < nrows; r += kWave) {
                uint32_t base = st[0], cnt = 0, rf = 0, rp = nfull;
#pragma unroll
                for (int k = 0; k < (int)kXq; ++k) {
                    const uint32_t nf = cn[k] / kWave, rem = cn[k] % kWave;
                    if (r >= rf && r < rf + nf) {
                        base = st[k] + kWave * (r - rf);
                        cnt = kWave;
                    }
                    if (rem && r == rp) {
                        base = st[k] + kWave * nf;
                        cnt = rem;
                    }
                    rf += nf;
                    rp += rem ? 1u : 0u;
                }
                uint32_t* const e = rows + q * 3 * nrows + r;
                e[0] = base;
                e[nrows] = cnt;
            }
            continue;
        }
        for (uint32_t r = lane; r < nrows; r += kWave) {
            const uint32_t lo = std::min(r * kWave, m - 1), hi = std::min(r * kWave + (kWave - 1), m - 1);
            uint32_t split = kWave;   // the first boundary inside (lo, hi]
#pragma unroll
            for (int k = kXq - 1; k >= 1; --k) {
                const uint32_t pk = hv[kXq - 1 + k];
                if (pk > lo && pk <= hi) split = pk - r * kWave;
            }
            uint32_t* const e = rows + q * 3 * nrows + r;
            e[0] = xq_offset(hv, lo);
            e[nrows] = xq_offset(hv, hi);
            e[2 * nrows] = split;
        }
    }
}

// bits: the plan's key span (br.bits1), kSubBits < bits <= kSubBits + kLowMax
// SA_LS_WFULL: waves whose slots all lie inside the window take the
// histogram, scatter and store loops without per-item bounds tests
#ifndef SA_LS_WFULL
#define SA_LS_WFULL 1
#endif
#ifndef SA_LS_CLAIMS
#define SA_LS_CLAIMS 1   // (must divide ITEMS; 3 / 6 / 9 at a time measured no faster: profiles/r06_t_ab_local_sort_claims.txt)
#endif
template <int BLOCK, int ITEMS, class Probe = NoProbe, bool XQ = false, int LSV = 0, bool CR = false>
__global__ __launch_bounds__(BLOCK, 4) void k_bucket_sort(const uint64_t* __restrict__ keys_in,
                                                       const uint4* __restrict__ hdr, uint32_t rb, uint32_t bits,
                                                       uint32_t ib, uint32_t* __restrict__ words,
                                                       uint64_t* __restrict__ keys_out, uint32_t* __restrict__ sa_out,
                                                       uint32_t* __restrict__ retry, SegOut so, XqWin xw = XqWin{}) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int CAP = BLOCK * ITEMS;
    static_assert(CAP <= (1 << kSlotBits), "load slots");
    // s_cnt first (LDS address 0: its byte addresses need no base); its
    // 16-bit counts, cursors and ends count BYTES of s_k (4 per word, at most
    // 4 CAP < 2^16), so a claimed cursor is the word's address
    // (one array: the compiler places separate __shared__ arrays largest first)
    // LSV bit 0: kNet words of padding after s_k (unconditional network reads)
    __shared__ uint32_t s_lds[kSubBuckets / 2 + CAP + ((LSV & 1) ? kNet : 0) + CAP];
    uint32_t* const s_cnt = s_lds;                    // two 16-bit halves per word: sub-buckets 2 t, 2 t + 1
    uint32_t* const s_k = s_lds + kSubBuckets / 2;   // (key bits below the sub-bucket) << kSlotBits | load slot
    uint32_t* const s_x = s_k + CAP + ((LSV & 1) ? kNet : 0);   // index of each load slot
    __shared__ uint32_t s_tmp[WAVES];
    __shared__ uint32_t s_cm[WAVES];
    __shared__ uint32_t s_ug[WAVES];
    __shared__ uint32_t s_q[2];
    __shared__ unsigned long long s_tot[3];   // heads, U, U groups of the workgroup's windows (thread 0)
    constexpr int WPT = kSubBuckets / 2 / BLOCK;   // counter words per thread
    static_assert(WPT * 2 == 4 && WPT * 2 * BLOCK == kSubBuckets, "four sub-buckets per thread");
    constexpr int ROWS = WAVES * ITEMS;   // XQ: row words per window (load_items_xq)

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    const uint32_t nwin = words[kHdrWord];
    const uint32_t low_bits = bits - kSubBits;
    const uint32_t dsh = ib + low_bits;
    const uint32_t lmask = (1u << low_bits) - 1u;
    const uint64_t imask = (1ull << ib) - 1ull;
    auto end_of = [&](uint32_t sb) -> uint32_t { return ((s_cnt[sb >> 1] >> (16 * (sb & 1))) & 0xFFFFu) >> 2; };
    static_assert(4 * CAP < (1 << 16), "byte counts in 16-bit halves");
    // sub-bucket sb = (w >> dsh) & 2047 of an item: y = w >> dsh, its counter
    // word's byte address (y << 1) & 0xFFC, the half's shift y << 4 (shifts
    // and bit-field extracts use the low 5 bits: (sb & 1) * 16)
    auto cnt_word = [&](uint32_t y) -> uint32_t* {
        return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_cnt) + ((y << 1) & 0xFFCu));
    };
    auto half_inc = [](uint32_t y) -> uint32_t {   // 4 << ((sb & 1) * 16)
        uint32_t r;
        asm("v_lshlrev_b32_e64 %0, %1, 4" : "=v"(r) : "v"(y << 4));
        return r;
    };
    Probe probe;
    if (threadIdx.x == 0) {
        s_q[0] = atomicAdd(&words[kTicketWord], 1u);
        s_tot[0] = s_tot[1] = s_tot[2] = 0;
    }
    __syncthreads();
    // window numbers and headers are uniform: scalar registers
    uint32_t q = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[0]);
    if (q >= nwin) return;   // uniform
    uint4 h = hdr[q];
    uint64_t w[ITEMS];
    // XQ: this window's row words (CR: its row counts mark the load slots
    // holding items)
    uint32_t rv[3] = {0u, 0u, 0u};
    if constexpr (XQ) {
        load_rows_xq<ITEMS, ROWS>(xw.rows + (uint64_t)q * 3 * ROWS, rv);
        if constexpr (CR) load_items_cr<ITEMS>(keys_in, rv, w);
        else load_items_xq<ITEMS>(keys_in, rv, h.z, w);
    } else {
        load_items<ITEMS>(keys_in, h.y, h.z, w);
    }
    uint32_t par = 0;
    for (;;) {
        probe.mark(-1);
        const uint32_t j = h.x, m = h.z;
        const uint64_t a = h.y;
        const uint64_t mn = (uint64_t)h.w << rb;
        if (threadIdx.x == 0) s_q[par ^ 1u] = atomicAdd(&words[kTicketWord], 1u);   // the next window
        for (int i = threadIdx.x; i < kSubBuckets / 2; i += BLOCK) s_cnt[i] = 0;
        __syncthreads();
        const uint32_t qn = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[par ^ 1u]);
        const bool more = qn < nwin;   // uniform
        // the next window's header (needed at the prefetch point only); past
        // the last window a dummy one-item window at 0, loaded but never
        // used -- an unconditional load keeps the current items dead after
        // the scatter (a conditional one kept them live through the sort)
        uint4 hn = make_uint4(0u, 0u, 1u, 0u);
        if (more) hn = hdr[qn];
        // XQ: the next window's row words of this wave (past the last
        // window: the current one's), for the prefetch
        uint32_t rwn[3] = {0u, 0u, 0u};
        if constexpr (XQ) load_rows_xq<ITEMS, ROWS>(xw.rows + (uint64_t)(more ? qn : q) * 3 * ROWS, rwn);
        probe.mark(0);
        const uint32_t l0 = slot0<ITEMS>();
        // 1. sub-bucket histogram (counts < 2^16: no carry between the halves)
        // wfull: this wave's SA positions all lie inside the window (the
        // store); sfull: its load slots all hold items (CR: its rows are all
        // full, else = wfull); slot_ok(i): item i of this lane holds one
        const bool wfull = SA_LS_WFULL && (wave + 1) * (uint32_t)(kWave * ITEMS) <= m;   // uniform per wave
        bool sfull = wfull;
        if constexpr (XQ && CR)
            sfull = SA_LS_WFULL && __ballot(lane < (uint32_t)ITEMS && rv[1] == kWave) == (1ull << ITEMS) - 1ull;
        auto slot_ok = [&](int i) -> bool {
            if constexpr (XQ && CR) return lane < (uint32_t)__builtin_amdgcn_readlane((int)rv[1], i);
            else return l0 + i * kWave < m;
        };
        if (sfull) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const uint32_t y = (uint32_t)(w[i] >> dsh);
                atomicAdd(cnt_word(y), half_inc(y));
            }
        } else {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                if (slot_ok(i)) {
                    const uint32_t y = (uint32_t)(w[i] >> dsh);
                    atomicAdd(cnt_word(y), half_inc(y));
                }
            }
        }
        __syncthreads();
        probe.mark(1);
        // exclusive scan of the counts and their maximum
        uint32_t big = 0;
        {
            uint32_t c[2 * WPT], sum = 0, cm = 0;
#pragma unroll
            for (int x = 0; x < WPT; ++x) {
                const uint32_t pw = s_cnt[WPT * dg + x];
                c[2 * x] = pw & 0xFFFFu;
                c[2 * x + 1] = pw >> 16;
            }
#pragma unroll
            for (int x = 0; x < 2 * WPT; ++x) {
                sum += c[x];
                cm = c[x] > cm ? c[x] : cm;
            }
            const uint32_t inc = wave_inclusive_sum(sum);
#pragma unroll
            for (int o = kWave / 2; o > 0; o >>= 1) {
                const uint32_t y = __shfl_xor(cm, o, kWave);
                cm = y > cm ? y : cm;
            }
            if (lane == kWave - 1) s_tmp[wave] = inc;
            if (lane == 0) s_cm[wave] = cm;
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int x = 0; x < WAVES; ++x) {
                off += (x < (int)wave) ? s_tmp[x] : 0u;
                big = s_cm[x] > big ? s_cm[x] : big;
            }
            uint32_t b = off + inc - sum;
#pragma unroll
            for (int x = 0; x < WPT; ++x) {
                const uint32_t b0 = b, b1 = b + c[2 * x];
                s_cnt[WPT * dg + x] = b0 | (b1 << 16);
                b = b1 + c[2 * x + 1];
            }
        }
        __syncthreads();
        probe.mark(2);
        if ((big >> 2) > kMaxSub) {   // uniform: clustered keys -> the measured-span kernel
            // (XQ: k_window_gather copies the retried windows to their SA
            // positions for it; storing the items here made this kernel spill)
            if (threadIdx.x == 0) retry[atomicAdd(&words[kRetryWord], 1u)] = j;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (XQ && CR) load_items_cr<ITEMS>(keys_in, rwn, w);
            else if constexpr (XQ) load_items_xq<ITEMS>(keys_in, rwn, hn.z, w);
            else load_items<ITEMS>(keys_in, hn.y, hn.z, w);
            __syncthreads();
        } else {
            // 2. scatter the 32-bit words into sub-buckets (any order inside
            // one); the indices stay by load slot
            auto scatter1 = [&](int i, uint32_t le) {
                const uint32_t y = (uint32_t)(w[i] >> dsh);
                const uint32_t old = atomicAdd(cnt_word(y), half_inc(y));
                const uint32_t at = __builtin_amdgcn_ubfe(old, y << 4, 16u);   // byte address in s_k
                *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_k) + at) =
                    (((uint32_t)(w[i] >> ib) & lmask) << kSlotBits) | le;
                s_x[le] = (uint32_t)(w[i] & imask);
            };
            if (sfull) {
                // claims in groups of SA_LS_CLAIMS (> 1: the atomics' round
                // trips overlap, at more live registers)
#pragma unroll
                for (int g = 0; g < ITEMS; g += SA_LS_CLAIMS) {
                    uint32_t y[SA_LS_CLAIMS], old[SA_LS_CLAIMS];
#pragma unroll
                    for (int t = 0; t < SA_LS_CLAIMS; ++t) {
                        y[t] = (uint32_t)(w[g + t] >> dsh);
                        old[t] = atomicAdd(cnt_word(y[t]), half_inc(y[t]));
                    }
#pragma unroll
                    for (int t = 0; t < SA_LS_CLAIMS; ++t) {
                        const int i = g + t;
                        const uint32_t le = l0 + i * kWave;
                        const uint32_t at = __builtin_amdgcn_ubfe(old[t], y[t] << 4, 16u);
                        *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_k) + at) =
                            (((uint32_t)(w[i] >> ib) & lmask) << kSlotBits) | le;
                        s_x[le] = (uint32_t)(w[i] & imask);
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < ITEMS; ++i) {
                    const uint32_t le = l0 + i * kWave;
                    if (slot_ok(i)) scatter1(i, le);
                }
            }
            // ... the window is in LDS: the next window's loads go out now (a
            // scheduling barrier: hoisted above the scatter, they would hold
            // a second window of registers)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (XQ && CR) load_items_cr<ITEMS>(keys_in, rwn, w);
            else if constexpr (XQ) load_items_xq<ITEMS>(keys_in, rwn, hn.z, w);
            else load_items<ITEMS>(keys_in, hn.y, hn.z, w);
            __syncthreads();
            probe.mark(3);
            // ... then each thread sorts its four consecutive sub-buckets,
            // largest first, with 4 / 8 / 12 / 16-input networks by the
            // wave's largest sub-bucket of this rank (larger: insertion)
            uint32_t nu = 0, ng = 0;
            uint32_t umask = 0;   // bit k: sub-bucket sb0 + k holds a group
            const uint32_t sb0 = 2 * WPT * dg;
            uint32_t order = 0;
            {
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t sb = sb0 + k;
                    o[k] = ((end_of(sb) - (sb ? end_of(sb - 1) : 0u)) << 2) | (uint32_t)k;
                }
                sort_net32<4>(o);
#pragma unroll
                for (int k = 0; k < 4; ++k) order |= (o[3 - k] & 3u) << (2 * k);
            }
#pragma unroll 1
            for (uint32_t i = 0; i < 4; ++i) {
                const uint32_t sb = sb0 + ((order >> (2 * i)) & 3u);
                const uint32_t lo = sb ? end_of(sb - 1) : 0u, hi = end_of(sb), cnt = hi - lo;
                const bool wide4 = __ballot(cnt > 4u) != 0ull, wide8 = __ballot(cnt > 8u) != 0ull,
                           wide12 = __ballot(cnt > 12u) != 0ull;   // uniform
                if (cnt == 0) continue;
                const uint32_t nu0 = nu;
                // (LSV & 2 with key samples: words written back, the samples read them)
                constexpr int LW = LSV & 1;
                bool grp;
                if ((LSV & 2) && !so.samples) {
                    if (!wide4) grp = sort_sub_words<4, LSV>(s_k, s_x, lo, cnt, nu, ng);
                    else if (!wide8) grp = sort_sub_words<8, LSV>(s_k, s_x, lo, cnt, nu, ng);
                    else if (!wide12) grp = sort_sub_words<12, LSV>(s_k, s_x, lo, cnt, nu, ng);
                    else if (cnt <= (uint32_t)kNet) grp = sort_sub_words<kNet, LSV>(s_k, s_x, lo, cnt, nu, ng);
                    else {
                        sort_sub_words_lds(s_k, lo, hi, nu, ng);
                        grp = true;   // the U walk converts its words (with or without groups)
                    }
                } else {
                    if (!wide4) sort_sub_words<4, LW>(s_k, s_x, lo, cnt, nu, ng);
                    else if (!wide8) sort_sub_words<8, LW>(s_k, s_x, lo, cnt, nu, ng);
                    else if (!wide12) sort_sub_words<12, LW>(s_k, s_x, lo, cnt, nu, ng);
                    else if (cnt <= (uint32_t)kNet) sort_sub_words<kNet, LW>(s_k, s_x, lo, cnt, nu, ng);
                    else sort_sub_words_lds(s_k, lo, hi, nu, ng);
                    grp = nu != nu0;
                }
                if (grp) umask |= 1u << (sb - sb0);
                // the sorted key1 of this sub-bucket's every-2^ksh-th SA
                // positions, from the sorted words (a global load here would
                // make the store phase wait for the next window's loads)
                // (sa_search.h for_each_sample: exact up to a + hi = 2^32)
                if (so.samples)
                    for_each_sample(a, lo, hi, so.ksh, [&](uint32_t q) {
                        keys_out[(a + q) >> so.ksh] = mn + (((uint64_t)sb << low_bits) | (s_k[q] >> kSlotBits));
                    });
            }
            probe.mark(4);
            // 3. U / U-group offsets (one scan of both; heads = m - U + G)
            uint32_t bu, bg, tu_w, tg_w;
            {
                const uint32_t iug = wave_inclusive_sum(nu | (ng << 16));
                if (lane == kWave - 1) s_ug[wave] = iug;
                __syncthreads();
                uint32_t oug = 0, tug = 0;
#pragma unroll
                for (int x = 0; x < WAVES; ++x) {
                    const uint32_t xug = s_ug[x];
                    oug += (x < (int)wave) ? xug : 0u;
                    tug += xug;
                }
                tu_w = tug & 0xFFFFu;
                tg_w = tug >> 16;
                bu = (oug & 0xFFFFu) + (iug & 0xFFFFu) - nu;
                bg = (oug >> 16) + (iug >> 16) - ng;
            }
            // LSV bit 1 (no key samples): s_k holds suffix indices except in
            // the sub-buckets with groups, which the U walk converts
            const bool idx_back = (LSV & 2) && !so.samples;   // uniform
            if (so.rank && threadIdx.x == 0) {
                so.cnt_u[j] = tu_w;
                so.cnt_g[j] = tg_w;
                s_tot[0] += m - tu_w + tg_w;
                s_tot[1] += tu_w;
                s_tot[2] += tg_w;
            }
            // the unsorted members of this thread's sub-buckets (rare)
            if (umask && (so.rank || idx_back)) {
                uint32_t ku = bu, kg = bg;
                for (uint32_t um = umask; um; um &= um - 1u) {
                    const uint32_t sb = sb0 + (uint32_t)__builtin_ctz(um);
                    const uint32_t lo = sb ? end_of(sb - 1) : 0u, hi = end_of(sb);
                    uint32_t head = lo, pr = ~0u;
                    for (uint32_t k = lo; k < hi; ++k) {
                        const uint32_t v = s_k[k], r = v >> kSlotBits;
                        const uint32_t nx = k + 1 < hi ? (s_k[k + 1] >> kSlotBits) : ~0u;
                        const bool eqp = k > lo && pr == r, eqn = k + 1 < hi && nx == r;
                        const uint32_t xi = s_x[v & kSlotMask];
                        if (idx_back) s_k[k] = xi;   // (s_k[k + 1] already read)
                        if (!eqp) head = k;
                        if (!eqp && eqn) ++kg;
                        if (so.rank && (eqp || eqn)) {
                            const uint32_t rv = (uint32_t)(so.rank_off + a + head + 1u);
                            if (so.tmp_rank) so.tmp_rank[a + ku] = rv;
                            else so.rank[xi] = rv;
                            atomicOr(&so.member[xi >> 5], 1u << (xi & 31));
                            so.tmp_pos[a + ku] = (uint32_t)(a + k);
                            so.tmp_idx[a + ku] = xi;
                            so.tmp_g[a + ku] = kg - 1u;
                            ++ku;
                        }
                        pr = r;
                    }
                }
            }
            probe.mark(5);
            // 4. the SA, coalesced: the index of each sorted word's load slot
            // (the U / G scan's barrier follows every thread's sort; with
            // idx_back one more waits for the U walk's conversions)
            if (idx_back) {
                __syncthreads();
                if (wfull) {
#pragma unroll 2
                    for (int i = 0; i < ITEMS; ++i) {
                        const uint32_t le = l0 + i * kWave;
                        sa_out[a + le] = s_k[le];
                    }
                } else {
#pragma unroll 2
                    for (int i = 0; i < ITEMS; ++i) {
                        const uint32_t le = l0 + i * kWave;
                        if (le < m) sa_out[a + le] = s_k[le];
                    }
                }
            } else if (wfull) {
#pragma unroll 2
                for (int i = 0; i < ITEMS; ++i) {
                    const uint32_t le = l0 + i * kWave;
                    sa_out[a + le] = s_x[s_k[le] & kSlotMask];
                }
            } else {
#pragma unroll 2
                for (int i = 0; i < ITEMS; ++i) {
                    const uint32_t le = l0 + i * kWave;
                    if (le < m) sa_out[a + le] = s_x[s_k[le] & kSlotMask];
                }
            }
            __syncthreads();   // s_k / s_x / s_cnt reuse by the next window
            probe.mark(6);
        }
        if (!more) break;
        q = qn;
        h = hn;
        if constexpr (XQ && CR) {
            rv[0] = rwn[0];
            rv[1] = rwn[1];
        }
        par ^= 1u;
    }
    probe.flush(words);
    __syncthreads();
    flush_totals(words, s_tot[0], s_tot[1], s_tot[2]);
}

// The skewed windows: stable LSD passes of 8 bits over the key span, each an
// in-wave ranking (match-any from 8 ballots, wave-major input order), per-
// digit wave prefixes, digit offsets, scatter into LDS, read back in order.
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_bucket_sort_lsd(const uint64_t* __restrict__ keys_in, BucketRel br,
                                                           const uint32_t* __restrict__ ws,
                                                           const uint32_t* __restrict__ skew,
                                                           uint32_t* __restrict__ words, uint32_t ib,
                                                           uint64_t* __restrict__ keys_out,
                                                           uint32_t* __restrict__ sa_out, SegOut so) {
    constexpr int WAVES = BLOCK / kWave;
    constexpr int CAP = BLOCK * ITEMS;
    constexpr int WT = kWave * ITEMS;
    static_assert(BLOCK >= kRadix, "one thread per digit");
    static_assert(CAP <= 65535, "16-bit LDS offsets");
    __shared__ uint64_t s_w[CAP];
    __shared__ uint16_t s_wcnt[WAVES][kRadix];
    __shared__ uint16_t s_start[kRadix];
    __shared__ uint32_t s_tmp[kWaves];
    __shared__ uint64_t s_red[2][WAVES];
    __shared__ uint32_t s_bk[2][32];

    const uint32_t wave = wave_id(), lane = lane_id();
    const uint32_t dg = threadIdx.x;
    uint32_t* err = words + 6;
    const uint32_t nskew = words[10];
    static_assert(WAVES * ITEMS * 8 <= WAVES * kRadix * 2, "per-row segment values fit in s_wcnt");
    uint64_t th = 0, tu = 0, tg = 0;
    for (uint32_t q = blockIdx.x; q < nskew; q += gridDim.x) {
        const uint32_t j = skew[q];
        const uint64_t a = ws[j];
        const uint32_t m = (uint32_t)(ws[j + 1] - a);
        uint64_t w[ITEMS];
        uint64_t mn;
        uint32_t bits;
        if (!load_window<BLOCK, ITEMS>(keys_in, br, j, a, m, ib, w, mn, bits, s_red, s_bk, err)) {
            __syncthreads();
            continue;
        }
        const uint32_t passes = (bits + 7) / 8;
        for (uint32_t p = 0; p < passes; ++p) {
            const uint32_t sh = ib + 8 * p;
            for (int i = threadIdx.x; i < WAVES * kRadix; i += BLOCK) (&s_wcnt[0][0])[i] = 0;
            __syncthreads();
            uint32_t r[ITEMS];
            uint16_t* wc = s_wcnt[wave];
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const uint32_t le = wave * WT + i * kWave + lane;
                const bool ok = le < m;
                const uint32_t d = ok ? (uint32_t)(w[i] >> sh) & 0xFFu : (uint32_t)kRadix;
                uint64_t peers = __ballot(ok);
#pragma unroll
                for (uint32_t bt = 0; bt < 8; ++bt) {
                    const bool bit = (d >> bt) & 1u;
                    const uint64_t bal = __ballot(bit);
                    peers &= bit ? bal : ~bal;
                }
                uint32_t cnt = 0;
                if (ok) cnt = wc[d];
                const uint32_t below = (uint32_t)__popcll(peers & lanemask_lt());
                r[i] = cnt + below;
                if (ok && below == 0) wc[d] = (uint16_t)(cnt + (uint32_t)__popcll(peers));
            }
            __syncthreads();
            uint32_t tot = 0;
            if (dg < (uint32_t)kRadix) {
#pragma unroll
                for (int x = 0; x < WAVES; ++x) {
                    const uint32_t y = s_wcnt[x][dg];
                    s_wcnt[x][dg] = (uint16_t)tot;
                    tot += y;
                }
            }
            {
                const uint32_t x = (dg < (uint32_t)kRadix) ? tot : 0u;
                const uint32_t inc = wave_inclusive_sum(x);
                if (lane == kWave - 1 && wave < (uint32_t)kWaves) s_tmp[wave] = inc;
                __syncthreads();
                uint32_t off = 0;
#pragma unroll
                for (int x2 = 0; x2 < kWaves; ++x2) off += (x2 < (int)wave) ? s_tmp[x2] : 0u;
                if (dg < (uint32_t)kRadix) s_start[dg] = (uint16_t)(off + inc - x);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                if (wave * WT + i * kWave + lane < m) {
                    const uint32_t d = (uint32_t)(w[i] >> sh) & 0xFFu;
                    s_w[s_start[d] + s_wcnt[wave][d] + r[i]] = w[i];
                }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const uint32_t le = wave * WT + i * kWave + lane;
                if (le < m) w[i] = s_w[le];
            }
            __syncthreads();
        }
        if (passes == 0) {   // one key: input order
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const uint32_t le = wave * WT + i * kWave + lane;
                if (le < m) s_w[le] = w[i];
            }
            __syncthreads();
        }
        if (so.rank)
            window_segments<BLOCK, ITEMS>(s_w, reinterpret_cast<uint64_t*>(&s_wcnt[0][0]), s_red, a, m, ib, j, so, th,
                                          tu, tg);
        store_window<BLOCK, ITEMS>(s_w, a, m, ib, mn, keys_out, sa_out, so.ksh);
        __syncthreads();
    }
    flush_totals(words, th, tu, tg);
}

}  // namespace sa
