// sa_round1.h -- host side of the bucketed first round (kernels: sa_bucket.h).
// Included by sa_build.hip inside namespace sa, after the radix helpers.
//
// plan_bucketed() decides whether the text's alphabet and size allow the
// key1 layout; round1_bucketed() runs pack -> 2 bucket passes -> window
// starts -> local sort and leaves the sorted key1 in keys[0] and the SA in
// d_sa.  When a window exceeds the LDS tile (skewed text: a long run, a short
// period) or its key span is too wide, it reports !done and the caller runs
// the full LSD sort of the packed K-symbol key instead.
#pragma once

// Launch shapes, overridable at build time for A/B runs
// (scripts/ab_build_variants.sh).  Bucket histogram workgroups per CU: 4 ->
// 64 took it from 0.62 to 0.47 ms at 2^30 (more waves in flight per CU).
#ifndef SA_HIST_WPC
#define SA_HIST_WPC 64
#endif
// range builds: records in one striped scan of the text (k_bucket_hist<.., 3>)
#ifndef SA_REC_STRIPED
#define SA_REC_STRIPED 1
#endif
// Extra bucket bits over the size-based default (+1 at 2^30: windows of
// ~4 K suffixes, local sort 7.3 -> 11.3 ms, second pass 5.9 -> 7.1 ms).
#ifndef SA_BB_EXTRA
#define SA_BB_EXTRA 0
#endif
// positions / pairs per lane of the two bucket passes (tile = 1024 x items)
#ifndef SA_ITEMS_A
#define SA_ITEMS_A 12
#endif
#ifndef SA_TEXT_BLOCK
#define SA_TEXT_BLOCK 512
#endif
#ifndef SA_LIST_BLOCK
#define SA_LIST_BLOCK 1024
#endif


#ifndef SA_SEG_BLOCK
#define SA_SEG_BLOCK 1024
#endif
// second bucket pass by per-XCD queues and regions (sa_split.h SegXq)
#ifndef SA_SEG_XQ
#define SA_SEG_XQ 1
#endif
#ifndef SA_ITEMS_B
#define SA_ITEMS_B 10
#endif
// pairs per lane of the second pass over packed items (SrcPk8: no spills;
// 8 / 10 / 12: 5.50 / 5.17 / 4.90 ms at 2^30 DNA, profiles/r02_ai_ab_pk8.txt)
#ifndef SA_ITEMS_PK
#define SA_ITEMS_PK 12
#endif
// the sorted key1 of every 2^kKeySample-th SA position is kept for the rank
// look-ups of later rounds (lower_bound_sampled)
#ifndef SA_KEY_SAMPLE
#define SA_KEY_SAMPLE 4
#endif
constexpr uint32_t kKeySample = SA_KEY_SAMPLE;
#ifndef SA_LAZY_SAMPLES
#define SA_LAZY_SAMPLES 1
#endif
// padded first-pass segments (k_bucket_sample) from 2^26 suffixes up to the
// bucketed round's one-GPU maximum; their starts live in the onesweep base
// scratch after the second pass's 2^hb (<= 1024) digit bases
constexpr uint64_t kPadMinN = 1ull << 26;
// the fixed-span local sort's variant (k_bucket_sort LSV; sa_opts.tune bits
// 16-19 + 1 select one for A/B runs, 0 = the default)
#ifndef SA_LS_VARIANT
#define SA_LS_VARIANT 0
#endif
static int ls_variant(const sa_context* c) {
    const uint32_t t = ((uint32_t)c->tune >> 16) & 0xFu;
    return t ? (int)(t - 1u) : SA_LS_VARIANT;
}

// first-pass cursor stripes with padded segments (sa_opts.tune bits 8-15
// override: 1 = one cursor per digit shared by every tile, ticketed tiles)
static uint32_t text_stripes(const sa_context* c) {
    const uint32_t e = ((uint32_t)c->tune >> 8) & 0xFFu;
    const uint32_t v = e ? e : 8u;
    return v >= 8 ? 8u : v >= 4 ? 4u : v >= 2 ? 2u : 1u;
}

// out[d] = sum of rows r < rows of in[r][d] (kLoRadix columns)
__global__ __launch_bounds__(kLoRadix) void k_sum_rows(const uint32_t* __restrict__ in, uint32_t rows,
                                                       uint32_t* __restrict__ out) {
    uint32_t t = 0;
    for (uint32_t r = 0; r < rows; ++r) t += in[r * kLoRadix + threadIdx.x];
    out[threadIdx.x] = t;
}
constexpr uint64_t kPadMaxN = 1ull << 31;
constexpr uint32_t kPadStartOff = kLoRadix + 1024;                 // kLoRadix + 1 words
constexpr uint32_t kPadDenseOff = kPadStartOff + kLoRadix + 64;    // kLoRadix words

struct BucketPlan {
    BucketSpec bs{};
    uint32_t ib = 0;   // bit width of n - 1 (index bits packed under the key in the local sort)
    uint32_t K = 0;    // s + R: symbols the first round sorts by
};

// round1: SA_ROUND1_AUTO / SA_ROUND1_LSD / SA_ROUND1_BUCKETED (sa_opts.round1)
// world: GPUs the bucket range is split over (sa_dist.h); one GPU sorts at
// most 2^18 buckets (the second pass's 10 digit bits), a rank of a wider
// build 2^bb / world of them.
// cmp: the compact low of BucketSpec (only when short_suffix_ties is false
// for the text)
static bool plan_bucketed(uint32_t sigma, uint64_t n, uint32_t K, int round1, int radix, BucketPlan* p,
                          int world = 1, int cmp = 0) {
    if (round1 == SA_ROUND1_LSD || radix != 0 || sigma < 2 || n < 2) return false;
    if (round1 == SA_ROUND1_AUTO && n < kBucketMinN) return false;
    // bucket bits: windows of about n / 2^bb suffixes must fit the
    // 9216-suffix LDS tile with room for random fluctuation (16 up to 2^29
    // suffixes, 17 up to 2^30, 18 up to 2^31, 19 up to 2^32)
    uint32_t bb = std::max<uint32_t>(16u, bit_width(n - 1) > 13 ? bit_width(n - 1) - 13 : 0u);
    if (world <= 1) bb = std::min<uint32_t>(bb, 18u);
    bb += SA_BB_EXTRA;
    if (bb > 18 + (uint32_t)bit_width((uint64_t)std::max(world, 1) - 1) || bb > 24) return false;
    uint64_t ps = 1;   // sigma^s >= 2^bb: the bb-bit bucket is dense
    uint32_t s = 0;
    while (ps < (1ull << bb)) {
        ps *= sigma;
        ++s;
    }
    // sigma^s a multiple of 2^bb (sigma a power of two): every bucket is an
    // equal range of D values.  Otherwise buckets hold floor or ceil of
    // sigma^s / 2^bb values -- up to 2x apart when the ratio is ~1 (alnum:
    // 9472-suffix windows at 2^30, over the LDS tile) -- so s grows until the
    // ratio is >= 64 (sizes within 1/64) while D stays below 2^32 (it rolls
    // in 32 bits)
    while (ps % (1ull << bb) != 0 && ps < (64ull << bb) && s + 1 < K && ps * sigma <= (1ull << 32)) {
        ps *= sigma;
        ++s;
    }
    if (ps > (1ull << 32)) return false;
    if (K <= s || K > (uint32_t)kMaxK) return false;
    const uint32_t ib = bit_width(n - 1);
    const uint32_t bd = bit_width(ps - 1);
    // D values per bucket, +1 bit for a window holding two buckets
    const uint32_t span = bit_width((ps + (1ull << bb) - 1) >> bb) + 1;
    for (uint32_t R = K - s; R >= 1; --R) {
        unsigned __int128 pr = 1;   // sigma^R
        for (uint32_t t = 0; t < R; ++t) pr *= sigma;
        unsigned __int128 lowmax = cmp == 2 ? pr - 1 : cmp ? 2 * pr - 1 : s + (pr - 1) * (R + 1) + R;
        uint32_t rb = 0;
        while (lowmax) {
            ++rb;
            lowmax >>= 1;
        }
        if (bd + rb > 64 || rb + span + ib > 64) continue;
        p->bs.pow_s1 = ps / sigma;
        p->bs.powR1 = (uint64_t)(pr / sigma);
        p->bs.cmul = (1ull << 48) / ps;   // bucket = (D * cmul) >> (48 - bb) < 2^bb
        p->bs.bb = bb;
        p->bs.bsh = 48u - bb;
        p->bs.sigma = sigma;
        p->bs.s = s;
        p->bs.R = R;
        p->bs.rb = rb;
        p->bs.cmp = (uint32_t)cmp;
        p->ib = ib;
        p->K = s + R;
        return true;
    }
    return false;
}

// The compact layout's precondition fails: two of the text's last K - 1
// suffixes share (D, r) with digit 0 past the end (the text ends in a run of
// its smallest symbol, e.g. ...AA for DNA: "A" and "AA" pad alike).  tail:
// the text's last t = min(n, kMaxK) >= K - 1 bytes; code: dense codes.
// last: how many of the last suffixes must differ (K - 1 for the compact
// layout, K for the E-only one); t >= last.
static bool short_suffix_ties(const uint8_t* tail, uint64_t n, uint32_t t, const uint16_t* code, uint32_t sigma,
                              uint32_t s, uint32_t R, uint32_t last = 0) {
    auto dig = [&](uint8_t x) -> uint32_t { return code[x] ? code[x] - 1u : 0u; };
    const uint32_t K = s + R;
    if (last == 0) last = K - 1;
    uint64_t Ds[kMaxK + 1];
    unsigned __int128 rs[kMaxK + 1];
    uint32_t cnt = 0;
    for (uint32_t L = 1; L <= last && L <= n && L <= t; ++L) {
        const uint8_t* x = tail + (t - L);
        uint64_t D = 0;
        unsigned __int128 r = 0;
        for (uint32_t q = 0; q < s; ++q) D = D * sigma + (q < L ? dig(x[q]) : 0u);
        for (uint32_t q = s; q < K; ++q) r = r * sigma + (q < L ? dig(x[q]) : 0u);
        for (uint32_t o = 0; o < cnt; ++o)
            if (Ds[o] == D && rs[o] == r) return true;
        Ds[cnt] = D;
        rs[cnt] = r;
        ++cnt;
    }
    return false;
}

// The first bucket pass may write one packed 64-bit item per suffix
// (k_split_text / k_split_list <.., PK8>, SrcPk8): a power-of-two alphabet,
// and the second pass's digit (of the local bucket), key1 below its bucket and
// the index fitting 64 bits
// np2 (one GPU): a non-power-of-two alphabet too -- key1 below its bucket =
// key1 - (Dmin(b) << rb) < (D values per bucket) 2^rb, D - Dmin(b) from the
// bucket's fraction of D cmul (k_split_text); the buckets of (D cmul) >> bsh hold at most
// ceil(sigma^s / 2^bb) + 1 values of D
static bool plan_pk8(const BucketPlan& bp, uint32_t hb, uint32_t dbg, bool np2 = false) {
    const uint32_t sg = bp.bs.sigma;
    if (sg < 2 || (dbg & SA_DEBUG_NO_PK8)) return false;
    if ((sg & (sg - 1)) != 0) {
        if (!np2) return false;
        const uint64_t ps = bp.bs.pow_s1 * sg;
        const uint64_t per = ((ps + (1ull << bp.bs.bb) - 1) >> bp.bs.bb) + 1;
        return hb + bit_width(per - 1) + bp.bs.rb + bp.ib <= 64;
    }
    const uint32_t lg = (uint32_t)__builtin_ctz(sg);
    if (lg * bp.bs.s < bp.bs.bb) return false;
    return hb + (lg * bp.bs.s - bp.bs.bb) + bp.bs.rb + bp.ib <= 64;
}

// The buckets [blo, bhi) this build sorts (local bucket = bucket - blo): all
// of them on one GPU; one rank's contiguous range in the range-partitioned
// build (sa_dist.h), whose m suffixes occupy SA positions [sa_off, sa_off + m)
// -- the SA, sorted keys and bucket starts written here are that range's,
// the ranks of unsorted suffixes global (rank_off).
struct BucketRange {
    uint32_t blo = 0, bhi = 0;
    uint64_t m = 0;
    uint64_t sa_off = 0;
    bool always_u = false;      // compact the unsorted set whatever its size
    uint32_t* rank = nullptr;   // n-entry rank array / n-bit member map of the
    uint32_t* member = nullptr; // unsorted set (null: the context's)
    // compact rank map (RankMap; the range-partitioned build): rank holds the
    // members' ranks in text order, prefix ((n + 31) / 32 words + the scan's
    // per-block sums) the member bitmap's exclusive popcount scan; tmp_rank
    // (m words) stages the ranks until the bitmap is complete
    uint32_t* prefix = nullptr;
    uint32_t* tmp_rank = nullptr;
};

static BucketRange full_range(const BucketPlan& bp, uint64_t n) {
    BucketRange r;
    r.blo = 0;
    r.bhi = 1u << bp.bs.bb;
    r.m = n;
    return r;
}

// second-pass digit bits for a range of nb local buckets (7..10)
static uint32_t range_hb(uint32_t nb) {
    const uint32_t w = bit_width(nb > 1 ? nb - 1 : 1);
    return std::max<uint32_t>(7u, w > kLoBits ? w - kLoBits : 0u);
}

// *done: the SA and keys[0] hold the sorted first round (keys[0]: the key1
// of every 2^*ksh-th SA position when *fused, else every key1).  *fused: the
// round-1 segments were produced with it (few unsorted suffixes): rank[] for
// the unsorted set only (member bitmap), the unsorted set compacted in
// u_pos/u_idx/u_g[0], and seg = {D, m, G}; otherwise the caller runs
// segments() on keys[0].
static int round1_bucketed(sa_context* c, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, const BucketPlan& bp,
                           const BucketRange& br_, hipStream_t s, Timer& tm, sa_stats* st, bool* done, bool* fused,
                           uint64_t seg[3], uint32_t* ksh, bool allow_pad = true, bool allow_xq = true) {
    *done = false;
    *fused = false;
    *ksh = 0;
    const uint64_t m = br_.m;   // suffixes of this range (= n on one GPU)
    const uint32_t blo = br_.blo, bhi = br_.bhi;
    if (bhi <= blo || bhi - blo > (1u << 18)) return set_err(SA_E_INTERNAL, "bucket range [%u, %u)", blo, bhi);
    int rc = onesweep_prepare(c, s);
    if (rc) return rc;
    // [0..2] D, m, G of the fused segments, [5] largest window, [6] local-sort
    // flags, [7] windows, [10] skewed windows
    SA_HIP(hipMemsetAsync(c->words, 0, 12, s));
    SA_HIP(hipMemsetAsync(c->words + 5, 0, 28, s));   // [5, 11]
    // digit totals of both bucket passes (one read of the text)
    // a rank's range of a multi-GPU build holding at most ~a quarter of the
    // text: the histogram pass counts the range's suffixes per workgroup, a
    // second launch over the same tiles emits their (key1, position) records
    // and the first pass scatters those (scripts/sim_ranks.py at 2^30 DNA,
    // G = 8: per-rank round 1 5.0 -> 4.0 ms against k_split_text filtering the
    // whole text; at G = 2 streaming the text through k_split_text is cheaper
    // than writing and reading 12-byte records for half of it)
    // (the first pass straight from the text through an LDS record buffer,
    // no records in HBM, was slower: G = 8 DNA 3.67 vs 3.29 ms per rank,
    // profiles/r04_f_ab_range_fused.txt)
    const bool listed = m * 10 <= n * 3;   // G >= 4: every rank's ~n/G (balanced cuts are within a few %)
    uint64_t* const lkeys = c->keys_u;   // m records (free until the second pass writes keys_u)
    uint32_t* const lpos = c->vals_u;    // (free until the later rounds)
    // striped records (k_bucket_hist<.., LM = 3>): one scan of the text
    // writes the records into kRecStripes regions of rcap, each tile's place
    // claimed from its stripe's cursor, instead of a counting scan + an
    // exclusive scan + a record scan; a stripe that overflows (a text whose
    // kept suffixes cluster on every kRecStripes-th tile) re-runs the round
    // with the counting scan.  SA_DEBUG_PAD_OVERFLOW: regions of half the
    // expected share (tests).
    const uint64_t rtiles = (n + kTile - 1) / kTile;
    const uint32_t rgrid = (uint32_t)(std::min<uint64_t>(rtiles, (uint64_t)SA_HIST_WPC * (uint32_t)c->cus) /
                                      kRecStripes * kRecStripes);
    const uint64_t rcap64 = (c->dbg & SA_DEBUG_PAD_OVERFLOW) ? m / kRecStripes / 2 + 1
                                                             : (m + m / 8) / kRecStripes + 2 * (uint64_t)kTile;
    const bool striped = SA_REC_STRIPED && listed && allow_pad && !(c->dbg & SA_DEBUG_NO_PAD) &&
                         rtiles >= 4ull * kRecStripes && rgrid >= kRecStripes && kRecStripes * rcap64 <= c->ucap;
    const uint32_t rcap = (uint32_t)std::min<uint64_t>(rcap64, UINT32_MAX);
    uint32_t* const rcur = c->hist;   // the stripes' cursors (the chunk histograms are free here)
    // (the regions live in keys_u / vals_u: ucap entries, rec_capacity(m) in range builds)
    // one GPU, the whole bucket range: padded first-pass segments sized from a
    // sample instead of the exact totals (k_bucket_sample, sa_bucket.h)
    const bool padded = allow_pad && !listed && blo == 0 && bhi == (1u << bp.bs.bb) && n >= kPadMinN &&
                        n <= kPadMaxN && c->cap_pad >= pad_capacity(n) && !(c->dbg & SA_DEBUG_NO_PAD);
    const uint32_t ssh = std::max<uint32_t>(6u, bit_width(n) > 21 ? bit_width(n) - 21 : 0u);
    uint32_t* const pstart = os_base(c) + kPadStartOff;   // kLoRadix + 1 padded segment starts
    uint32_t* const dlo = os_base(c) + kPadDenseOff;      // kLoRadix dense segment starts
    if (st) st->round1_segments = padded ? 1 : striped ? 3 : 0;
    tm.begin(SA_K_PACK);
    if (padded) {
        const bool pow2 = (bp.bs.sigma & (bp.bs.sigma - 1)) == 0;
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(((n >> ssh) + kBlock - 1) / kBlock,
                                                                               4u * (uint32_t)c->cus));
        if (pow2)
            hipLaunchKernelGGL(k_bucket_sample<true>, dim3(g), dim3(kBlock), 0, s, d_text, n,
                               (const uint16_t*)c->code, bp.bs, ssh, os_ghist(c));
        else
            hipLaunchKernelGGL(k_bucket_sample<false>, dim3(g), dim3(kBlock), 0, s, d_text, n,
                               (const uint16_t*)c->code, bp.bs, ssh, os_ghist(c));
        // SA_DEBUG_PAD_OVERFLOW (tests): segments of exactly the sampled
        // estimate, so the first pass overflows and the round re-runs exactly
        hipLaunchKernelGGL(k_pad_starts, dim3(1), dim3(kLoRadix), 0, s, (const uint32_t*)os_ghist(c), ssh,
                           (c->dbg & SA_DEBUG_PAD_OVERFLOW) ? 1u : 0u, (uint32_t)c->cap_pad, pstart);
    } else {
        const uint64_t tiles = (n + kTile - 1) / kTile;
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles, (uint64_t)SA_HIST_WPC * (uint32_t)c->cus));
        const bool pow2 = (bp.bs.sigma & (bp.bs.sigma - 1)) == 0;
        uint32_t* const wgcnt = c->hist;       // per-workgroup kept counts, then offsets (the
        uint32_t* const wgoff = c->hist + g;   // chunk histograms are free in the bucketed round)
#define SA_HIST_G(G, P, L, W)                                                                                 \
    hipLaunchKernelGGL((k_bucket_hist<P, false, L>), dim3(G), dim3(kBlock), 0, s, d_text, n,                  \
                       (const uint16_t*)c->code, bp.bs, os_ghist(c), 0ull, n, blo, bhi, lkeys, lpos, W, rcap,  \
                       c->words + 11)
#define SA_HIST_ID_G(G, L, W)                                                                                 \
    hipLaunchKernelGGL((k_bucket_hist<true, false, L, true>), dim3(G), dim3(kBlock), 0, s, d_text, n,         \
                       (const uint16_t*)c->code, bp.bs, os_ghist(c), 0ull, n, blo, bhi, lkeys, lpos, W, rcap,  \
                       c->words + 11)
#define SA_HIST(P, L, W) SA_HIST_G(g, P, L, W)
#define SA_HIST_ID(L, W) SA_HIST_ID_G(g, L, W)
        const bool ident = bp.bs.sigma == 256;
        // (the records in one pass with offsets by a decoupled look-back over
        // the 4096-position tiles was 2.3x slower: the chain over 2^18 - 2^20
        // tiles serialises, profiles/r04_q_ab_range_lookback.txt)
        if (striped) {
            SA_HIP(hipMemsetAsync(rcur, 0, kRecStripes * kRecCurStride * 4, s));
            if (ident) SA_HIST_ID_G(rgrid, 3, rcur);
            else if (pow2 && SA_DNA_SWAR && c->dna)
                hipLaunchKernelGGL((k_bucket_hist<true, false, 3, false, true>), dim3(rgrid), dim3(kBlock), 0, s, d_text,
                                   n, (const uint16_t*)c->code, bp.bs, os_ghist(c), 0ull, n, blo, bhi, lkeys, lpos, rcur,
                                   rcap, c->words + 11);
            else if (pow2) SA_HIST_G(rgrid, true, 3, rcur);
            else SA_HIST_G(rgrid, false, 3, rcur);
            // an overflowed stripe dropped records: stop before any pass reads them
            SA_HIP(hipMemcpyAsync(c->host_words + 11, c->words + 11, 4, hipMemcpyDeviceToHost, s));
            SA_HIP(host_sync(s));
            if (c->host_words[11]) {
                SA_TRACE("  bucketed round 1: a record stripe overflowed, again with the counting scan");
                tm.end();
                const int rc = round1_bucketed(c, d_text, n, d_sa, bp, br_, s, tm, st, done, fused, seg, ksh, false,
                                               allow_xq);
                if (st) st->round1_segments = 4;
                return rc;
            }
        } else if (ident && listed) SA_HIST_ID(1, wgcnt);
        else if (pow2 && listed) SA_HIST(true, 1, wgcnt);
        else if (pow2) SA_HIST(true, 0, wgcnt);
        else if (listed) SA_HIST(false, 1, wgcnt);
        else SA_HIST(false, 0, wgcnt);
        if (listed && !striped) {
            hipLaunchKernelGGL(k_exscan_u32, dim3(1), dim3(kBlock), 0, s, (const uint32_t*)wgcnt, wgoff, g);
            if (ident) SA_HIST_ID(2, wgoff);
            else if (pow2) SA_HIST(true, 2, wgoff);
            else SA_HIST(false, 2, wgoff);
        }
#undef SA_HIST
#undef SA_HIST_ID
#undef SA_HIST_G
#undef SA_HIST_ID_G
    }
    tm.end();
    add_bytes(st, SA_K_PACK, padded ? (n >> ssh) * 64 : n + (striped ? 12 * m : listed ? n + 12 * m : 0));
    // second-pass digit bits (7..10): bb - kLoBits on one GPU
    const uint32_t hb = (blo == 0 && bhi == (1u << bp.bs.bb)) ? bp.bs.bb - kLoBits : range_hb(bhi - blo);
    if (hb < 7 || hb > 10) return set_err(SA_E_INTERNAL, "second bucket pass of %u bits", hb);
    const uint32_t nb_tab = 1u << (hb + kLoBits);   // local buckets in the start table
    const bool np2 = (bp.bs.sigma & (bp.bs.sigma - 1)) != 0;
    const bool pk8 = plan_pk8(bp, hb, c->dbg, !br_.always_u);   // (non-power-of-two alphabets: one GPU)
    // the local sort's key span: a one-bucket window's keys fill bits1 bits
    // (compact layout); 0 = measured per window
    uint32_t bits1 = 0;
    if (bp.bs.cmp) {
        const uint64_t ps = bp.bs.pow_s1 * bp.bs.sigma, per = (ps + (1ull << bp.bs.bb) - 1) >> bp.bs.bb;
        // (a power-of-two alphabet's buckets hold exactly per values of D;
        // (D cmul) >> bsh buckets up to per + 1, so key1 - Dmin(b) << rb
        // reaches per << rb)
        const bool exact = (ps & ((1ull << bp.bs.bb) - 1)) == 0;
        bits1 = bit_width(exact ? per - 1 : per) + bp.bs.rb;
        // tests: a span wider than the keys' (they cluster in the low
        // sub-buckets), so every window takes the measured-span recount
        if (c->span_extra > 0) bits1 = std::min<uint32_t>(bits1 + (uint32_t)c->span_extra, 64u - bp.ib);
    }
    // the fixed-span 32-bit local sort (k_bucket_sort): the key bits below a
    // sub-bucket fit beside the load slot, and buckets are large enough that
    // windows hold one bucket each (suffixes per bucket of the range >= 4
    // window strides; a rank's range holds m suffixes in bhi - blo buckets --
    // m >> bb undercounted them by G, and ranges took k_bucket_sort_wide)
    const bool fast32 = bits1 > (uint32_t)kSubBits && bits1 - kSubBits <= kLowMax &&
                        m / (uint64_t)(bhi - blo) >= 4ull * kWinStride && !(c->dbg & SA_DEBUG_NO_FAST32);
    // the second pass by per-XCD queues and regions (sa_split.h SegXq): the
    // fixed-span local sort (which loads a one-bucket window's 8 chunks), a
    // grid of whole XCDs, the regions' slack in keys_u (ensure_u_capacity:
    // 2^26 entries and up; one GPU or a rank's range)
    // The regions' offsets are 32-bit (k_split_seg<.., XQ>, k_bucket_starts_xq,
    // load_items_xq): the whole region space must stay below 2^32
    static_assert(kXqQueues == kXq && kXqRegionSlack == kXqSlack, "sa_limits.h mirrors sa_split.h");
    const bool xq = SA_SEG_XQ && allow_xq && fast32 && c->cus % (int)kXq == 0 && !(c->dbg & SA_DEBUG_NO_XQ) &&
                    c->kucap >= xq_region_space(m) + kWave && xq_offsets_fit(m);   // (+ a row: load_items_cr)
    if (st) st->round1_layout = (bp.bs.cmp ? 1 : 0) | (pk8 ? 2 : 0) | (xq ? 4 : 0) | (bp.bs.cmp == 2 ? 8 : 0);
    // XQ workspace: queue cursors / bases / claim counts / tickets, the digit
    // sub-region starts, the per-region chunk starts and counts per bucket
    const uint64_t xqw = xq_words(1u << hb);
    uint32_t* xq_dh = nullptr;
    uint32_t* xq_pc = nullptr;
    uint32_t* xq_pn = nullptr;
    if (xq) {
        const uint64_t need = xqw + 1032 + 2ull * kXq * nb_tab;
        if (c->segx_words < need) {
            hipFree(c->segx);
            c->segx = nullptr;
            c->segx_words = 0;
            if (hipMalloc(&c->segx, need * 4) != hipSuccess) {
                (void)hipGetLastError();
                return set_err(SA_E_NOMEM, "second-pass queue workspace (%llu words)", (unsigned long long)need);
            }
            c->segx_words = need;
        }
        xq_dh = c->segx + xqw;
        xq_pc = xq_dh + 1032;
        xq_pn = xq_pc + (uint64_t)kXq * nb_tab;
    }
    // os layout: ghist [0, kLoRadix) low totals, [kLoRadix, +2^hb) high
    // totals, [1280, +kLoRadix) the first pass's cursors; base [0, kLoRadix)
    // low, [kLoRadix, +2^hb) high
    uint32_t* const g_lo = os_ghist(c);
    uint32_t* const g_hi = os_ghist(c) + kLoRadix;
    // padded segments: the first pass's cursors striped over `stripes`
    // sub-segments (k_split_text; rows [s][digit] in the chunk histograms,
    // free in the bucketed round), the row sums after them
    const uint32_t stripes = padded ? text_stripes(c) : 1u;
    uint32_t* const cursor = stripes > 1 ? c->hist : os_ghist(c) + 5 * kRadix;
    uint32_t* const cursor_sum = stripes > 1 ? c->hist + kMaxStripes * kLoRadix : cursor;
    if (stripes > 1) SA_HIP(hipMemsetAsync(cursor, 0, (size_t)stripes * kLoRadix * 4, s));
    if (!padded) {
        tm.begin(SA_K_SCAN);
        hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, s, (const uint32_t*)g_lo, kLoRadix, os_base(c));
        tm.end();
    }
    // two passes over the bucket: its low kLoBits (any order within a
    // digit), then its high hb bits, keeping the low digit's order (text
    // order -> bucket order; sa_split.h)
    tm.begin(SA_K_SCATTER_FIRST);
    {
        // 12288-position tiles (8192: 5.7 ms, measured on the same box)
        constexpr int kItemsA = SA_ITEMS_A;
        // power-of-two alphabets: two 512-thread workgroups per CU (4.09 -> 3.62 ms
        // at 1 GiB DNA); others one 1024-thread workgroup (ascii127 5.09 ms vs 6.15
        // at 512, alnum 5.13 vs 4.90: profiles/r02_bc_ab_text_block_kinds.txt)
        constexpr int kTextBlock = SA_TEXT_BLOCK;
        const bool pow2 = (bp.bs.sigma & (bp.bs.sigma - 1)) == 0;
        // (the DNA kernel keys each position from a 32-symbol window)
        const bool dna = SA_DNA_SWAR && c->dna && bp.bs.s + bp.bs.R + kItemsA - 1 <= 32 && 2 * bp.bs.s <= 32;
        // (sigma = 256: each position's key from the 8-byte window at it)
        const bool ident = SA_TEXT_IDENT && bp.bs.sigma == 256 && bp.bs.s + bp.bs.R <= 8 && bp.bs.s <= 4;
        auto text_grid = [&](int block) {
            const uint64_t tile = (uint64_t)block * kItemsA;
            return (uint32_t)std::max<uint64_t>(
                1, std::min<uint64_t>((n + tile - 1) / tile, (uint64_t)c->cus * (kSpBlock / block)));
        };
#define SA_TEXT_PASS(P, PK, BLK, DNA, ID)                                                                     \
    hipLaunchKernelGGL((k_split_text<kItemsA, BLK, P, PK, DNA, ID>), dim3(text_grid(BLK)), dim3(BLK), 0, s, d_text, n, \
                       (const uint16_t*)c->code, bp.bs, (const uint32_t*)(padded ? pstart : os_base(c)),           \
                       os_tickets(c), c->keys[0], c->vals_alt, g_hi, cursor, m, blo, bhi,                          \
                       padded ? (const uint32_t*)pstart + 1 : nullptr, padded ? c->words + 11 : nullptr, hb, bp.ib, \
                       stripes)
        if (listed) {
            constexpr int kItemsL = SA_ITEMS_B, kListBlock = SA_LIST_BLOCK;
            const uint64_t tl = (uint64_t)kListBlock * kItemsL;
            const uint32_t gl = (uint32_t)std::max<uint64_t>(
                1, std::min<uint64_t>((m + tl - 1) / tl, (uint64_t)c->cus * (kSpBlock / kListBlock)));
            if (pk8)
                hipLaunchKernelGGL((k_split_list<kItemsL, kListBlock, true>), dim3(gl), dim3(kListBlock), 0, s, bp.bs,
                                   (const uint64_t*)lkeys, (const uint32_t*)lpos, m, blo, (const uint32_t*)os_base(c),
                                   os_tickets(c), c->keys[0], c->vals_alt, g_hi, cursor, hb, bp.ib,
                                   striped ? (const uint32_t*)rcur : nullptr, rcap);
            else
                hipLaunchKernelGGL((k_split_list<kItemsL, kListBlock, false>), dim3(gl), dim3(kListBlock), 0, s, bp.bs,
                                   (const uint64_t*)lkeys, (const uint32_t*)lpos, m, blo, (const uint32_t*)os_base(c),
                                   os_tickets(c), c->keys[0], c->vals_alt, g_hi, cursor, 0u, 0u,
                                   striped ? (const uint32_t*)rcur : nullptr, rcap);
        } else if (pk8 && np2) {
#define SA_TEXT_NP2(R32)                                                                                         \
    hipLaunchKernelGGL((k_split_text<kItemsA, kSpBlock, false, true, false, false, R32>), dim3(text_grid(kSpBlock)), \
                       dim3(kSpBlock), 0, s, d_text, n, (const uint16_t*)c->code, bp.bs,                           \
                       (const uint32_t*)(padded ? pstart : os_base(c)), os_tickets(c), c->keys[0], c->vals_alt, g_hi, \
                       cursor, m, blo, bhi, padded ? (const uint32_t*)pstart + 1 : nullptr,                        \
                       padded ? c->words + 11 : nullptr, hb, bp.ib, stripes)
            if (bp.bs.powR1 * (uint64_t)bp.bs.sigma <= 0xFFFFFFFFull && !(((uint32_t)c->tune >> 28) & 1u))
                SA_TEXT_NP2(true);
            else
                SA_TEXT_NP2(false);
#undef SA_TEXT_NP2
        } else if (pk8 && dna) {
            SA_TEXT_PASS(true, true, kTextBlock, true, false);
        } else if (pk8 && ident) {
            SA_TEXT_PASS(true, true, kTextBlock, false, true);
        } else if (pk8) {
            SA_TEXT_PASS(true, true, kTextBlock, false, false);
        } else if (pow2 && ident) {
            SA_TEXT_PASS(true, false, kTextBlock, false, true);
        } else if (pow2) {
            SA_TEXT_PASS(true, false, kTextBlock, false, false);
        } else if (bp.bs.powR1 * (uint64_t)bp.bs.sigma <= 0xFFFFFFFFull && !(((uint32_t)c->tune >> 28) & 1u)) {
            // sigma^R < 2^32: the remainder in 32 bits (tune bit 28: off, for A/B runs)
            hipLaunchKernelGGL((k_split_text<kItemsA, kSpBlock, false, false, false, false, true>),
                               dim3(text_grid(kSpBlock)), dim3(kSpBlock), 0, s, d_text, n, (const uint16_t*)c->code,
                               bp.bs, (const uint32_t*)(padded ? pstart : os_base(c)), os_tickets(c), c->keys[0],
                               c->vals_alt, g_hi, cursor, m, blo, bhi, padded ? (const uint32_t*)pstart + 1 : nullptr,
                               padded ? c->words + 11 : nullptr, hb, bp.ib, stripes);
        } else {
            SA_TEXT_PASS(false, false, kSpBlock, false, false);
        }
#undef SA_TEXT_PASS
    }
    tm.end();
    add_bytes(st, SA_K_SCATTER_FIRST, listed ? (pk8 ? 20 : 24) * m : n + (pk8 ? 8 : 12) * m);
    tm.begin(SA_K_SCAN);   // the second pass's digit totals came from the first
    hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, s, (const uint32_t*)g_hi, 1u << hb,
                       os_base(c) + kLoRadix);
    if (xq)   // the digits' sub-regions of each queue's region
        hipLaunchKernelGGL(k_xq_dh, dim3(1), dim3(1024), 0, s, (const uint32_t*)g_hi, 1u << hb,
                           (c->dbg & SA_DEBUG_XQ_OVERFLOW) ? 1u : 0u, xq_dh);
    // padded: the dense segment starts from the first pass's final cursors
    if (padded) {
        if (stripes > 1)
            hipLaunchKernelGGL(k_sum_rows, dim3(1), dim3(kLoRadix), 0, s, (const uint32_t*)cursor, stripes, cursor_sum);
        hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, s, (const uint32_t*)cursor_sum, kLoRadix, dlo);
    }
    tm.end();
    tm.begin(SA_K_SCATTER_KEYS);
    {
        // 12288-pair units cut at the first pass's digit boundaries, places
        // claimed per (low digit, high digit) by atomic cursors (sa_split.h)
        constexpr int kItemsB = SA_ITEMS_B, kItemsPk = SA_ITEMS_PK;
        const SrcBucketKeys sb{c->keys[0], c->vals_alt, bp.bs.rb, bp.bs.bsh, bp.bs.cmul, blo};
        const SrcPk8 sp{c->keys[0]};
        uint32_t* tk = os_tickets(c) + 1;
        const uint32_t* hbase = os_base(c) + kLoRadix;
        SA_HIP(hipMemsetAsync(c->segw, 0, segw_words(1u << hb) * 4, s));   // <= 3 MiB
        SegXq sx;
        if (xq) {
            SA_HIP(hipMemsetAsync(c->segx, 0, xqw * 4, s));   // <= 25 MiB
            sx.cur = c->segx;
            sx.sbase = reinterpret_cast<uint64_t*>(c->segx + (uint64_t)kXq * kSegs * (1u << hb));
            sx.done = c->segx + 3ull * kXq * kSegs * (1u << hb);
            sx.tickets = sx.done + kXq * kSegs;
            sx.dh = xq_dh;
            sx.err2 = c->words + 9;
            sx.cap = (uint32_t)std::min<uint64_t>(c->kucap, UINT32_MAX);
        }
        // workgroups of kSegBlock threads (1024 / kSegBlock per CU) for radices up to 512
        constexpr int kSegBlock = SA_SEG_BLOCK;
        const int sblk = hb <= 9 ? kSegBlock : kSpBlock;
        const uint64_t ut = (uint64_t)sblk * (pk8 ? kItemsPk : kItemsB);
        const uint64_t units = (m + ut - 1) / ut + kSegs;
        const uint32_t grid = xq ? (uint32_t)c->cus * (kSpBlock / sblk)   // whole XCDs
                                 : (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(units, (uint64_t)c->cus * (kSpBlock / sblk)));
        switch (hb) {
#define SA_SEG_LAUNCH(S, B, SRC, SH, IT)                                                                      \
    if (xq)                                                                                                   \
        hipLaunchKernelGGL((k_split_seg<S, B, IT, (B <= 9 ? kSegBlock : kSpBlock), true>), dim3(grid),        \
                           dim3(B <= 9 ? kSegBlock : kSpBlock), 0, s, SRC, m, SH,                              \
                           (const uint32_t*)(padded ? pstart : os_base(c)), hbase, c->segw, tk, bp.ib, c->keys_u,      \
                           c->words + 4, padded ? (const uint32_t*)cursor : nullptr,                           \
                           padded ? (const uint32_t*)dlo : nullptr, stripes, sx);                              \
    else                                                                                                      \
        hipLaunchKernelGGL((k_split_seg<S, B, IT, (B <= 9 ? kSegBlock : kSpBlock)>), dim3(grid),                \
                           dim3(B <= 9 ? kSegBlock : kSpBlock), 0, s, SRC, m, SH,                              \
                           (const uint32_t*)(padded ? pstart : os_base(c)), hbase, c->segw, tk, bp.ib, c->keys_u,      \
                           c->words + 4, padded ? (const uint32_t*)cursor : nullptr,                           \
                           padded ? (const uint32_t*)dlo : nullptr, stripes)
#define SA_SEG_PASS(B)                                                                                        \
    case B:                                                                                                   \
        if (pk8) SA_SEG_LAUNCH(SrcPk8, B, sp, 64u - B, kItemsPk);                                             \
        else SA_SEG_LAUNCH(SrcBucketKeys, B, sb, kLoBits, kItemsB);                                           \
        break;
            SA_SEG_PASS(7)
            SA_SEG_PASS(8)
            SA_SEG_PASS(9)
            SA_SEG_PASS(10)
#undef SA_SEG_PASS
#undef SA_SEG_LAUNCH
            default: return set_err(SA_E_INTERNAL, "second bucket pass of %u bits", hb);
        }
        // bucket starts and smallest D values (the local sort rebuilds key1
        // from them; sparse rank look-ups search one bucket)
        const uint32_t gb = (uint32_t)std::min<uint64_t>(((uint64_t)nb_tab + kBlock) / kBlock, 1024);
        uint32_t* bstart = c->segw + kBstartOff;
        uint32_t* bdmin = bstart + kBstartWords;
#define SA_BSTARTS(R)                                                                                         \
    if (xq)                                                                                                   \
        hipLaunchKernelGGL(k_bucket_starts_xq<R>, dim3(R), dim3(kLoRadix), 0, s, hbase, (const uint32_t*)sx.cur, \
                           (const uint32_t*)xq_dh, m, bp.bs.cmul, bp.bs.bsh, bstart, bdmin, xq_pc, xq_pn, blo); \
    else                                                                                                      \
        hipLaunchKernelGGL(k_bucket_starts<R>, dim3(gb), dim3(kBlock), 0, s, (const uint32_t*)(padded ? dlo : os_base(c)), \
                           hbase, (const uint32_t*)c->segw, m, bp.bs.cmul, bp.bs.bsh, bstart, bdmin, blo)
        switch (hb) {
            case 7: SA_BSTARTS(128); break;
            case 8: SA_BSTARTS(256); break;
            case 9: SA_BSTARTS(512); break;
            default: SA_BSTARTS(1024); break;
        }
#undef SA_BSTARTS
    }
    tm.end();
    add_bytes(st, SA_K_SCATTER_KEYS, (pk8 ? 16 : 20) * m);
    SA_HIP(hipGetLastError());
    // windows of whole buckets; ws lives in vals_alt (free again; nw + 1 <= m)
    const uint64_t nw = (m + kWinStride - 1) / kWinStride;
    uint32_t* ws = c->vals_alt;
    uint32_t* list = c->vals_alt + nw + 1;   // non-empty windows (2 nw + 1 <= n)
    tm.begin(SA_K_WINDOWS);
    {
        const uint32_t g1 = (uint32_t)std::min<uint64_t>((nw + kBlock) / kBlock, 8192);
        hipLaunchKernelGGL(k_window_starts_tab, dim3(g1), dim3(kBlock), 0, s, (const uint32_t*)(c->segw + kBstartOff),
                           nb_tab, m, nw, ws, list + 4 * nw + 2);   // wb: see br below
        const uint32_t g2 = (uint32_t)std::min<uint64_t>((nw + kBlock - 1) / kBlock, 1024);
        hipLaunchKernelGGL(k_window_list, dim3(g2), dim3(kBlock), 0, s, (const uint32_t*)ws, nw, list, c->words);
    }
    tm.end();
    add_bytes(st, SA_K_WINDOWS, 8 * nw);
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(c->host_words, c->words, 48, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    if (c->host_words[4]) return set_err(SA_E_INTERNAL, "radix look-back did not complete");
    if (padded && c->host_words[11]) {   // a digit outgrew its sampled segment: exact totals
        SA_TRACE("  bucketed round 1: padded segment overflow, again with exact digit totals");
        const int rc = round1_bucketed(c, d_text, n, d_sa, bp, br_, s, tm, st, done, fused, seg, ksh, false, allow_xq);
        if (st) st->round1_segments = 2;
        return rc;
    }
    if (xq && c->host_words[9]) {   // a queue's digit outgrew its sub-region: one region
        SA_TRACE("  bucketed round 1: second-pass queue overflow, again with one region");
        return round1_bucketed(c, d_text, n, d_sa, bp, br_, s, tm, st, done, fused, seg, ksh, allow_pad, false);
    }
    if (st) st->largest_window = (int32_t)std::min<uint32_t>(c->host_words[5], INT32_MAX);
    if (c->host_words[5] > (uint32_t)kBsCap) {
        SA_TRACE("  bucketed round 1: window of %u > %d suffixes, full sort instead", c->host_words[5], kBsCap);
        return SA_OK;
    }
    // windows with clustered keys, then per-window U / U-group counts (scanned
    // in place: nw + 1 each), then each window's first bucket (nw + 1,
    // written by k_window_starts_tab); 6 nw + 4 <= capacity
    uint32_t* skew = list + nw;
    uint32_t* cnt_u = skew + nw;
    uint32_t* cnt_g = cnt_u + nw + 1;
    BucketRel br{cnt_g + nw + 1, c->segw + kBstartOff, c->segw + kBstartOff + kBstartWords, bp.bs.rb};
    // the local sort's sub-buckets split a one-bucket window's whole key span
    // (D values per bucket x 2^rb) when the compact layout fills it; also for
    // alphabets whose buckets fill ~80 % of that span (1 GiB alnum / ascii127
    // local sort 7.05 / 6.85 ms with measured spans, 4.75 / 4.56 with the
    // fixed one: profiles/r02_av_ab_kinds_fixed_span_pow2_only.txt)
    br.bits1 = bits1;
    SA_HIP(hipMemsetAsync(cnt_u, 0, (2 * nw + 2) * 4, s));
    uint32_t* const rank_arr = br_.rank ? br_.rank : c->rank;
    uint32_t* const member = br_.member ? br_.member : c->member;
    SA_HIP(hipMemsetAsync(member, 0, (n + 31) / 32 * 4, s));
    // sorted key1 sampled (every 2^kKeySample-th SA position) for the sparse
    // rank look-ups; a round that turns out dense re-runs the sort with every
    // key1 below (segments() reads them all)
    SegOut so{rank_arr, member, br_.sa_off, c->u_pos[1], c->u_idx[1], c->u_g[1], cnt_u, cnt_g, kKeySample};
    so.tmp_rank = br_.prefix ? br_.tmp_rank : nullptr;
    // one GPU: no samples now (round 2 keys by key1 from the text); a later
    // round that needs them rebuilds them (build_packed, k_key1_samples).
    // Range builds answer other ranks' look-ups from them: always written.
    so.samples = (SA_LAZY_SAMPLES && !br_.always_u && !(c->dbg & SA_DEBUG_NO_KEY1_ROUND)) ? 0u : 1u;
    // fixed-span windows whose keys cluster, for a second launch with the
    // measured span (after the windows' first buckets: 7 nw + 4 <= capacity)
    uint32_t* const retry = cnt_g + 2 * nw + 2;
    BucketRel br_measured = br;
    br_measured.bits1 = 0;
    // one-bucket window headers after the retry list (16-byte aligned; 11 nw + 8 <= capacity)
    uint4* const hdr = reinterpret_cast<uint4*>(((uintptr_t)(retry + nw + 4) + 15) & ~(uintptr_t)15);
    // XQ: the one-bucket windows' chunk headers after them (16 words each; 27 nw + 8 <= capacity), and the
    // windows for the measured-span / LSD kernels at their SA positions in keys[1] (free in the bucketed round)
    uint32_t* const hx = xq ? reinterpret_cast<uint32_t*>(hdr + nw + 1) : nullptr;
    // and their row tables (3 kBsRows words each; 27 nw + 432 (nw + 1) + 24 <= capacity)
    constexpr uint32_t kBsRows = (kBsBlock / kWave) * kBsItems;
    uint32_t* const xrows = xq ? hx + 16 * (nw + 1) : nullptr;
    const uint64_t* const wide_in = xq ? c->keys[1] : c->keys_u;
    auto local_sort = [&](const SegOut& o) {
        const uint32_t g = std::max<uint32_t>(1, std::min(c->host_words[7], kBsGrid));
        // (no SA_HIP here: its error return would make the lambda non-void)
        (void)hipMemsetAsync(c->words + kRetryWord, 0, 12, s);   // retry count, one-bucket windows, ticket
        if (fast32) {
            const uint32_t gs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nw + kBlock - 1) / kBlock, 1024));
            // XQ chunk rows (sa_bucket.h load_items_cr; tune bit 29: the
            // window-order rows with a per-lane chunk select)
            const bool cr = xq && !(((uint32_t)c->tune >> 29) & 1u);
            hipLaunchKernelGGL(k_window_split, dim3(gs), dim3(kBlock), 0, s, (const uint32_t*)list, (const uint32_t*)ws,
                               br, c->words, hdr, retry, 1u, (const uint32_t*)xq_pc, (const uint32_t*)xq_pn, nb_tab, hx,
                               cr ? kBsRows : 0u);
            if (xq) {
                if (cr)
                    hipLaunchKernelGGL(k_window_rows<true>, dim3(2048), dim3(kBlock), 0, s, (const uint32_t*)c->words,
                                       (const uint4*)hdr, (const uint32_t*)hx, kBsRows, xrows);
                else
                    hipLaunchKernelGGL(k_window_rows<false>, dim3(2048), dim3(kBlock), 0, s, (const uint32_t*)c->words,
                                       (const uint4*)hdr, (const uint32_t*)hx, kBsRows, xrows);
                XqWin xw;
                xw.hx = hx;
                xw.rows = xrows;
#define SA_LS_XQ(V, CR)                                                                                          \
    hipLaunchKernelGGL((k_bucket_sort<kBsBlock, kBsItems, NoProbe, true, V, CR>), dim3(kBsWpc * (uint32_t)c->cus), \
                       dim3(kBsBlock), 0, s, (const uint64_t*)c->keys_u, (const uint4*)hdr, bp.bs.rb, br.bits1,  \
                       bp.ib, c->words, c->keys[0], d_sa, retry, o, xw)
                switch (ls_variant(c) | (cr ? 4 : 0)) {
                case 1: SA_LS_XQ(1, false); break;
                case 2: SA_LS_XQ(2, false); break;
                case 3: SA_LS_XQ(3, false); break;
                case 4: SA_LS_XQ(0, true); break;
                case 5: SA_LS_XQ(1, true); break;
                case 6: SA_LS_XQ(2, true); break;
                case 7: SA_LS_XQ(3, true); break;
                default: SA_LS_XQ(0, false); break;
                }
#undef SA_LS_XQ
                // the windows for the measured-span kernel (several buckets, or
                // clustered keys), from their chunks to their SA positions
                hipLaunchKernelGGL(k_window_gather, dim3(1024), dim3(kBlock), 0, s, (const uint32_t*)retry,
                                   (const uint32_t*)c->words, (const uint32_t*)ws, (const uint32_t*)br.wb,
                                   (const uint32_t*)xq_pc, (const uint32_t*)xq_pn, nb_tab, (const uint64_t*)c->keys_u,
                                   c->keys[1]);
            } else {
#define SA_LS(V)                                                                                                 \
    hipLaunchKernelGGL((k_bucket_sort<kBsBlock, kBsItems, NoProbe, false, V>), dim3(kBsWpc * (uint32_t)c->cus),  \
                       dim3(kBsBlock), 0, s, (const uint64_t*)c->keys_u, (const uint4*)hdr, bp.bs.rb, br.bits1,  \
                       bp.ib, c->words, c->keys[0], d_sa, retry, o)
                switch (ls_variant(c)) {
                case 1: SA_LS(1); break;
                case 2: SA_LS(2); break;
                case 3: SA_LS(3); break;
                default: SA_LS(0); break;
                }
#undef SA_LS
            }
        } else {
            hipLaunchKernelGGL((k_bucket_sort_wide<kBsBlock, kBsItems>), dim3(g), dim3(kBsBlock), 0, s,
                               (const uint64_t*)c->keys_u, br, (const uint32_t*)ws, (const uint32_t*)list, c->words,
                               bp.ib, c->keys[0], d_sa, skew, o, br.bits1 ? retry : (uint32_t*)nullptr, 7u);
        }
        if (br.bits1)   // rare: a small grid loops over the retried windows (measured span)
            hipLaunchKernelGGL((k_bucket_sort_wide<kBsBlock, kBsItems>), dim3(std::min<uint32_t>(g, 1024)),
                               dim3(kBsBlock), 0, s, wide_in, br_measured, (const uint32_t*)ws,
                               (const uint32_t*)retry, c->words, bp.ib, c->keys[0], d_sa, skew, o, (uint32_t*)nullptr,
                               (uint32_t)kRetryWord);
        // skewed windows are rare: a small grid loops over them (one
        // workgroup per listed window spent 0.1 ms on empty workgroups)
        const uint32_t gl = std::min<uint32_t>(g, 1024);
        hipLaunchKernelGGL((k_bucket_sort_lsd<kBsBlock, kBsItems>), dim3(gl), dim3(kBsBlock), 0, s,
                           wide_in, br, (const uint32_t*)ws, (const uint32_t*)skew, c->words, bp.ib,
                           c->keys[0], d_sa, o);
    };
    tm.begin(SA_K_LOCAL_SORT);
    local_sort(so);
    tm.end();
    add_bytes(st, SA_K_LOCAL_SORT, 12 * m + (so.samples ? (m >> kKeySample) * 8 : 0));
    SA_HIP(hipGetLastError());
    // the unsorted set, in SA order, compacted before the counts are read
    // back (its launches overlap that round trip; a round that turns out
    // dense, or falls back, ignores it: segments() writes the set again)
    tm.begin(SA_K_SEG_WRITE);
    {
        const uint32_t wb = (uint32_t)((nw + 1 + kWsBlock - 1) / kWsBlock);
        uint32_t* part = c->hist;   // 2 words per block (<= 2 * 256 * kMaxChunks)
        hipLaunchKernelGGL(k_wscan_reduce, dim3(wb), dim3(kBlock), 0, s, (const uint32_t*)cnt_u, (const uint32_t*)cnt_g,
                           nw, part);
        hipLaunchKernelGGL(k_wscan_top, dim3(1), dim3(kBlock), 0, s, part, wb);
        hipLaunchKernelGGL(k_wscan_apply, dim3(wb), dim3(kBlock), 0, s, cnt_u, cnt_g, nw, (const uint32_t*)part);
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((c->host_words[7] + kWaves - 1) / kWaves, 4096));
        RankMap rm;
        if (br_.prefix) {
            // the member bitmap is complete: its popcount prefix gives each
            // member's slot in the compact rank map
            const uint64_t nwb = (n + 31) / 32;
            const uint32_t pb = (uint32_t)((nwb + kPcBlock - 1) / kPcBlock);
            uint32_t* ppart = br_.prefix + nwb + 1;
            hipLaunchKernelGGL(k_popc_reduce, dim3(pb), dim3(kBlock), 0, s, (const uint32_t*)member, nwb, ppart);
            hipLaunchKernelGGL(k_popc_top, dim3(1), dim3(kPcTop), 0, s, ppart, pb);
            hipLaunchKernelGGL(k_popc_apply, dim3(pb), dim3(kBlock), 0, s, (const uint32_t*)member, nwb,
                               (const uint32_t*)ppart, br_.prefix);
            rm = RankMap{member, br_.prefix};
        }
        hipLaunchKernelGGL(k_u_gather, dim3(g), dim3(kBlock), 0, s, (const uint32_t*)list, (const uint32_t*)c->words,
                           (const uint32_t*)ws, (const uint32_t*)cnt_u, (const uint32_t*)cnt_g, so, c->u_pos[0],
                           c->u_idx[0], c->u_g[0], rm);
    }
    tm.end();
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(c->host_words, c->words, 44, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    if (c->host_words[6]) {
        SA_TRACE("  bucketed round 1: local sort flags %u, full sort instead", c->host_words[6]);
        return SA_OK;
    }
    seg[0] = c->host_words[0];
    seg[1] = c->host_words[1];
    seg[2] = c->host_words[2];
    add_bytes(st, SA_K_LOCAL_SORT, seg[1] * 28);   // unsorted set: rank, member bit, 3 tmp words
    add_bytes(st, SA_K_SEG_WRITE, 8 * (2 * nw + 2) + seg[1] * 24);
    if (!br_.always_u && seg[1] > n / kSparseDiv) {
        // dense ranks follow (segments() over every key1): the same sort
        // again, writing every key1 and nothing of the unsorted set
        SegOut full{};
        full.ksh = 0;
        SA_HIP(hipMemsetAsync(c->words + 10, 0, 4, s));   // the skewed-window list is rebuilt
        tm.begin(SA_K_LOCAL_SORT);
        local_sort(full);
        tm.end();
        add_bytes(st, SA_K_LOCAL_SORT, 20 * m);
        SA_HIP(hipGetLastError());
    } else {
        *ksh = kKeySample;
        *fused = true;
        c->samples_pending = so.samples == 0u;
    }
    SA_TRACE("  bucketed round 1: s=%u R=%u rb=%u cmp=%u pk8=%d windows=%u (skewed %u) largest=%u", bp.bs.s, bp.bs.R,
             bp.bs.rb, bp.bs.cmp, pk8 ? 1 : 0, c->host_words[7], c->host_words[10], c->host_words[5]);
    *done = true;
    return SA_OK;
}
