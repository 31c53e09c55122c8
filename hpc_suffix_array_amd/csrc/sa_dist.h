// sa_dist.h -- per-rank phases of the range-partitioned multi-GPU build
// (one process per GPU; hpc_suffix_array_amd/distributed.py drives them and
// runs the RCCL collectives between them).  Included by sa_build.hip inside
// namespace sa, after the packed schedule.
//
// Replaces the reference's MPI strategy (src/mpi/manber_myers_mpi.c:22-160:
// Scatterv of 12-byte records, then per round a local qsort, a Gatherv of ALL
// records to rank 0, a serial qsort of n records there and a Bcast of the
// n-int rank array), which moves O(n) bytes per round through one process.
//
// Layout.  Every rank holds the text (1 byte per suffix; main_mpi.c:51
// broadcasts it too).  Everything else -- keys, SA, ranks, unsorted sets --
// is partitioned by SA ranges: the bucketed first round's buckets (the first
// s symbols of a suffix, sa_bucket.h) are cut into `world` contiguous ranges
// of about n / world suffixes, and rank q sorts the suffixes of its range,
// which occupy SA positions [sa_off_q, sa_off_q + m_q).  A rank finds its
// suffixes by scanning its own copy of the text: HBM reads (8 TB/s) replace
// the bucket exchange over xGMI (7 x ~150 GB/s) that records would need.
//
//   begin    alphabet codes, K, the bucket plan for the global n; histogram of
//            the coarse bucket (top 12 bits) over this rank's text slice
//   [host]   all_reduce of the coarse histograms -> identical cuts on every rank
//   cuts     this rank's bucket range, m, sa_off; coarse bucket -> owner table
//   round1   the bucketed first round restricted to the range (the two bucket
//            passes scan the whole text and keep the range's suffixes): the
//            local SA, sorted key1, bucket starts, and the unsorted set with
//            ranks = global group-head position + 1 (n-entry arrays written
//            for the unsorted suffixes only)
//   rounds   h = K, 2K, ... while any rank has unsorted suffixes:
//            req_count  the owner of rank[x + h] for each unsorted x (the rank
//                       whose range holds x + h's bucket)
//            [host]     all_gather of the counts
//            req_fill   the requests grouped by owner
//            [host]     all_to_all of the requests
//            answer     rank[j] for the requests this rank owns: the member
//                       map, else j's round-1 group head by a binary search of
//                       key1(j) in the range's sorted keys (inside its bucket)
//            [host]     all_to_all of the answers back
//            refine     sort the unsorted set by (group, rank[x + h]), re-rank,
//                       write SA positions, compact the next unsorted set
// Groups never straddle ranks (a group is a set of equal K-prefixes, inside
// one bucket), so every sort and re-rank is local; only rank look-ups cross.
#pragma once
// workgroups per CU of the coarse histogram (each flushes its 4096 bins
// with device atomics): over an eighth of 1 GiB DNA 2 / 4 / 16 per CU took
// 109 / 82 / 115 us (profiles/r03_z_ab_coarse_grid.txt)
#ifndef SA_COARSE_WPC
#define SA_COARSE_WPC 4
#endif


constexpr int kDistMaxWorld = 1024;

struct DistState {
    uint64_t n = 0;
    int world = 1, rank = 0;
    uint32_t sigma = 0, K = 0;
    bool planned = false;
    const uint8_t* text = nullptr;   // this rank's copy of the whole text (HBM)
    BucketPlan bp;
    // cuts (coarse bucket boundaries, identical on every rank)
    std::vector<uint32_t> cut;
    uint32_t blo = 0, bhi = 0;
    uint64_t m = 0, sa_off = 0, mcap = 0;
    uint32_t* sa = nullptr;          // this range's SA (the caller's slice, from round 1 on)
    uint32_t ksh = 0;                // round-1 key samples: every 2^ksh-th key1
    // device
    uint64_t cap_n = 0, cap_m = 0;
    uint16_t* owner_tab = nullptr;   // kCoarse: coarse bucket -> rank
    uint32_t* gmember = nullptr;     // n bits: this range's round-1 unsorted suffixes
    uint32_t* gprefix = nullptr;     // n / 32 words + scan sums: the bitmap's popcount prefix
    uint32_t* crank = nullptr;       // cap_m: their ranks, in text order (RankMap)
    uint64_t* r1 = nullptr;          // cap_m: rank[x + h] of each unsorted x
    uint32_t* perm = nullptr;        // cap_m: request slot -> unsorted index
    uint32_t* owner = nullptr;       // cap_m: owner of each unsorted x's request
    uint32_t* cnt = nullptr;         // [0, W) counts, [W, 2W) cursors, [2W] error flags
    // unsorted set (u_pos / u_idx / u_g[uo] of the context)
    uint64_t mu = 0, gu = 0;
    int uo = 0;
    std::vector<uint64_t> send;      // requests per owner of the current round
    uint64_t nsend = 0;
    int rounds = 0;
};

static void free_dist(sa_context* c) {
    DistState* d = c->dist;
    if (!d) return;
    hipFree(d->owner_tab);
    hipFree(d->gmember);
    hipFree(d->gprefix);
    hipFree(d->crank);
    hipFree(d->r1);
    hipFree(d->perm);
    hipFree(d->owner);
    hipFree(d->cnt);
    delete d;
    c->dist = nullptr;
}

static DistState* dist_of(sa_context* c) {
    if (!c->dist) c->dist = new DistState();
    return c->dist;
}

static int ensure_dist_n(sa_context* c, uint64_t n) {
    DistState* d = dist_of(c);
    if (d->gmember && d->cap_n >= n) return SA_OK;
    hipFree(d->gprefix);
    hipFree(d->gmember);
    d->gprefix = nullptr;
    d->gmember = nullptr;
    d->cap_n = 0;
    if (!d->owner_tab && hipMalloc(&d->owner_tab, kCoarse * 2) != hipSuccess) d->owner_tab = nullptr;
    if (!d->cnt && hipMalloc(&d->cnt, (2 * kDistMaxWorld + 8) * 4) != hipSuccess) d->cnt = nullptr;
    // the member bitmap and its popcount prefix (+ the scan's block sums):
    // 8 bytes per 32 positions, not the 4 per position of an n-entry rank
    // array -- per-rank memory falls with the world size (RankMap)
    const uint64_t nwb = (std::max<uint64_t>(n, 1) + 31) / 32;
    if (!d->owner_tab || !d->cnt ||
        hipMalloc(&d->gprefix, (nwb + 1 + (nwb + kWsBlock - 1) / kWsBlock + 64) * 4) != hipSuccess ||
        hipMalloc(&d->gmember, align_up(std::max<uint64_t>(n, 1), 1024) / 8) != hipSuccess) {
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "range-partitioned build: rank arrays for n=%llu", (unsigned long long)n);
    }
    d->cap_n = n;
    return SA_OK;
}

static int ensure_dist_m(sa_context* c, uint64_t m);

// Everything a range build of up to max_n symbols over `world` ranks
// allocates (the n-entry member map and its prefix, the range's workspace
// for the largest range plan_cuts accepts: n/W + n/(2W) + 65536 suffixes),
// ahead of the first build: the first 8-rank build spent 2.68 s in cuts
// allocating it.
static int dist_reserve(sa_context* c, uint64_t max_n, int world) {
    if (world < 1 || world > kDistMaxWorld) return set_err(SA_E_INVALID, "world %d", world);
    SA_HIP(hipSetDevice(c->device));
    int rc = ensure_dist_n(c, max_n);
    if (rc) return rc;
    const uint64_t w = (uint64_t)world;
    const uint64_t m = std::min<uint64_t>(max_n, max_n / w + max_n / (2 * w) + 65536);
    return ensure_dist_m(c, std::max<uint64_t>(m, 1));
}

static int ensure_dist_m(sa_context* c, uint64_t m) {
    DistState* d = dist_of(c);
    int rc = ensure_capacity(c, m);
    if (rc) return rc;
    rc = ensure_u_capacity(c, rec_capacity(m));   // round 1's striped records (sa_round1.h)
    if (rc) return rc;
    if (d->r1 && d->cap_m >= m) return SA_OK;
    hipFree(d->r1);
    hipFree(d->perm);
    hipFree(d->owner);
    hipFree(d->crank);
    d->r1 = nullptr;
    d->perm = d->owner = d->crank = nullptr;
    d->cap_m = 0;
    const uint64_t a = align_up(std::max<uint64_t>(m, 1), 64);
    if (hipMalloc(&d->r1, a * 8) != hipSuccess || hipMalloc(&d->perm, a * 4) != hipSuccess ||
        hipMalloc(&d->owner, a * 4) != hipSuccess || hipMalloc(&d->crank, a * 4) != hipSuccess) {
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "range-partitioned build: unsorted-set buffers for m=%llu", (unsigned long long)m);
    }
    d->cap_m = m;
    return SA_OK;
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// the 256-entry byte -> dense digit map in LDS (code - 1, absent bytes 0)
__device__ __forceinline__ void load_map(const uint16_t* __restrict__ code, uint8_t* s_map) {
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
        const uint32_t cv = code[i];
        s_map[i] = (uint8_t)(cv ? cv - 1u : 0u);
    }
    __syncthreads();
}

// Owner of rank[x + h] for each unsorted x (x + h < n): the rank whose bucket
// range holds x + h's bucket (its first s symbols, read from the text);
// counts per owner, aggregated per wave (few owners, many requests).
__global__ __launch_bounds__(kBlock) void k_dist_owner(const uint32_t* __restrict__ u_idx, uint64_t mu, uint64_t h,
                                                       const uint8_t* __restrict__ text, uint64_t n,
                                                       const uint16_t* __restrict__ code, BucketSpec b,
                                                       const uint16_t* __restrict__ owner_tab, uint32_t cshift,
                                                       uint32_t* __restrict__ owner, uint32_t* __restrict__ counts) {
    __shared__ uint8_t s_map[256];
    load_map(code, s_map);
    const uint32_t lane = lane_id();
    for (uint64_t e0 = (uint64_t)blockIdx.x * kBlock; e0 < mu; e0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t e = e0 + threadIdx.x;
        uint32_t o = 0xFFFFFFFFu;
        if (e < mu) {
            const uint64_t j = (uint64_t)u_idx[e] + h;
            if (j < n) {
                uint32_t D;
                key1_words<false>(text, n, s_map, b, j, &D);
                const uint32_t bk = (uint32_t)(((uint64_t)D * b.cmul) >> b.bsh);
                o = owner_tab[bk >> cshift];
            }
            owner[e] = o;
        }
        // one atomic per distinct owner per wave
        uint64_t pending = __ballot(o != 0xFFFFFFFFu);
        while (pending) {
            const uint32_t lead = (uint32_t)__builtin_ctzll(pending);
            const uint32_t ow = (uint32_t)__shfl((int)o, (int)lead, kWave);
            const uint64_t same = __ballot(o == ow);
            if (lane == lead) atomicAdd(&counts[ow], (uint32_t)__popcll(same));
            pending &= ~same;
        }
    }
}

// requests j = x + h grouped by owner (order within an owner arbitrary),
// perm[slot] = the unsorted index the answer returns to
__global__ __launch_bounds__(kBlock) void k_dist_fill(const uint32_t* __restrict__ u_idx, uint64_t mu, uint64_t h,
                                                      const uint32_t* __restrict__ owner,
                                                      uint32_t* __restrict__ cursor, uint32_t* __restrict__ req,
                                                      uint32_t* __restrict__ perm) {
    const uint32_t lane = lane_id();
    for (uint64_t e0 = (uint64_t)blockIdx.x * kBlock; e0 < mu; e0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t e = e0 + threadIdx.x;
        const uint32_t o = e < mu ? owner[e] : 0xFFFFFFFFu;
        uint64_t pending = __ballot(o != 0xFFFFFFFFu);
        uint32_t slot = 0;
        while (pending) {
            const uint32_t lead = (uint32_t)__builtin_ctzll(pending);
            const uint32_t ow = (uint32_t)__shfl((int)o, (int)lead, kWave);
            const uint64_t same = __ballot(o == ow);
            uint32_t base = 0;
            if (lane == lead) base = atomicAdd(&cursor[ow], (uint32_t)__popcll(same));
            base = (uint32_t)__shfl((int)base, (int)lead, kWave);
            if (o == ow) slot = base + (uint32_t)__popcll(same & lanemask_lt());
            pending &= ~same;
        }
        if (o != 0xFFFFFFFFu) {
            req[slot] = (uint32_t)(u_idx[e] + h);
            perm[slot] = (uint32_t)e;
        }
    }
}

// rank[j] for requests this rank owns: the member map (unsorted suffixes of
// this range), else the round-1 group head of key1(j) in the range's sorted
// keys, searched inside j's bucket.  err bit 0: a request outside the range.
struct DistLookup {
    const uint32_t* __restrict__ crank;    // the members' ranks (compact, RankMap rm)
    RankMap rm;
    const uint64_t* __restrict__ keys1;    // this range's sorted key1: every 2^ksh-th of m
    const uint32_t* __restrict__ sa;       // this range's SA (m; key1 of the other slots)
    uint32_t ksh;
    const uint32_t* __restrict__ bstart;   // local bucket starts
    const uint8_t* __restrict__ text;
    const uint16_t* __restrict__ code;
    uint64_t n;
    BucketSpec bs;
    uint32_t blo, nb;
    uint64_t sa_off;
};

// rank[j] (j < n) by the owner of j's bucket; *bad set on a j outside the range
__device__ __forceinline__ uint64_t dist_rank_of(const DistLookup& L, const uint8_t* s_map, uint64_t j, bool* bad) {
    if ((L.rm.member[j >> 5] >> (j & 31)) & 1u) return L.crank[L.rm.slot((uint32_t)j)];
    uint32_t D;
    const uint64_t x = key1_words<true>(L.text, L.n, s_map, L.bs, j, &D);
    const uint32_t b = (uint32_t)(((uint64_t)D * L.bs.cmul) >> L.bs.bsh) - L.blo;
    if (b >= L.nb) {
        *bad = true;
        return 0;
    }
    auto key_at = [&](uint64_t p) {
        uint32_t d;
        return key1_words<true>(L.text, L.n, s_map, L.bs, p, &d);
    };
    return L.sa_off + lower_bound_sampled(L.keys1, L.ksh, L.sa, L.bstart[b], L.bstart[b + 1], x, key_at) + 1;
}

__global__ __launch_bounds__(kBlock) void k_dist_answer(const uint32_t* __restrict__ req, uint64_t nreq, DistLookup L,
                                                        uint64_t* __restrict__ ans, uint32_t* __restrict__ err) {
    __shared__ uint8_t s_map[256];
    load_map(L.code, s_map);
    bool bad = false;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < nreq; t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t j = req[t];
        uint64_t r = 0;
        if (j >= L.n) bad = true;
        else r = dist_rank_of(L, s_map, j, &bad);
        ans[t] = r;
    }
    if (bad) atomicOr(err, 1u);
}

// one rank (world 1): rank[x + h] looked up in place, no requests
__global__ __launch_bounds__(kBlock) void k_dist_r1_local(const uint32_t* __restrict__ u_idx, uint64_t mu, uint64_t h,
                                                          DistLookup L, uint64_t* __restrict__ r1,
                                                          uint32_t* __restrict__ err) {
    __shared__ uint8_t s_map[256];
    load_map(L.code, s_map);
    bool bad = false;
    for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < mu; e += (uint64_t)gridDim.x * kBlock) {
        const uint64_t j = (uint64_t)u_idx[e] + h;
        r1[e] = j < L.n ? dist_rank_of(L, s_map, j, &bad) : 0;
    }
    if (bad) atomicOr(err, 1u);
}

// answers back into unsorted order (r1 zeroed first: x + h >= n keeps 0)
__global__ __launch_bounds__(kBlock) void k_dist_place(const uint64_t* __restrict__ ans, uint64_t nsend,
                                                       const uint32_t* __restrict__ perm, uint64_t* __restrict__ r1) {
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < nsend; t += (uint64_t)gridDim.x * kBlock)
        r1[perm[t]] = ans[t];
}

// key source of a distributed unsorted-set round: (group, rank[x + h]) with
// rank[x + h] fetched from its owner beforehand
struct SrcUArr {
    const uint32_t* __restrict__ u_idx;
    const uint32_t* __restrict__ u_g;
    const uint64_t* __restrict__ r1;
    uint32_t wr;
    __device__ __forceinline__ uint64_t key(uint64_t e) const { return ((uint64_t)u_g[e] << wr) | r1[e]; }
    __device__ __forceinline__ uint32_t val(uint64_t e) const { return u_idx[e]; }
};

// ---------------------------------------------------------------------------
// host phases
// ---------------------------------------------------------------------------
static uint32_t dist_cshift(const DistState& d) { return d.bp.bs.bb - kCoarseBits; }

#ifndef SA_DIST_SHORT_K
#define SA_DIST_SHORT_K 1
#endif

static int dist_begin(sa_context* c, const uint8_t* d_text, uint64_t n, int world, int rank,
                      const uint32_t present[8], uint64_t* d_coarse, hipStream_t s, sa_dist_info* info) {
    std::memset(info, 0, sizeof *info);
    if (world < 1 || world > kDistMaxWorld || rank < 0 || rank >= world)
        return set_err(SA_E_INVALID, "rank %d of world %d", rank, world);
    if (n < 2 || n > (1ull << 32)) return set_err(SA_E_INVALID, "n = %llu outside [2, 2^32]", (unsigned long long)n);
    if (!d_text || !present) return set_err(SA_E_INVALID, "NULL argument");
    SA_HIP(hipSetDevice(c->device));
    DistState* d = dist_of(c);
    d->n = n;
    d->world = world;
    d->rank = rank;
    d->planned = false;
    d->text = d_text;
    d->rounds = 0;
    uint16_t* h_code = reinterpret_cast<uint16_t*>(c->host_words + 320);
    uint32_t sigma = 0;
    for (int b = 0; b < 256; ++b) h_code[b] = ((present[b >> 5] >> (b & 31)) & 1u) ? (uint16_t)(++sigma) : 0;
    c->dna = sigma == 4 && h_code['A'] && h_code['C'] && h_code['G'] && h_code['T'];
    SA_HIP(hipMemcpyAsync(c->code, h_code, 256 * 2, hipMemcpyHostToDevice, s));
    // the text's tail (every rank holds the text: all take the same layout)
    const uint32_t tail_n = (uint32_t)std::min<uint64_t>(n, (uint64_t)kMaxK);
    uint8_t* h_tail = reinterpret_cast<uint8_t*>(c->host_words + 2048);
    SA_HIP(hipMemcpyAsync(h_tail, d_text + (n - tail_n), tail_n, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    d->sigma = sigma;
    const uint32_t K = choose_chars(sigma, n, 0);
    info->sigma = (int32_t)sigma;
    BucketPlan bp;
    c->radix = 0;
    bool planned = plan_bucketed(sigma, n, K, SA_ROUND1_BUCKETED, 0, &bp, world, !(c->dbg & SA_DEBUG_NO_CMP));
    if (planned && bp.bs.cmp && short_suffix_ties(h_tail, n, tail_n, h_code, sigma, bp.bs.s, bp.bs.R))
        planned = plan_bucketed(sigma, n, K, SA_ROUND1_BUCKETED, 0, &bp, world, false);
    if (!planned) {
        info->status = SA_DIST_UNSUPPORTED;   // one symbol / a key layout that does not fit
        return SA_OK;
    }
    // one symbol fewer when that lets a range's first pass write packed
    // 8-byte items (PK8: 8 + 12 bytes per suffix less through the two bucket
    // passes) and sigma^K stays >= 256 n, i.e. about n / 256 suffixes left
    // unsorted by round 1 for one more look-up round: configs[3] (byte256,
    // n = 2^32, G = 8) K = 6 -> 5, 8 + 5 + 25 + 32 -> 8 + 5 + 17 + 32 bits.
    // Every rank derives the same K (sigma, n and world only).
    if (SA_DIST_SHORT_K && world > 1 && bp.K > bp.bs.s + 1) {
        const uint32_t hb_est = range_hb((uint32_t)((3ull << bp.bs.bb) / (2ull * (uint64_t)world)));
        unsigned __int128 pk = 1;
        for (uint32_t t = 0; t + 1 < bp.K; ++t) pk *= sigma;
        BucketPlan b2;
        if (!plan_pk8(bp, hb_est, c->dbg) && pk >= (unsigned __int128)n * 256u &&
            plan_bucketed(sigma, n, bp.K - 1, SA_ROUND1_BUCKETED, 0, &b2, world, bp.bs.cmp != 0) &&
            (!b2.bs.cmp || !short_suffix_ties(h_tail, n, tail_n, h_code, sigma, b2.bs.s, b2.bs.R)) &&
            plan_pk8(b2, hb_est, c->dbg))
            bp = b2;
    }
    d->bp = bp;
    d->K = bp.K;
    d->planned = true;
    info->K = (int32_t)bp.K;
    info->bucket_bits = (int32_t)bp.bs.bb;
    info->status = SA_DIST_OK;
    if (world > 1) {
        if (!d_coarse) return set_err(SA_E_INVALID, "NULL coarse histogram");
        SA_HIP(hipMemsetAsync(d_coarse, 0, kCoarse * 8, s));
        const uint64_t lo = n * (uint64_t)rank / world, hi = n * (uint64_t)(rank + 1) / world;
        if (hi > lo) {
            const uint64_t tiles = (hi - lo + kTile - 1) / kTile;
            const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles, (uint64_t)SA_COARSE_WPC * (uint32_t)c->cus));
            if (sigma == 256)
                hipLaunchKernelGGL((k_bucket_hist<true, true, 0, true>), dim3(g), dim3(kBlock), 0, s, d_text, n,
                                   (const uint16_t*)c->code, bp.bs, (uint32_t*)d_coarse, lo, hi, 0u, 1u << bp.bs.bb);
            else if ((sigma & (sigma - 1)) == 0)
                hipLaunchKernelGGL((k_bucket_hist<true, true>), dim3(g), dim3(kBlock), 0, s, d_text, n,
                                   (const uint16_t*)c->code, bp.bs, (uint32_t*)d_coarse, lo, hi, 0u, 1u << bp.bs.bb);
            else
                hipLaunchKernelGGL((k_bucket_hist<false, true>), dim3(g), dim3(kBlock), 0, s, d_text, n,
                                   (const uint16_t*)c->code, bp.bs, (uint32_t*)d_coarse, lo, hi, 0u, 1u << bp.bs.bb);
            SA_HIP(hipGetLastError());
        }
    }
    return SA_OK;
}

// The cut plan (host only): W contiguous ranges of coarse buckets from the
// prefix sums pre[0 .. kCoarse] of the global coarse histogram.  Cut q is the
// coarse boundary nearest q n / W, clamped so that every range holds at most
// cap = 2^18 >> cs coarse buckets (the second pass's local buckets) -- also
// the ranges still to come: cut[q] >= kCoarse - (W - q) cap.  Returns whether
// the plan is usable: every range within the cap and the largest within 1.5x
// of the mean (+ 65536); *mmax = the largest range's suffix count.
static bool plan_cuts(int W, uint64_t n, uint32_t cs, const uint64_t* pre, uint32_t* cut, uint64_t* mmax) {
    const uint64_t cap = (1ull << 18) >> cs;
    cut[0] = 0;
    cut[W] = kCoarse;
    for (int q = 1; q < W; ++q) {
        const uint64_t t = n * (uint64_t)q / W;
        uint32_t lo = cut[q - 1], hi = kCoarse;   // first i >= cut[q - 1] with pre[i] >= t
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (pre[mid] >= t) hi = mid;
            else lo = mid + 1;
        }
        // the boundary just before it when that one is nearer to t
        if (lo > cut[q - 1] && t - pre[lo - 1] < pre[lo] - t) --lo;
        const uint64_t hi_cap = (uint64_t)cut[q - 1] + cap;
        const uint64_t rest = (uint64_t)(W - q) * cap;
        const uint64_t lo_cap = rest >= kCoarse ? 0 : kCoarse - rest;
        uint64_t x = lo;
        if (x > hi_cap) x = hi_cap;
        if (x < lo_cap) x = lo_cap;
        if (x < cut[q - 1]) x = cut[q - 1];
        if (x > kCoarse) x = kCoarse;
        cut[q] = (uint32_t)x;
    }
    bool ok = true;
    uint64_t mx = 0;
    for (int q = 0; q < W; ++q) {
        mx = std::max(mx, pre[cut[q + 1]] - pre[cut[q]]);
        if ((uint64_t)(cut[q + 1] - cut[q]) > cap) ok = false;
    }
    *mmax = mx;
    return ok && mx <= (n / W) + (n / W) / 2 + 65536;
}

// h_coarse: the global coarse histogram (sum over ranks; NULL at world 1)
static int dist_cuts(sa_context* c, const uint64_t* h_coarse, sa_dist_info* info) {
    DistState* d = c->dist;
    if (!d || !d->planned) return set_err(SA_E_INVALID, "sa_dist_cuts before a successful sa_dist_begin");
    const int W = d->world;
    const uint64_t n = d->n;
    std::vector<uint64_t> pre(kCoarse + 1, 0);
    if (W == 1) {
        pre[kCoarse] = n;
        for (uint32_t i = 1; i < kCoarse; ++i) pre[i] = 0;   // never read: one range
    } else {
        if (!h_coarse) return set_err(SA_E_INVALID, "NULL coarse histogram");
        for (uint32_t i = 0; i < kCoarse; ++i) pre[i + 1] = pre[i] + h_coarse[i];
        if (pre[kCoarse] != n)
            return set_err(SA_E_INTERNAL, "coarse histogram sums to %llu, not n = %llu",
                           (unsigned long long)pre[kCoarse], (unsigned long long)n);
    }
    const uint32_t cs = dist_cshift(*d);
    d->cut.assign(W + 1, 0);
    uint64_t mmax = 0;
    const bool ok = plan_cuts(W, n, cs, pre.data(), d->cut.data(), &mmax);
    const int r = d->rank;
    d->blo = d->cut[r] << cs;
    d->bhi = d->cut[r + 1] << cs;
    d->m = pre[d->cut[r + 1]] - pre[d->cut[r]];
    d->sa_off = pre[d->cut[r]];
    info->m = d->m;
    info->sa_off = d->sa_off;
    info->m_max = mmax;
    info->bucket_lo = d->blo;
    info->bucket_hi = d->bhi;
    info->status = ok ? SA_DIST_OK : SA_DIST_UNBALANCED;
    if (!ok) return SA_OK;
    // owner of each coarse bucket
    std::vector<uint16_t> tab(kCoarse);
    for (int q = 0; q < W; ++q)
        for (uint32_t i = d->cut[q]; i < d->cut[q + 1]; ++i) tab[i] = (uint16_t)q;
    int rc = ensure_dist_n(c, n);
    if (rc) return rc;
    rc = ensure_dist_m(c, std::max<uint64_t>(d->m, 1));
    if (rc) return rc;
    SA_HIP(host_memcpy(d->owner_tab, tab.data(), kCoarse * 2, hipMemcpyHostToDevice));
    return SA_OK;
}

static int dist_round1(sa_context* c, const uint8_t* d_text, uint32_t* d_sa, hipStream_t s, sa_dist_info* info,
                       sa_stats* st) {
    DistState* d = c->dist;
    if (!d || !d->planned || d->cut.empty()) return set_err(SA_E_INVALID, "sa_dist_round1 before sa_dist_cuts");
    if (d->m && !d_sa) return set_err(SA_E_INVALID, "NULL SA slice");
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->n_kinds = SA_K_COUNT;
    }
    Timer tm{c, s, st != nullptr, st};
    c->radix = 0;
    SA_HIP(hipMemsetAsync(c->words, 0, 64, s));
    SA_HIP(hipMemsetAsync(d->cnt, 0, (2 * kDistMaxWorld + 8) * 4, s));
    d->mu = d->gu = 0;
    d->uo = 0;
    info->round1_ok = 1;
    info->heads = 0;
    if (d->m == 0) {   // an empty range (more ranks than coarse buckets with suffixes)
        info->unsorted = 0;
        info->groups = 0;
        return SA_OK;
    }
    BucketRange br;
    br.blo = d->blo;
    br.bhi = d->bhi;
    br.m = d->m;
    br.sa_off = d->sa_off;
    br.always_u = true;
    br.rank = d->crank;
    br.member = d->gmember;
    br.prefix = d->gprefix;
    br.tmp_rank = d->perm;   // free until the first request round
    bool done = false, fused = false;
    uint64_t seg[3] = {0, 0, 0};
    int rc = round1_bucketed(c, d_text, d->n, d_sa, d->bp, br, s, tm, st, &done, &fused, seg, &d->ksh);
    d->sa = d_sa;
    tm.flush();
    if (rc) return rc;
    if (!done || !fused) {
        info->round1_ok = 0;   // a window over the LDS tile: the caller falls back
        return SA_OK;
    }
    d->mu = seg[1];
    d->gu = seg[2];
    d->uo = 0;
    d->rounds = 1;
    info->heads = seg[0];
    info->unsorted = seg[1];
    info->groups = seg[2];
    return SA_OK;
}

static int dist_req_count(sa_context* c, uint64_t h, uint64_t* h_counts, hipStream_t s, sa_dist_info* info) {
    DistState* d = c->dist;
    if (!d || !d->planned) return set_err(SA_E_INVALID, "sa_dist_req_count before sa_dist_round1");
    const int W = d->world;
    d->send.assign(W, 0);
    d->nsend = 0;
    info->unsorted = d->mu;
    info->groups = d->gu;
    if (d->mu > 0 && W > 1) {
        SA_HIP(hipMemsetAsync(d->cnt, 0, W * 4, s));
        const uint32_t grid = (uint32_t)std::min<uint64_t>((d->mu + kBlock - 1) / kBlock, 8192);
        hipLaunchKernelGGL(k_dist_owner, dim3(grid), dim3(kBlock), 0, s, (const uint32_t*)c->u_idx[d->uo], d->mu, h,
                           d->text, d->n, (const uint16_t*)c->code, d->bp.bs, (const uint16_t*)d->owner_tab,
                           dist_cshift(*d), d->owner, d->cnt);
        SA_HIP(hipGetLastError());
        uint32_t* hc = c->host_words + 1024;   // pinned scratch (W <= kDistMaxWorld)
        SA_HIP(hipMemcpyAsync(hc, d->cnt, W * 4, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        for (int q = 0; q < W; ++q) {
            d->send[q] = hc[q];
            d->nsend += hc[q];
        }
    }
    for (int q = 0; q < W; ++q) h_counts[q] = d->send[q];
    return SA_OK;
}

// the owners' first request slots: exclusive prefix of the per-owner counts
// k_dist_owner left in cnt[0, W), into the fill cursors cnt[kDistMaxWorld ..]
// (on the device: no host round trip, no wait)
__global__ void k_dist_cursors(uint32_t* __restrict__ cnt, uint32_t W) {
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t q = 0; q < W; ++q) {
            cnt[kDistMaxWorld + q] = run;
            run += cnt[q];
        }
    }
}

static int dist_req_fill(sa_context* c, uint64_t h, uint32_t* d_req, hipStream_t s) {
    DistState* d = c->dist;
    if (!d) return set_err(SA_E_INVALID, "no distributed state");
    if (d->nsend == 0) return SA_OK;
    if (!d_req) return set_err(SA_E_INVALID, "NULL request buffer");
    hipLaunchKernelGGL(k_dist_cursors, dim3(1), dim3(64), 0, s, d->cnt, (uint32_t)d->world);
    const uint32_t grid = (uint32_t)std::min<uint64_t>((d->mu + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_dist_fill, dim3(grid), dim3(kBlock), 0, s, (const uint32_t*)c->u_idx[d->uo], d->mu, h,
                       (const uint32_t*)d->owner, d->cnt + kDistMaxWorld, d_req, d->perm);
    SA_HIP(hipGetLastError());
    return SA_OK;
}

static int dist_answer(sa_context* c, const uint32_t* d_req, uint64_t nreq, uint64_t* d_ans, hipStream_t s) {
    DistState* d = c->dist;
    if (!d) return set_err(SA_E_INVALID, "no distributed state");
    if (nreq == 0) return SA_OK;
    if (!d_req || !d_ans) return set_err(SA_E_INVALID, "NULL request / answer buffer");
    const uint32_t nbl = d->bhi - d->blo;
    const DistLookup L{d->crank, RankMap{d->gmember, d->gprefix}, c->keys[0], d->sa, d->ksh, c->segw + kBstartOff, d->text, (const uint16_t*)c->code,
                       d->n, d->bp.bs, d->blo, nbl, d->sa_off};
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nreq + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_dist_answer, dim3(grid), dim3(kBlock), 0, s, d_req, nreq, L, d_ans, d->cnt + 2 * kDistMaxWorld);
    SA_HIP(hipGetLastError());
    return SA_OK;
}

static int dist_refine(sa_context* c, uint64_t h, const uint64_t* d_ans, uint32_t* d_sa, hipStream_t s,
                       sa_dist_info* info) {
    DistState* d = c->dist;
    if (!d) return set_err(SA_E_INVALID, "no distributed state");
    info->heads = 0;
    // a request outside this rank's range (k_dist_answer) is a bug
    uint32_t* hc = c->host_words + 1024;
    SA_HIP(hipMemcpyAsync(hc, d->cnt + 2 * kDistMaxWorld, 4, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    if (hc[0]) return set_err(SA_E_INTERNAL, "rank request outside this rank's bucket range");
    if (d->mu == 0) {
        info->unsorted = 0;
        info->groups = 0;
        return SA_OK;
    }
    if (d->nsend && !d_ans) return set_err(SA_E_INVALID, "NULL answer buffer");
    if (h >= 2 * d->n) return set_err(SA_E_INTERNAL, "doubling did not converge (h=%llu)", (unsigned long long)h);
    Timer tm{c, s, false, nullptr};
    const uint64_t m = d->mu, G = d->gu;
    if (d->world == 1) {   // every look-up is local: no request / answer exchange
        const DistLookup L{d->crank, RankMap{d->gmember, d->gprefix}, c->keys[0], d->sa, d->ksh, c->segw + kBstartOff, d->text, (const uint16_t*)c->code,
                           d->n, d->bp.bs, d->blo, d->bhi - d->blo, d->sa_off};
        const uint32_t grid = (uint32_t)std::min<uint64_t>((m + kBlock - 1) / kBlock, 8192);
        hipLaunchKernelGGL(k_dist_r1_local, dim3(grid), dim3(kBlock), 0, s, (const uint32_t*)c->u_idx[d->uo], m, h, L,
                           d->r1, d->cnt + 2 * kDistMaxWorld);
        SA_HIP(hipGetLastError());
    } else {
        SA_HIP(hipMemsetAsync(d->r1, 0, m * 8, s));
    }
    if (d->world > 1 && d->nsend) {
        const uint32_t grid = (uint32_t)std::min<uint64_t>((d->nsend + kBlock - 1) / kBlock, 8192);
        hipLaunchKernelGGL(k_dist_place, dim3(grid), dim3(kBlock), 0, s, d_ans, d->nsend, (const uint32_t*)d->perm,
                           d->r1);
        SA_HIP(hipGetLastError());
    }
    const uint32_t wr = bit_width(d->n);   // rank values 0..n
    const uint32_t wg = G > 1 ? bit_width(G - 1) : 0;
    const uint32_t bits = wg + wr;
    if (bits > 64) return set_err(SA_E_INTERNAL, "key of %u bits", bits);
    const int ui = d->uo;
    const int uo = ui ^ 1;
    const SrcUArr src{c->u_idx[ui], c->u_g[ui], d->r1, wr};
    uint64_t* ukb0 = c->keys[1];   // keys[0] holds the round-1 keys (look-ups)
    uint64_t* ukb1 = c->keys_u;
    uint64_t* sorted = nullptr;
    uint32_t P = 0;
    if (G > 0 && m <= kUsAvg * G) {
        SA_HIP(hipMemsetAsync(c->words + kUsFlagWord, 0, 4, s));
        const uint32_t grid = (uint32_t)std::min<uint64_t>((m + kBlock - 1) / kBlock, 8192);
        hipLaunchKernelGGL(k_usort_small<SrcUArr>, dim3(grid), dim3(kBlock), 0, s, src, c->u_g[ui], m, ukb0,
                           c->vals_u, c->words + kUsFlagWord);
        SA_HIP(hipGetLastError());
        SA_HIP(hipMemcpyAsync(c->host_words + kUsFlagWord, c->words + kUsFlagWord, 4, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        if (c->host_words[kUsFlagWord] == 0) sorted = ukb0;
    }
    if (!sorted) {
        int rc = onesweep_prepare(c, s);
        if (rc) return rc;
        const uint32_t Pu = (bits + 7) / 8;
        const uint32_t grid = (uint32_t)std::min<uint64_t>((m + kBlock - 1) / kBlock, 2048);
        hipLaunchKernelGGL(k_materialize<SrcUArr>, dim3(grid), dim3(kBlock), 0, s, src, m, Pu, ukb1, os_ghist(c));
        SA_HIP(hipGetLastError());
        rc = radix_sort(c, SrcKeys{ukb1, c->u_idx[ui]}, 12 * m, plan_chunks(m), bits, c->vals_u, c->vals_alt, ukb0,
                        ukb1, s, tm, nullptr, &sorted, &P, true, true);
        if (rc) return rc;
    }
    uint64_t Du = 0, m2 = 0, G2 = 0;
    int rc = segments(c, sorted, c->vals_u, plan_chunks(m), PosArray{c->u_pos[ui]}, false, nullptr, d_sa, uo, s, tm,
                      nullptr, &Du, &m2, &G2, d->crank, d->sa_off, RankMap{d->gmember, d->gprefix});
    if (rc) return rc;
    if (d->world == 1) {   // the local look-ups' range check (segments() synchronised the stream)
        SA_HIP(host_memcpy(hc, d->cnt + 2 * kDistMaxWorld, 4, hipMemcpyDeviceToHost));
        if (hc[0]) return set_err(SA_E_INTERNAL, "rank look-up outside the bucket range");
    }
    d->mu = m2;
    d->gu = G2;
    d->uo = uo;
    d->rounds++;
    info->heads = Du;
    info->unsorted = m2;
    info->groups = G2;
    return SA_OK;
}
