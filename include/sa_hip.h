/*
 * include/sa_hip.h -- extended 64-bit C ABI of libsa_hip.so.
 *
 * The reference has no 64-bit or device-resident entry point; these replace
 * what its callers do around build_suffix_array (manber_myers.c:81-133):
 *   sa_build_ex      -- host text in, host SA out (create+build of
 *                       main_sequential.c:97-109 without the int n limit,
 *                       SURVEY.md 8(b) "What the replacement exports" (2))
 *   sa_build_device  -- text already resident in HBM, SA written to HBM
 *                       (what bench.py times)
 *   sa_check[_device]-- O(n) validity check replacing is_valid_suffix_array
 *                       (manber_myers.c:184-202), SURVEY.md 8(b) (3)
 * All functions return 0 on success or a negative SA_E* code; the text of
 * the last error of the calling thread is available from sa_last_error().
 * No torch types cross this boundary: plain pointers, sizes and a stream
 * handle (hipStream_t passed as void*, NULL = the null stream).
 */
#ifndef SA_HIP_H
#define SA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_OK 0
#define SA_E_INVALID (-1)   /* bad argument (NULL pointer, width, n too large) */
#define SA_E_NOMEM (-2)     /* device or host allocation failed */
#define SA_E_HIP (-3)       /* HIP runtime error (no device, launch failure) */
#define SA_E_INTERNAL (-4)  /* internal consistency check failed */

#define SA_MAX_ROUNDS 64

/* kernel kinds timed when sa_opts.profile != 0 */
enum sa_kernel_kind {
    SA_K_INIT = 0,           /* text -> rank_1 (reference schedule) */
    SA_K_HIST_FIRST = 1,     /* digit histogram, keys generated (text/ranks) */
    SA_K_HIST_KEYS = 2,      /* digit histogram over stored keys */
    SA_K_SCAN = 3,           /* digit x chunk offset scan */
    SA_K_SCATTER_FIRST = 4,  /* stable scatter, keys generated (text/ranks) */
    SA_K_SCATTER_KEYS = 5,   /* stable scatter over stored (key, idx) */
    SA_K_HEADS = 6,          /* group-head count per chunk (reference schedule) */
    SA_K_HEADS_SCAN = 7,     /* chunk scan of head counts, D_j */
    SA_K_RERANK = 8,         /* dense rank -> rank[idx] scatter */
    SA_K_SEG_COUNT = 9,      /* heads / unsorted / group counts per chunk */
    SA_K_SEG_SCAN = 10,      /* chunk scan of those counts */
    SA_K_SEG_WRITE = 11,     /* rank + SA update, unsorted-set compaction */
    SA_K_ALPHABET = 12,      /* byte histogram of the text */
    SA_K_PACK = 13,          /* packed K-symbol keys + first digit histogram */
    SA_K_SORT_U = 14,        /* every pass of an unsorted-set (later round) sort */
    SA_K_WINDOWS = 15,       /* bucketed round 1: window starts over the bucket-sorted keys */
    SA_K_LOCAL_SORT = 16,    /* bucketed round 1: per-window LDS sort */
    SA_K_PIVOT_KEYS = 17,    /* pivot round: keys (g, rank[i + h]) and group starts */
    SA_K_PIVOT_COUNT = 18,   /* pivot round: class counts (< = > pivot) per chunk, scanned */
    SA_K_PIVOT_WRITE = 19,   /* pivot round: tied blocks out, the rest compacted */
    SA_K_COUNT = 20
};

/* first round of the packed schedule */
#define SA_ROUND1_AUTO 0      /* bucketed when n >= 2^20 and it fits, else LSD */
#define SA_ROUND1_LSD 1       /* LSD radix sort of the packed K-symbol key */
#define SA_ROUND1_BUCKETED 2  /* two bucket passes + per-window LDS sort (falls
                                 back to LSD when a window exceeds the LDS tile) */
#define SA_ROUND1_PIVOT 3     /* sa_stats.round1 only: the LSD round's keys split
                                 around the key of suffix 0, half or more of the
                                 suffixes tied to it (sa_pivot.h) */

/* doubling schedules */
#define SA_SCHEDULE_PACKED 0     /* default: first round sorts a packed K-symbol
                                    prefix; later rounds re-sort only suffixes
                                    whose group is not yet a singleton */
#define SA_SCHEDULE_REFERENCE 1  /* the reference's schedule (manber_myers.c:
                                    94-125): h = 1, 2, 4, ...; D_0 = 256; every
                                    round sorts all n (rank[i], rank[i+h]) pairs */

/* sa_opts.debug: alternative code paths the tests and A/B runs force (0 in
 * production; the library reads no environment variable that changes a
 * build).  Every combination gives the same suffix array. */
#define SA_DEBUG_NO_CMP 0x1u            /* bucketed round 1: original key1 low, not the compact one */
#define SA_DEBUG_NO_PK8 0x2u            /* bucketed round 1: key1 + position, not packed 8-byte items */
#define SA_DEBUG_NO_PAD 0x4u            /* bucketed round 1: exact digit totals, not sampled padded segments */
#define SA_DEBUG_PAD_OVERFLOW 0x8u      /* forced overflow of the padded round-1 layouts, which then re-run exactly:
                                           one GPU: padded first-pass segments with no slack; range builds
                                           (sa_dist_round1): striped record regions of half their share, the
                                           round re-runs with the counting record scan */
#define SA_DEBUG_NO_FAST32 0x10u        /* local sort: measured-span kernel, not the fixed-span 32-bit one */
#define SA_DEBUG_NO_PIVOT 0x20u         /* later rounds: full sorts, never the three-way pivot split */
#define SA_DEBUG_PERM_ALWAYS 0x40u      /* reference schedule: permutation re-rank at every n */
#define SA_DEBUG_NO_XQ 0x80u            /* bucketed round 1: second pass into one region (one ticket), not per-XCD
                                           queues and regions */
#define SA_DEBUG_XQ_OVERFLOW 0x100u     /* per-XCD second pass with sub-regions of exactly 1/8 of each digit: a queue
                                           overflows and the round re-runs with the one-region pass */
#define SA_DEBUG_NO_KEY1_ROUND 0x400u   /* the first round after a sparse bucketed round 1 takes its keys' ranks by
                                           the sample search (RankLookup), not as key1 rebuilt from the text */
#define SA_DEBUG_NO_TIED 0x200u         /* pivot rounds: tied blocks through the sorted output and segments(), not
                                           written straight to the next unsorted set (sa_pivot.h) */
#define SA_DEBUG_NO_EONLY 0x800u        /* non-power-of-two alphabets: keep the compact key1 layout (and 12-byte
                                           first-pass items) instead of the E-only layout that packs them */
#define SA_DEBUG_EONLY 0x1000u          /* bucketed round 1: the E-only key1 layout whenever the text's tail allows
                                           it (tests; production takes it only for packed non-power-of-two items) */

typedef struct {
    int32_t profile;        /* 1: time every launch with HIP events */
    int32_t schedule;       /* SA_SCHEDULE_* */
    int32_t init_chars;     /* packed schedule: symbols in the first key, 0 = auto */
    int32_t radix;          /* 0: single-pass radix (decoupled look-back, default);
                               1: reduce-then-scan radix (3 kernels per pass) */
    int32_t round1;         /* SA_ROUND1_* (packed schedule, onesweep radix) */
    uint32_t debug;         /* SA_DEBUG_* flags (0 = production paths) */
    int32_t span_extra;     /* debug: bits added to the local sort's fixed key span
                               (its windows all take the measured-span retry) */
    int32_t tune;           /* A/B shapes, 0 = defaults: bits 0-7 the reference
                               schedule's widest LSD digit (8..10), bits 8-15 the
                               first bucket pass's cursor stripes (1, 2, 4, 8),
                               16-19 local-sort variants, 20-23 checker level-1
                               bins / persistent split, 24-27 = 1 the persistent
                               re-rank split, 28 no 32-bit rolling (12-byte
                               first-pass items), 29 window-order local-sort
                               rows (no chunk rows), 30 LCP by the random gather
                               (no permutations) */
} sa_opts;

typedef struct {
    int32_t rounds;                      /* doubling rounds executed */
    int32_t n_kinds;                     /* = SA_K_COUNT */
    double total_ms;                     /* build time on the stream (HBM in -> HBM out) */
    double h2d_ms, d2h_ms;               /* sa_build_ex only: PCIe copies */
    double round_ms[SA_MAX_ROUNDS];      /* per doubling round */
    uint64_t distinct[SA_MAX_ROUNDS];    /* D_j: distinct h-prefix groups after round j */
    int32_t passes[SA_MAX_ROUNDS];       /* radix passes in round j */
    uint64_t sorted_n[SA_MAX_ROUNDS];    /* suffixes (re-)sorted in round j */
    uint64_t prefix_len[SA_MAX_ROUNDS];  /* h after round j (prefix length sorted) */
    int32_t schedule;                    /* SA_SCHEDULE_* used */
    int32_t init_chars;                  /* K of the packed schedule */
    int32_t sigma;                       /* distinct symbols in the text */
    int32_t sparse_ranks;                /* 1: round-1 ranks kept for unsorted suffixes only */
    int32_t round1;                      /* SA_ROUND1_LSD, _BUCKETED or _PIVOT: first round taken */
    int32_t largest_window;              /* bucketed round 1: largest window (suffixes) */
    uint64_t model_bytes;                /* SURVEY.md 8(d)'s model of the REFERENCE-shaped schedule (12-B records
                                            through P_j LSD passes per round), summed; not the bytes of the
                                            packed schedule (round_bytes / kern_bytes are) */
    double kern_ms[SA_K_COUNT];          /* profile only */
    uint64_t kern_launches[SA_K_COUNT];  /* profile only */
    uint64_t kern_bytes[SA_K_COUNT];     /* algorithmic bytes moved per kind */
    int32_t round1_segments;             /* bucketed round 1: 0 exact digit totals, 1 sampled padded segments,
                                            2 padded segments overflowed and the round ran again exactly;
                                            range builds: 3 records by one striped text scan, 4 a record
                                            stripe overflowed and the round ran again with the counting scan */
    int32_t round1_layout;               /* bucketed round 1: bit 0 compact key1 low (BucketSpec.cmp),
                                            bit 1 packed 8-byte first-pass items (PK8), bit 2 the second
                                            pass by per-XCD queues and regions (XQ), bit 3 the E-only
                                            key1 low (no end bit; non-power-of-two alphabets' PK8) */
    uint64_t round_bytes[SA_MAX_ROUNDS]; /* algorithmic bytes of the kernels launched in round j (the kern_bytes
                                            added between its boundaries; the schedule actually run) */
} sa_stats;

typedef struct sa_context sa_context;

/* Device workspace for texts of up to max_n symbols on `device`. */
int sa_context_create(int device, uint64_t max_n, sa_context** out);
/* The debug / tune fields of opts (NULL: defaults) for the calls on ctx that
 * take no sa_opts -- the range-partitioned build's sa_dist_* phases;
 * sa_build_device applies its own opts. */
int sa_context_set_debug(sa_context* ctx, const sa_opts* opts);
void sa_context_destroy(sa_context* ctx);
/* bytes of device memory a context for max_n needs */
uint64_t sa_workspace_bytes(uint64_t max_n);

/* d_text: n bytes in device memory; d_sa: n uint32 in device memory.
 * n <= 2^32 - 1.  Enqueued on `stream`; returns after the SA is complete
 * (one 4-byte D_j read-back per round synchronises the stream). */
int sa_build_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, uint32_t* d_sa,
                    void* stream, const sa_opts* opts, sa_stats* stats);

/* Host in, host out.  sa_width is 4 (int32/uint32) or 8 (int64). */
int sa_build_ex(const uint8_t* text, uint64_t n, void* sa_out, int sa_width,
                const sa_opts* opts, sa_stats* stats);

/* O(n) check on the GPU: 1 valid, 0 invalid, <0 error. */
int sa_check_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa,
                    void* stream);
int sa_check(const uint8_t* text, uint64_t n, const void* sa, int sa_width);

/* LCP array and longest repeated substring on the GPU (replaces
 * build_lcp_array, manber_myers.c:135-157, and the lcp scan of
 * find_longest_repeated_substring, :159-182).  d_lcp[0] = 0 and
 * d_lcp[r] = lcp(SA[r-1], SA[r]) (n uint32 in device memory, may not alias
 * d_sa).  lrs_len / lrs_pos (optional) receive the first r >= 1 with the
 * strictly largest lcp: its length and SA[r] (0, 0 when nothing repeats).
 * Synchronises `stream` before returning. */
int sa_lcp_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, uint32_t* d_lcp,
                  uint64_t* lrs_len, uint64_t* lrs_pos, void* stream);
/* Host in, host out: sa and lcp_out have width sa_width (4 or 8). */
int sa_lcp(const uint8_t* text, uint64_t n, const void* sa, int sa_width, void* lcp_out, uint64_t* lrs_len,
           uint64_t* lrs_pos);

/* ---- building blocks of the range-partitioned multi-GPU build ----------
 * (hpc_suffix_array_amd/distributed.py drives these per rank; the exchange
 * steps between them are RCCL collectives over xGMI.)                      */

/* 256-bit byte-presence mask of the n device bytes (host out: 8 words). */
int sa_alphabet_device(const uint8_t* d_text, uint64_t n, uint32_t present_out[8], void* stream);

/* Packed K-symbol keys of positions [lo, hi) of the n-byte text:
 * key(i) = sum_t code[text[i+t]] * base^(K-1-t) (0 past the end);
 * code = 256 dense symbol codes (host array), base^K <= 2^64. */
int sa_pack_keys_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, uint64_t lo, uint64_t hi,
                        const uint16_t code[256], uint64_t base, uint32_t K, uint64_t* d_keys_out,
                        void* stream);

/* Stable LSD radix sort of m (u64 key, u32 value) pairs by key bits
 * [0, bits) into keys_out / vals_out (may not alias the inputs). */
int sa_sort_pairs_device(sa_context* ctx, const uint64_t* d_keys_in, const uint32_t* d_vals_in, uint64_t m,
                         uint32_t bits, uint64_t* d_keys_out, uint32_t* d_vals_out, void* stream);

/* dst[idx[i] - base] = src[i] for i < m (8-byte values, int64 indices):
 * the owner-side scatters of the exchange steps (new ranks, SA slices).
 * Indices outside [base, base + dst_n) are skipped and reported as
 * SA_E_INVALID; synchronous on `stream`. */
int sa_scatter_u64_device(uint64_t* d_dst, uint64_t dst_n, const int64_t* d_idx, int64_t base,
                          const uint64_t* d_src, uint64_t m, void* stream);

/* dst[i] = src[idx[i] - base] for i < m (8-byte values, int64 indices):
 * the permutations of the exchange steps.  Indices outside
 * [base, base + src_n) read 0 and are reported as SA_E_INVALID. */
int sa_gather_u64_device(uint64_t* d_dst, const uint64_t* d_src, uint64_t src_n, const int64_t* d_idx, int64_t base,
                         uint64_t m, void* stream);

/* In-place inclusive running max of m int64 values (the group-start
 * carries of the distributed re-rank); asynchronous on `stream`. */
int sa_running_max_i64_device(int64_t* d_v, uint64_t m, void* stream);
/* In-place inclusive prefix sum of m int64 values; asynchronous. */
int sa_inclusive_sum_i64_device(int64_t* d_v, uint64_t m, void* stream);
/* d_out[i] = the number of d_sorted[0 .. m) (non-decreasing) below d_q[i]
 * (at most d_q[i] when right != 0), for i < nq; asynchronous. */
int sa_count_below_u64_device(const uint64_t* d_sorted, uint64_t m, const uint64_t* d_q, uint64_t nq, int right,
                              int64_t* d_out, void* stream);
/* Positions (int64, in order) of the non-zero bytes of d_mask[0 .. m) into
 * d_out (capacity m; NULL: count only); *count = their number.
 * Synchronises `stream`. */
int sa_select_u8_device(const uint8_t* d_mask, uint64_t m, int64_t* d_out, uint64_t* count, void* stream);

/* ---- range-partitioned multi-GPU build, per rank ------------------------
 * Replaces src/mpi/manber_myers_mpi.c:22-160 (and main_mpi.c:43-54).  Every
 * rank holds the whole text in HBM; the SA is split into `world` contiguous
 * ranges of buckets (the first symbols of a suffix), rank q sorting the
 * suffixes of its range, which land at SA positions [sa_off, sa_off + m).
 * Sequence per build (the caller runs the collectives in brackets; see
 * hpc_suffix_array_amd/distributed.py):
 *   [all_reduce MAX of the 256-bit alphabet masks of the ranks' slices]
 *   sa_dist_begin   -> coarse bucket histogram of this rank's slice (d_coarse)
 *   [all_reduce SUM of d_coarse, copied to the host]
 *   sa_dist_cuts    -> m, sa_off (identical cuts on every rank)
 *   sa_dist_round1  -> the first round of the range into d_sa_local (m uint32)
 *   per round h = K, 2K, ... while any rank has unsorted suffixes:
 *     sa_dist_req_count -> requests per owner   [all_gather of counts]
 *     sa_dist_req_fill  -> requests by owner     [all_to_all]
 *     sa_dist_answer    -> ranks of the received requests   [all_to_all back]
 *     sa_dist_refine    -> sort / re-rank the unsorted set
 * status: SA_DIST_OK, or a reason the caller must build another way (all
 * ranks agree on it through a collective). */
#define SA_DIST_OK 0
#define SA_DIST_UNSUPPORTED 1   /* one symbol, or no bucketed key layout for this n */
#define SA_DIST_UNBALANCED 2    /* the bucket ranges cannot balance (skewed text) */

typedef struct {
    int32_t status;         /* SA_DIST_* */
    int32_t sigma;          /* distinct symbols */
    int32_t K;              /* symbols sorted by the first round */
    int32_t bucket_bits;    /* bucket = first symbols, bucket_bits wide */
    uint64_t m;             /* suffixes of this rank's range */
    uint64_t sa_off;        /* its first SA position */
    uint64_t m_max;         /* largest range over all ranks */
    uint32_t bucket_lo, bucket_hi;   /* this rank's buckets [lo, hi) */
    int32_t round1_ok;      /* 0: a window exceeded the LDS tile (fall back) */
    int32_t reserved;
    uint64_t heads;         /* groups completed in the last phase (local) */
    uint64_t unsorted;      /* this rank's unsorted suffixes after it */
    uint64_t groups;        /* their groups */
} sa_dist_info;

/* present: OR of all ranks' alphabet masks; d_coarse: 4096 uint64 (world > 1) */
int sa_dist_begin(sa_context* ctx, const uint8_t* d_text, uint64_t n, int world, int rank,
                  const uint32_t present[8], uint64_t* d_coarse, void* stream, sa_dist_info* info);
/* h_coarse: the all-reduced coarse histogram on the host (NULL at world 1) */
int sa_dist_cuts(sa_context* ctx, const uint64_t* h_coarse, sa_dist_info* info);
/* Frees the range-partitioned build's per-rank buffers of ctx (rank and
 * member arrays, request buffers); the context stays usable (a fallback
 * driver reuses its workspace).  Synchronises the device first. */
/* Allocate ahead of the first build everything a range build of up to
 * max_n symbols over `world` ranks needs (sa_dist_cuts would otherwise do it
 * inside the first build). */
int sa_dist_reserve(sa_context* ctx, uint64_t max_n, int world);
int sa_dist_release(sa_context* ctx);
/* The cut plan sa_dist_cuts applies (host only, no device): world + 1 cuts
 * into the 4096 coarse buckets of h_coarse (summing to n) at bucket width
 * bucket_bits; every range holds at most 2^18 buckets.  Returns SA_DIST_OK or
 * SA_DIST_UNBALANCED (largest range m_max above 1.5x the mean), < 0 on bad
 * arguments. */
int sa_dist_plan_cuts(int world, uint64_t n, int bucket_bits, const uint64_t* h_coarse, uint32_t* cuts_out,
                      uint64_t* m_max);
/* d_sa_local: info->m uint32 (global text positions, SA order) */
int sa_dist_round1(sa_context* ctx, uint32_t* d_sa_local, void* stream, sa_dist_info* info, sa_stats* stats);
/* counts_out: world uint64 -- requests this rank sends to each rank */
int sa_dist_req_count(sa_context* ctx, uint64_t h, uint64_t* counts_out, void* stream, sa_dist_info* info);
/* d_req: sum(counts_out) uint32, grouped by destination rank */
int sa_dist_req_fill(sa_context* ctx, uint64_t h, uint32_t* d_req, void* stream);
/* ranks of nreq received positions (all in this rank's range) -> d_ans (uint64) */
int sa_dist_answer(sa_context* ctx, const uint32_t* d_req, uint64_t nreq, uint64_t* d_ans, void* stream);
/* d_ans: the answers to this rank's requests, in request order */
int sa_dist_refine(sa_context* ctx, uint64_t h, const uint64_t* d_ans, uint32_t* d_sa_local, void* stream,
                   sa_dist_info* info);

/* Seeded synthetic text in device memory: the splitmix64 generator of
 * SURVEY.md 8(d) (symbol i = alphabet[((z >> 32) * sigma) >> 32]); the
 * stand-in for scripts/generate_large_datasets.py:12-28, seeded. */
int sa_generate_text_device(uint8_t* d_out, uint64_t n, uint64_t seed, const uint8_t* alphabet,
                            uint32_t sigma, void* stream);

const char* sa_last_error(void);
/* number of visible HIP devices (0 when none; never aborts) */
int sa_device_count(void);
/* library build identification, e.g. "sa_hip gfx950 <date>" */
const char* sa_version(void);
/* Host waits (stream synchronisations and blocking copies) the library has
 * made in this process so far; a driver differences it around a build. */
uint64_t sa_host_syncs(void);

/* sizeof(sa_stats) (which = 0) / sizeof(sa_opts) (which = 1), for bindings */
uint64_t sa_struct_size(int which);

#ifdef __cplusplus
}
#endif

#endif /* SA_HIP_H */
