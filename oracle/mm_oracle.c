/*
 * oracle/mm_oracle.c -- CPU restatement of the reference's Manber-Myers
 * suffix-array builder.  TEST INFRASTRUCTURE ONLY: this file is the checker
 * for tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
 * product path (hpc_suffix_array_amd/, libsa_hip.so) never links or calls it.
 *
 * What it restates (reference = /root/reference, snapshot 2025-10-17):
 *   - build_suffix_array          src/sequential/manber_myers.c:81-133
 *   - radix_sort_suffixes_seq     src/sequential/manber_myers.c:37-48
 *   - counting_sort_radix_seq     src/sequential/manber_myers.c:15-34
 *   - build_lcp_array (Kasai)     src/sequential/manber_myers.c:135-157
 *   - find_longest_repeated_substring  manber_myers.c:159-182
 *   - is_valid_suffix_array       src/sequential/manber_myers.c:184-202
 *
 * Deliberate, documented differences:
 *   - ranks are UNSIGNED bytes + 1 and the end-of-string sentinel is 0
 *     (reference: signed char, sentinel -1, get_rank_val adds 1 at :10-12).
 *     Inside the reference's valid domain (bytes 0x01..0x7F) the order, the
 *     number of rounds and every D_j are identical; outside it the reference
 *     is undefined (heap underflow at :20, 0xFF collides with the sentinel).
 *   - 64-bit loop bound and counters, so n = 2^30 works (reference :97
 *     overflows `2 * n` and returns the identity permutation).
 *   - records are {u32 index; u32 rank[2]}: the same 12-byte cost model as
 *     the reference's Suffix (suffix_array.h:11-14), valid for n <= 2^32.
 *
 * Parity pinning: the SA produced here is compared against the reference
 * compiled from its own sources (oracle/_ref/libmm.so, built by
 * oracle/Makefile) and against the SHA-256 known answers in
 * tests/golden/known_answers.json.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define ORACLE_API __attribute__((visibility("default")))

typedef struct {
    uint32_t index;
    uint32_t rank[2];
} oracle_rec;

/* ---------------------------------------------------------------------
 * Seeded input generator: splitmix64 finaliser applied to
 * seed + (i+1) * golden-gamma; symbol = alphabet[((z >> 32) * sigma) >> 32].
 * -------------------------------------------------------------------- */
static inline uint64_t splitmix_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

ORACLE_API void oracle_gen_text(uint8_t* out, uint64_t n, uint64_t seed,
                                const uint8_t* alphabet, uint32_t sigma) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t z = splitmix_at(seed, i);
        out[i] = alphabet[((z >> 32) * (uint64_t)sigma) >> 32];
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* Stable counting sort over one rank field: histogram, inclusive prefix,
 * backward scatter.  Restates counting_sort_radix_seq (manber_myers.c:15-34);
 * the bin of a record is its rank directly (ranks here are already >= 0,
 * the reference adds 1 at :10-12 to lift its -1 sentinel). */
static int counting_pass(const oracle_rec* in, oracle_rec* out, uint64_t n,
                         int field, uint64_t bins) {
    uint64_t* count = (uint64_t*)calloc(bins, sizeof(uint64_t));
    if (!count) return -1;
    for (uint64_t i = 0; i < n; i++) count[in[i].rank[field]]++;       /* :19-21 */
    for (uint64_t b = 1; b < bins; b++) count[b] += count[b - 1];      /* :23-25 */
    for (uint64_t i = n; i-- > 0;) out[--count[in[i].rank[field]]] = in[i]; /* :27-31 */
    free(count);
    return 0;
}

/* Reference-identical rank-doubling loop (manber_myers.c:81-133).
 * sa_out receives n u32 indices.  round_ms (optional, capacity max_rounds)
 * receives the wall time of every doubling round (sort + re-rank + update);
 * distinct (optional) receives D_j, the number of distinct ranks after each
 * round (= the reference's max_rank_value + 1 at :110).
 * Returns the number of rounds, or -1 on allocation failure. */
ORACLE_API int oracle_build_sa(const uint8_t* text, uint64_t n, uint32_t* sa_out,
                               double* round_ms, uint64_t* distinct, int max_rounds) {
    if (n == 0) return 0;
    oracle_rec* rec = (oracle_rec*)malloc(n * sizeof(oracle_rec));
    oracle_rec* tmp = (oracle_rec*)malloc(n * sizeof(oracle_rec));
    uint32_t* rank_of = (uint32_t*)malloc(n * sizeof(uint32_t));
    if (!rec || !tmp || !rank_of) { free(rec); free(tmp); free(rank_of); return -1; }

    /* init (:88-92): rank0 = byte, rank1 = next byte or sentinel */
    for (uint64_t i = 0; i < n; i++) {
        rec[i].index = (uint32_t)i;
        rec[i].rank[0] = (uint32_t)text[i] + 1u;
        rec[i].rank[1] = (i + 1 < n) ? (uint32_t)text[i + 1] + 1u : 0u;
    }
    uint64_t max_rank = 256;                       /* :94, shifted by +1 */
    int rounds = 0;
    for (uint64_t k = 2; k < 2 * n; k *= 2) {      /* :97 with a 64-bit bound */
        double t0 = now_s();
        /* radix_sort_suffixes_seq (:37-48): low field first, then high */
        if (counting_pass(rec, tmp, n, 1, max_rank + 2) ||
            counting_pass(tmp, rec, n, 0, max_rank + 2)) {
            free(rec); free(tmp); free(rank_of); return -1;
        }
        /* dense re-rank (:101-110); ranks start at 1 so 0 stays the sentinel */
        uint64_t cur = 1;
        rank_of[rec[0].index] = 1;
        for (uint64_t i = 1; i < n; i++) {
            if (rec[i].rank[0] != rec[i - 1].rank[0] || rec[i].rank[1] != rec[i - 1].rank[1])
                cur++;
            rank_of[rec[i].index] = (uint32_t)cur;
        }
        max_rank = cur;
        if (distinct && rounds < max_rounds) distinct[rounds] = cur;
        int done = (cur == n);                     /* :113 (max_rank_value == n-1) */
        if (!done) {
            /* update (:116-124): gather rank of i and of i+k */
            for (uint64_t i = 0; i < n; i++) {
                uint64_t idx = rec[i].index;
                rec[i].rank[0] = rank_of[idx];
                rec[i].rank[1] = (idx + k < n) ? rank_of[idx + k] : 0u;
            }
        }
        if (round_ms && rounds < max_rounds) round_ms[rounds] = 1e3 * (now_s() - t0);
        rounds++;
        if (done) break;
    }
    for (uint64_t i = 0; i < n; i++) sa_out[i] = rec[i].index;     /* :127-129 */
    free(rec); free(tmp); free(rank_of);
    return rounds;
}

/* Kasai LCP (manber_myers.c:135-157): lcp[r] = LCP(SA[r-1], SA[r]), lcp[0]=0. */
ORACLE_API int oracle_lcp(const uint8_t* text, uint64_t n, const uint32_t* sa, uint32_t* lcp) {
    if (n == 0) return 0;
    uint32_t* rank = (uint32_t*)malloc(n * sizeof(uint32_t));
    if (!rank) return -1;
    for (uint64_t r = 0; r < n; r++) rank[sa[r]] = (uint32_t)r;
    uint64_t h = 0;
    lcp[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (rank[i] > 0) {
            uint64_t j = sa[rank[i] - 1];
            while (i + h < n && j + h < n && text[i + h] == text[j + h]) h++;
            lcp[rank[i]] = (uint32_t)h;
            if (h > 0) h--;
        }   /* rank[i] == 0: h is carried as in the reference (it is 0 there) */
    }
    free(rank);
    return 0;
}

/* Longest repeated substring (manber_myers.c:159-182): first r with the
 * strictly largest lcp[r], r >= 1.  Returns its length, writes SA[r] to *pos
 * (or returns 0 when no repeat exists). */
ORACLE_API uint64_t oracle_lrs(uint64_t n, const uint32_t* sa, const uint32_t* lcp, uint64_t* pos) {
    uint64_t best = 0, at = 0;
    for (uint64_t r = 1; r < n; r++)
        if (lcp[r] > best) { best = lcp[r]; at = r; }
    if (pos) *pos = best ? sa[at] : 0;
    return best;
}

/* Reference validator semantics (manber_myers.c:184-202): permutation, then
 * adjacent suffixes non-decreasing under strcmp (unsigned, stops at NUL). */
ORACLE_API int oracle_is_valid_ref(const uint8_t* text, uint64_t n, const uint32_t* sa) {
    uint8_t* seen = (uint8_t*)calloc(n ? n : 1, 1);
    if (!seen) return 0;
    for (uint64_t r = 0; r < n; r++) {
        if (sa[r] >= n || seen[sa[r]]) { free(seen); return 0; }
        seen[sa[r]] = 1;
    }
    free(seen);
    for (uint64_t r = 1; r < n; r++) {
        const uint8_t* a = text + sa[r - 1];
        const uint8_t* b = text + sa[r];
        uint64_t la = n - sa[r - 1], lb = n - sa[r];
        uint64_t m = la < lb ? la : lb, q = 0;
        while (q < m && a[q] == b[q] && a[q] != 0) q++;
        int ca = q < la ? a[q] : 0, cb = q < lb ? b[q] : 0;
        if (ca > cb) return 0;
    }
    return 1;
}

/* O(n) suffix-array checker (Burkhardt-Kaerkkaeinen style):
 * SA is a permutation and for every adjacent pair (a, b):
 *   text[a] < text[b], or text[a] == text[b] and ISA[a+1] < ISA[b+1]
 * with ISA[n] = -1 (the empty suffix sorts first).  Unsigned bytes. */
ORACLE_API int oracle_check_sa(const uint8_t* text, uint64_t n, const uint32_t* sa) {
    if (n == 0) return 1;
    int64_t* isa = (int64_t*)malloc((n + 1) * sizeof(int64_t));
    if (!isa) return 0;
    for (uint64_t i = 0; i <= n; i++) isa[i] = -2;
    for (uint64_t r = 0; r < n; r++) {
        if (sa[r] >= n || isa[sa[r]] != -2) { free(isa); return 0; }
        isa[sa[r]] = (int64_t)r;
    }
    isa[n] = -1;
    int ok = 1;
    for (uint64_t r = 1; r < n && ok; r++) {
        uint64_t a = sa[r - 1], b = sa[r];
        if (text[a] > text[b]) ok = 0;
        else if (text[a] == text[b] && !(isa[a + 1] < isa[b + 1])) ok = 0;
    }
    free(isa);
    return ok;
}
