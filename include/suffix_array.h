/*
 * include/suffix_array.h -- drop-in C ABI of libsa_hip.so.
 *
 * Replaces the reference interface src/common/suffix_array.h:11-29
 * (a-rtemis99/hpc_suffix_array).  Same type layout and the same six symbols,
 * so a caller compiled against the reference header links against
 * libsa_hip.so unchanged.
 *
 *   SuffixArray layout (x86-64 SysV, 32 bytes): str@0  n@8  sa@16  lcp@24
 *   -- identical to suffix_array.h:16-21.
 *
 * Semantics honoured:
 *   create_suffix_array   manber_myers.c:51-69   private copy of the text with
 *                         strncpy semantics (bytes after the first NUL become
 *                         NUL), malloc'd sa/lcp; NULL on allocation failure.
 *   destroy_suffix_array  manber_myers.c:71-78
 *   build_suffix_array    manber_myers.c:81-133  synchronous; sa->sa is the
 *                         suffix array on return.  Built on the GPU (HIP,
 *                         gfx950).  Like the reference (assert at :85) it
 *                         aborts the process on failure, after printing the
 *                         reason to stderr -- there is no CPU fallback.
 *   build_lcp_array       manber_myers.c:135-157 lcp[0] = 0, lcp[r] =
 *                         LCP(SA[r-1], SA[r]).
 *   find_longest_repeated_substring  manber_myers.c:159-182  malloc'd string
 *                         the caller free()s; NULL when no substring repeats.
 *   is_valid_suffix_array manber_myers.c:184-202  1 if valid, else 0 (O(n)
 *                         GPU checker instead of the reference's O(n*LCP)).
 * Ordering: unsigned bytes, end of string smallest.  Inside the reference's
 * valid domain (1 <= n <= 2^30-1, bytes 0x01..0x7F) results are bit-exact
 * with the reference; outside it the reference is undefined
 * and this library returns the true suffix array.
 */
#ifndef SA_HIP_SUFFIX_ARRAY_H
#define SA_HIP_SUFFIX_ARRAY_H

#ifdef __cplusplus
extern "C" {
#endif

/* internal record of the reference (suffix_array.h:11-14); kept for source
 * compatibility, not used by this library */
typedef struct {
    int index;
    int rank[2];
} Suffix;

typedef struct {
    char* str;   /* private copy of the text, NUL-terminated */
    int n;       /* text length */
    int* sa;     /* suffix array, n entries */
    int* lcp;    /* LCP array, n entries */
} SuffixArray;

SuffixArray* create_suffix_array(const char* str, int n);
void destroy_suffix_array(SuffixArray* sa);
void build_suffix_array(SuffixArray* sa);
void build_lcp_array(SuffixArray* sa);
char* find_longest_repeated_substring(SuffixArray* sa);
int is_valid_suffix_array(SuffixArray* sa);

#ifdef __cplusplus
}
#endif

#endif /* SA_HIP_SUFFIX_ARRAY_H */
